#!/bin/bash
# scratch GPU session script (the command of the last gpurun call): fused residual + LayerNorm on single-stream
# launches -- bit-identity tests, then the pair step + L/14 leg A/B: A = default (fused on single-stream
# encodes: the L/14 leg), B = $CLM_FUSED_LN=0 (separate LayerNorm launches everywhere)
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_encode.py \
  -k "fused_resid_layernorm or pair_streams or text_varlen or last_layer_pruning or l14" > gpurun_out/r06x_tests.log 2>&1; rc=$?
tail -12 gpurun_out/r06x_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for arm in A B; do
    envs=""; [ $arm = B ] && envs="CLM_FUSED_LN=0"
    env $envs timeout -k 10 300 python bench.py --no-search --no-cpu-baseline --no-varlen --no-index-build --no-unmerged \
      --no-parity-mode --no-trace --no-single --no-encode-item --no-near-dup --no-persist > gpurun_out/ab/l$arm.$rep.json 2> gpurun_out/ab/l$arm.$rep.err
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/ab/l$arm.$rep.err; exit $rc; }
    python -c "import json; d=json.load(open('gpurun_out/ab/l$arm.$rep.json')); print('$arm', $rep, d['value'], d['ms_per_step'], d['l14']['images_per_s'], d['l14'].get('ms_per_step'))"
  done
done

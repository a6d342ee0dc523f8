#!/bin/bash
# scratch GPU session script (the command of the last gpurun call): fused residual + LayerNorm -- bit-identity
# tests, then the pair-step A/B: A = fused (default), B = separate LayerNorm launches, C = LayerNorms skipped
# (wrong embeddings, the upper bound of the LayerNorm launches' cost)
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_encode.py \
  -k "fused_resid_layernorm or pair_streams or text_varlen or last_layer_pruning" > gpurun_out/r06w_tests.log 2>&1; rc=$?
tail -15 gpurun_out/r06w_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=3 ARMS="A=cur B=cur:CLM_FUSED_LN=0 C=cur:CLM_FUSED_LN=0,CLM_SKIP_LN=1" \
  BENCH_ARGS="--no-trace --no-single --no-encode-item --no-near-dup --no-persist" bash tools/ab.sh

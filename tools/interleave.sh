#!/bin/bash
# interleaved tower launches (CLM_PAIR_INTERLEAVE=1): encode tests, pair-step A/B, kernel trace
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/il
CLM_PAIR_INTERLEAVE=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_encode.py tests/test_gpu_dropin.py > gpurun_out/il/tests.log 2>&1 || { tail -30 gpurun_out/il/tests.log; exit 1; }
tail -1 gpurun_out/il/tests.log
for rep in 1 2 3; do for m in 0 1; do
  CLM_PAIR_INTERLEAVE=$m timeout -k 10 200 python bench.py --no-search --no-cpu-baseline --no-l14 --no-varlen --no-index-build --no-unmerged --no-parity-mode --no-trace > gpurun_out/il/m$m.$rep.json 2> gpurun_out/il/m$m.$rep.err || { tail -5 gpurun_out/il/m$m.$rep.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/il/m$m.$rep.json')); print('interleave $m', $rep, d['value'], d['ms_per_step'], d['parity']['max_score_err'])"
done; done
CLM_PAIR_INTERLEAVE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/il/tr -o run -- python3 bench.py --steps 6 --warmup 2 --no-search --no-cpu-baseline --no-l14 --no-varlen --no-index-build --no-unmerged --no-parity-mode --no-trace > gpurun_out/il/tr.json 2> gpurun_out/il/tr.err

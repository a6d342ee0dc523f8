#!/bin/bash
# LayerNorm 4 rows per wave (CLM_LN_ROWS=4) vs 2: kernel probe, LN tests, pair step A/B
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/lnr
timeout -k 10 120 python -u tools/ln_bench.py > gpurun_out/lnr/r2.jsonl 2>&1 || exit 1
CLM_LN_ROWS=4 timeout -k 10 120 python -u tools/ln_bench.py > gpurun_out/lnr/r4.jsonl 2>&1 || exit 1
CLM_LN_ROWS=4 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_encode.py > gpurun_out/lnr/tests.log 2>&1 || { tail -20 gpurun_out/lnr/tests.log; exit 1; }
tail -1 gpurun_out/lnr/tests.log
for rep in 1 2 3; do for m in 2 4; do
  CLM_LN_ROWS=$m timeout -k 10 200 python bench.py --no-search --no-cpu-baseline --no-l14 --no-varlen --no-index-build --no-unmerged --no-parity-mode --no-trace > gpurun_out/lnr/m$m.$rep.json 2> gpurun_out/lnr/m$m.$rep.err || { tail -5 gpurun_out/lnr/m$m.$rep.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/lnr/m$m.$rep.json')); print('rows $m', $rep, d['value'], d['ms_per_step'], d['parity']['max_score_err'])"
done; done

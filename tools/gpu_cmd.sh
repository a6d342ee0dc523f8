#!/bin/bash
# scratch GPU session script (the command of the last gpurun call)
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_kernels.py tests/test_gpu_encode.py -x -v \
  --timeout 200 --timeout-method thread -k "small or group_maxima or all_paths or attention or timed or pair_streams" \
  > gpurun_out/r06a_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAIL|Error|assert|passed|failed" gpurun_out/r06a_pytest.log | tail -15; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-l14 --no-index-build --no-cpu-baseline --no-trace \
  --no-parity-mode --no-varlen --no-unmerged --no-near-dup --no-persist > gpurun_out/r06a_bench.json 2> gpurun_out/r06a_bench.err
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/r06a_bench.json; exit $rc

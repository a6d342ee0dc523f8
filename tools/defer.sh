#!/bin/bash
# G2 deferred epilogue: GEMM tests, exactness vs gemm_kernel tiles, fc1 timing, pair-step A/B old vs new lib
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_encode.py > gpurun_out/defer_tests.log 2>&1 || { tail -30 gpurun_out/defer_tests.log; exit 1; }
tail -2 gpurun_out/defer_tests.log
PROBE_TIME=0 timeout -k 10 120 python -u tools/pp_probe.py 5,9 odd,v_fc1,t_fc1 > gpurun_out/defer_exact.jsonl 2>&1 || exit 1
timeout -k 10 200 python -u tools/pp_probe.py 9 v_fc1,t_fc1 > gpurun_out/defer_time.jsonl 2>&1 || exit 1
CLM_LIB=ab/libclm_old.so timeout -k 10 200 python -u tools/pp_probe.py 9 v_fc1,t_fc1 > gpurun_out/defer_time_old.jsonl 2>&1 || exit 1
LIBS="old=ab/libclm_old.so new=ab/libclm_new.so" BENCH_ARGS="--no-l14 --no-varlen --no-index-build --no-unmerged --no-parity-mode --no-trace" timeout -k 10 600 bash tools/ab_bench.sh > gpurun_out/defer_ab.txt 2>&1

#!/bin/bash
# fused q/k/v + attention with G2's main-loop schedule: encode tests (bit identity), pair-step A/B
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_encode.py tests/test_gpu_dropin.py > gpurun_out/fa2_tests.log 2>&1 || { tail -30 gpurun_out/fa2_tests.log; exit 1; }
tail -1 gpurun_out/fa2_tests.log
LIBS="base=ab/libclm_base.so fa2=ab/libclm_fa2.so" BENCH_ARGS="--no-l14 --no-varlen --no-index-build --no-unmerged --no-parity-mode --no-trace --no-search" timeout -k 10 700 bash tools/ab_bench.sh > gpurun_out/fa2_ab.txt 2>&1
LIBS="base=ab/libclm_base.so fa2=ab/libclm_fa2.so" BENCH_ARGS="--no-l14 --no-varlen --no-index-build --no-unmerged --no-parity-mode --no-trace --no-search" timeout -k 10 700 bash tools/ab_bench.sh >> gpurun_out/fa2_ab.txt 2>&1

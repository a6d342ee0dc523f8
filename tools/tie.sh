#!/bin/bash
# text RESID tile 192x128 vs 128x192 (tie-break) in the pair step: alternating A/B
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_encode.py > gpurun_out/tie_tests.log 2>&1 || { tail -20 gpurun_out/tie_tests.log; exit 1; }
tail -1 gpurun_out/tie_tests.log
LIBS="base=ab/libclm_base.so tie=ab/libclm_tie.so" BENCH_ARGS="--no-l14 --no-varlen --no-index-build --no-unmerged --no-parity-mode --no-trace --no-search" timeout -k 10 700 bash tools/ab_bench.sh > gpurun_out/tie_ab.txt 2>&1
LIBS="base=ab/libclm_base.so tie=ab/libclm_tie.so" BENCH_ARGS="--no-l14 --no-varlen --no-index-build --no-unmerged --no-parity-mode --no-trace --no-search" timeout -k 10 700 bash tools/ab_bench.sh >> gpurun_out/tie_ab.txt 2>&1

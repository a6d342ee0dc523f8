#!/bin/bash
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_search.py > gpurun_out/nd_tests.log 2>&1 || { tail -20 gpurun_out/nd_tests.log; exit 1; }
timeout -k 10 600 python -u tools/neardup_ab.py default: cfg1:CLM_GEMM_CFG=1 > gpurun_out/neardup_ab2.txt 2>&1 && timeout -k 10 600 python -u tools/search_ab.py default: > gpurun_out/nd_search.txt 2>&1

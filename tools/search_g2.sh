#!/bin/bash
# filter GEMM on G2: search parity tests, then the configs[4] search A/B
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_search.py > gpurun_out/g2s_tests.log 2>&1 || { tail -30 gpurun_out/g2s_tests.log; exit 1; }
tail -2 gpurun_out/g2s_tests.log
timeout -k 10 600 python -u tools/search_ab.py default: all8:CLM_GEMM_CFG=8 old1:CLM_GEMM_CFG=1 noskip:CLM_FILTER_SKIP=0 > gpurun_out/g2s_search.txt 2>&1

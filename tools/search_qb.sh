#!/bin/bash
# configs[4] search vs the query block cap (CLM_SEARCH_QB), filter GEMM on G2 tiles
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_search.py > gpurun_out/qb_tests.log 2>&1 || { tail -20 gpurun_out/qb_tests.log; exit 1; }
timeout -k 10 900 python -u tools/search_ab.py default: q4096:CLM_SEARCH_QB=4096 q3072:CLM_SEARCH_QB=3072 default2: > gpurun_out/search_qb3.txt 2>&1

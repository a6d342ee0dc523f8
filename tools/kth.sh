#!/bin/bash
# streaming k-th thresholds: search parity tests, then the configs[4] search A/B against the radix path
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_search.py > gpurun_out/kth_tests.log 2>&1 || exit 1
timeout -k 10 500 python -u tools/search_ab.py default: radix:CLM_KTH_RADIX=1 noepi:CLM_GEMM_DEBUG=1 > gpurun_out/kth_search.txt 2>&1

#!/bin/bash
# FILTER row scales / thresholds staged in LDS (G2): search tests, then search A/B vs the previous lib
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_search.py > gpurun_out/fst_tests.log 2>&1 || { tail -30 gpurun_out/fst_tests.log; exit 1; }
tail -1 gpurun_out/fst_tests.log
timeout -k 10 900 python -u tools/search_ab.py new: base:CLM_LIB=ab/libclm_base.so new2: base2:CLM_LIB=ab/libclm_base.so noepi:CLM_GEMM_DEBUG=1 > gpurun_out/fst_search.txt 2>&1
timeout -k 10 600 python -u tools/neardup_ab.py new: base:CLM_LIB=ab/libclm_base.so > gpurun_out/fst_neardup.txt 2>&1

#!/bin/bash
# skip-test bounds decoded once per launch: search tests + A/B vs the previous lib
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_search.py > gpurun_out/cb_tests.log 2>&1 || { tail -30 gpurun_out/cb_tests.log; exit 1; }
tail -1 gpurun_out/cb_tests.log
timeout -k 10 900 python -u tools/search_ab.py new: base:CLM_LIB=ab/libclm_base.so new2: base2:CLM_LIB=ab/libclm_base.so > gpurun_out/cb_search.txt 2>&1

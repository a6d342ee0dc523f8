#!/bin/bash
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_search.py -k "many_query_blocks" > gpurun_out/blk_tests.log 2>&1; rc=$?; tail -5 gpurun_out/blk_tests.log; exit $rc

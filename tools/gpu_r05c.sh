#!/bin/bash
# round-5 session c: new search / distributed / host tests
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_kernels.py tests/test_gpu_distributed.py -x -v --timeout 300 --timeout-method thread -k "large_k or wide_dim or merge_past or filter_tile or host_check or sanitiz or index_build_1m or sharded_build or overflow or near_dup" > gpurun_out/r05c_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|Error|assert" gpurun_out/r05c_pytest.log | head -40; tail -3 gpurun_out/r05c_pytest.log; exit $rc

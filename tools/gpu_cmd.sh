#!/bin/bash
# scratch GPU session script (the command of the last gpurun call): G5 correctness + probe
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -k gemm > gpurun_out/r06h_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAIL|Error|assert|passed|failed" gpurun_out/r06h_pytest.log | tail -8; [ $rc -eq 0 ] || exit $rc
PROBE_VARIANTS="blas,full,noepi,nostore" timeout -k 10 600 python3 tools/gemm_probe.py 1,9,13,15 sq8k,l_qkv,l_fc1,l_out,l_fc2,v_fc1,t_fc1,v_fc2,t_fc2 > gpurun_out/r06h_probe.jsonl 2>gpurun_out/r06h_probe.err; rc=$?
echo "probe rc=$rc"; python3 -c "
import json
for l in open('gpurun_out/r06h_probe.jsonl'):
    d=json.loads(l)
    if 'variant' in d: print(d['shape'], d['variant'], d['us'], d['tflops'])
"; exit $rc

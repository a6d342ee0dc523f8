#!/bin/bash
# scratch GPU session script (the command of the last gpurun call): hipBLASLt-sized one-round tiles
# (160 x 256 = config 15, 256 x 160 = config 16, gemm_kernel with 4 waves) on the B/32 shapes
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
PROBE_VARIANTS="blas,full" timeout -k 10 600 python3 tools/gemm_probe.py 3,15,16,9 v_out,v_fc2,t_out,t_fc2,v_fc1,t_fc1 > gpurun_out/r06r_probe.jsonl 2>gpurun_out/r06r_probe.err; rc=$?
echo "probe rc=$rc"; python3 -c "
import json
for l in open('gpurun_out/r06r_probe.jsonl'):
    d=json.loads(l)
    if 'variant' in d: print(d['shape'], d['variant'], d['us'], d['tflops'])
"; exit $rc

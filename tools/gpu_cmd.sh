#!/bin/bash
# scratch GPU session script (the command of the last gpurun call): G4 one-tile-per-workgroup grids
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
PROBE_VARIANTS="blas,full,np" timeout -k 10 600 python3 tools/gemm_probe.py 1,3,9,13,14 l_qkv,l_fc1,l_out,l_fc2,v_fc1,t_fc1,v_fc2,v_out,t_fc2,t_out > gpurun_out/r06j_probe.jsonl 2>gpurun_out/r06j_probe.err; rc=$?
echo "probe rc=$rc"; python3 -c "
import json
for l in open('gpurun_out/r06j_probe.jsonl'):
    d=json.loads(l)
    if 'variant' in d: print(d['shape'], d['variant'], d['us'], d['tflops'])
"; exit $rc

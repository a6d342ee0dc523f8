#!/bin/bash
# scratch GPU session script (the command of the last gpurun call): G4 with a three-buffer ring (config 15) --
# the GEMM tests over every config, then the GEMM probe on the L/14 and B/32 shapes for configs 1 / 13 / 14 / 15
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "gemm" > gpurun_out/r06z_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r06z_tests.log; [ $rc -eq 0 ] || exit $rc
PROBE_VARIANTS=blas,full,noepi timeout -k 10 600 python -u tools/gemm_probe.py 1,3,9,13,14,15 l_qkv,l_fc1,l_fc2,v_qkv,v_fc1,t_fc1,v_fc2 > gpurun_out/r06z_probe.jsonl 2> gpurun_out/r06z_probe.err; rc=$?
[ $rc -eq 0 ] || { tail -5 gpurun_out/r06z_probe.err; exit $rc; }
python3 -c "
import json
rows=[json.loads(l) for l in open('gpurun_out/r06z_probe.jsonl')]
for r in rows: print(r['shape'], r['variant'], r['us'], r['tflops'])
"

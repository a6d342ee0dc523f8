#!/bin/bash
# scratch GPU session script (the command of the last gpurun call)
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
cp ab/libclm_B.so clip-lora-match_amd/libclm.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_encode.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t8.log 2>&1; rc=$?; tail -2 gpurun_out/t8.log; [ $rc -eq 0 ] || exit $rc
ARMS="A=A F=B" bash tools/ab_lib.sh || exit 1

#!/bin/bash
# round-4 GPU session: the GPU test suite + smoke, then the default bench line with its step trace
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
bash tools/gpu_cmd.sh || exit $?
CLM_TRACE_KEEP=gpurun_out/trace timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
echo "bench rc=$rc"; tail -c 400 gpurun_out/bench.json; exit $rc

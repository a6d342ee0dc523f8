#!/bin/bash
# the default bench line with its step trace
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
CLM_TRACE_KEEP=gpurun_out/trace timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
echo "bench rc=$rc"; tail -c 300 gpurun_out/bench.json; exit $rc

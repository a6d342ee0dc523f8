#!/bin/bash
# scratch GPU session script (the command of the last gpurun call): the default bench line at HEAD with
# its step trace kept, and a rocprofv3 --stats summary of the headline step
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
rm -rf gpurun_out/trace
CLM_TRACE_KEEP=gpurun_out/trace timeout -k 10 900 python -u bench.py > gpurun_out/r06p_bench.json 2> gpurun_out/r06p_bench.err; rc=$?
echo "bench rc=$rc"; tail -c 300 gpurun_out/r06p_bench.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/r06p_bench.err; exit $rc; }
ls gpurun_out/trace | head

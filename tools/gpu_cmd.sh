#!/bin/bash
# scratch GPU session script (the command of the last gpurun call)
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
DO_TEST=0 DO_PROF=1 bash tools/gpu_r03.sh || exit 1
DO_TEST=0 DO_BENCH=1 bash tools/gpu_r03.sh || exit 1

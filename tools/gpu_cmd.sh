#!/bin/bash
# scratch GPU session script (the command of the last gpurun call)
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
ARMS="A=A B=B" bash tools/ab_lib.sh

#!/bin/bash
# scratch GPU session script (the command of the last gpurun call): pair step with the text tower captured first
# (A = HEAD: vision first)
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
REPS=3 ARMS="A=cur B=cur:CLM_PAIR_TEXT_FIRST=1" BENCH_ARGS="--no-trace --no-single --no-encode-item --no-near-dup --no-persist" bash tools/ab.sh

#!/bin/bash
# scratch GPU session script (the command of the last gpurun call): the pair step with the single-stream RESID
# tile choice (160 x 128, config 7, one round of 2-workgroup slots) instead of the concurrent-tower one
# (128 x 192): A = HEAD, B = $CLM_GEMM_CONCURRENT=-1
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
REPS=4 ARMS="A=cur B=cur:CLM_GEMM_CONCURRENT=-1" BENCH_ARGS="--no-trace --no-single --no-encode-item --no-near-dup --no-persist" bash tools/ab.sh

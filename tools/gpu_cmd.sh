#!/bin/bash
# scratch GPU session script (the command of the last gpurun call): tower stream priorities A/B
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
ARMS="p0=cur:CLM_PAIR_PRIO=0 p1=cur:CLM_PAIR_PRIO=1 p2=cur:CLM_PAIR_PRIO=2 n0=cur:CLM_PAIR_PRIO=0|--no-graph n1=cur:CLM_PAIR_PRIO=1|--no-graph" REPS=2 BENCH_ARGS="--no-trace --no-encode-item" bash tools/ab.sh

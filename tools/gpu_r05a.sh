#!/bin/bash
# round-5 session a: grouped pair encode -- parity tests, then a same-session A/B
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_encode.py -x -v --timeout 120 --timeout-method thread -k "grouped or pair or fused or varlen or golden" > gpurun_out/r05a_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/r05a_pytest.log; [ $rc -eq 0 ] || exit $rc
REPS=2 BENCH_ARGS="--no-trace" ARMS="S=cur:CLM_PAIR_GROUPED=0 G=cur G0=cur:CLM_PAIR_CFG_RESID=0 G3=cur:CLM_PAIR_CFG_RESID=3 G9=cur:CLM_PAIR_CFG_GELU=9 GP=cur:CLM_PAIR_PERSIST=1" bash tools/ab.sh

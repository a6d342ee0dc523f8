#!/bin/bash
# scratch GPU session script (the command of the last gpurun call): persistent fused q/k/v + attention
# (next tile's first K-step and bias fetched under the attention): encode tests, then a same-session
# A/B of the pair step (A = HEAD, B = persistent)
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_dropin.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06q_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/r06q_pytest.log | tail -5; [ $rc -eq 0 ] || exit $rc
ARMS="A=A B=B" REPS=3 BENCH_ARGS="--no-trace --no-encode-item" bash tools/ab.sh

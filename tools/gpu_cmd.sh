#!/bin/bash
# scratch GPU session script (the command of the last gpurun call): full GPU suite + smoke at HEAD
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06s_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/r06s_pytest.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06s_smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 gpurun_out/r06s_smoke.log; exit $rc

#!/bin/bash
# scratch GPU session script (the command of the last gpurun call): the HEAD GPU suite -- every -m gpu test,
# smoke(), then the default bench line (with its rocprofv3 step trace)
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06y_gpu_tests.log 2>&1; rc=$?
tail -4 gpurun_out/r06y_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06y_smoke.log 2>&1; rc=$?
tail -2 gpurun_out/r06y_smoke.log; [ $rc -eq 0 ] || exit $rc
[ -n "$SKIP_BENCH" ] && exit 0
timeout -k 10 900 python -u bench.py > gpurun_out/r06y_bench.json 2> gpurun_out/r06y_bench.err; rc=$?
echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r06y_bench.err; exit $rc; }
python3 -c "
import json
d=json.loads(open('gpurun_out/r06y_bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['search']['qps'], d['search']['single']['ms_per_query'], d['search']['single']['device_hbm_frac'], d['l14']['images_per_s'], d['index_build']['images_per_s'])
"

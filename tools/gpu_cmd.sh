#!/bin/bash
# scratch GPU session script (the command of the last gpurun call): full GPU suite, smoke, full bench
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r06d_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/r06d_pytest.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06d_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/r06d_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py > gpurun_out/r06d_bench.json 2> gpurun_out/r06d_bench.err; rc=$?
echo "bench rc=$rc"; python3 -c "
import json; d=json.load(open('gpurun_out/r06d_bench.json'))
print('value', d['value'], 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'])
s=d.get('search',{}); print('search qps', s.get('qps'), s.get('check'), 'single', {k:s.get('single',{}).get(k) for k in ('ms_per_query','hbm_frac','device_ms_per_query','equal_to_exact_scan')})
print('encode_item', d.get('encode_item')); print('l14', {k:d.get('l14',{}).get(k) for k in ('images_per_s','gemm_tflops','attn_tflops')})
print('cpu', d.get('cpu_baseline',{}).get('value'))"
exit $rc

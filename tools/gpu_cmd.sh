#!/bin/bash
# scratch GPU session script (the command of the last gpurun call): small-batch graph tests, then the
# per-item encode leg with and without the graph (CLM_SMALL_GRAPH=0), alternating
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_image.py tests/test_gpu_dropin.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06o_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/r06o_pytest.log | tail -5; [ $rc -eq 0 ] || exit $rc
for arm in off1:0 on1:1 off2:0 on2:1; do
  name=${arm%%:*}; v=${arm#*:}
  CLM_SMALL_GRAPH=$v timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-l14 --no-parity-mode --no-varlen --no-index-build --no-unmerged --no-trace --no-search > gpurun_out/r06o_$name.json 2> gpurun_out/r06o_$name.err; rc=$?
  [ $rc -eq 0 ] || { tail -5 gpurun_out/r06o_$name.err; exit $rc; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/r06o_$name.json').read().strip().splitlines()[-1])
e=d['encode_item']; print('$name', {k: e.get(k) for k in ('encode_image_ms','encode_text_ms','gpu_encode_image_ms','gpu_encode_text_ms')}, d['value'])
"
done

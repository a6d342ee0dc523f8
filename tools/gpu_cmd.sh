#!/bin/bash
# scratch GPU session script (the command of the last gpurun call): search tests with the filter GEMM on
# G4 (config 13), then the configs[4] search leg, G2 (CLM_G4_FILTER=0) vs G4, alternating
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06n_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/r06n_pytest.log | tail -5; [ $rc -eq 0 ] || exit $rc
for arm in g2a:0 g4a:1 g2b:0 g4b:1; do
  name=${arm%%:*}; v=${arm#*:}
  CLM_G4_FILTER=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-l14 --no-parity-mode --no-varlen --no-index-build --no-unmerged --no-trace --no-persist --no-single --no-encode-item --steps 3 --warmup 1 > gpurun_out/r06n_$name.json 2> gpurun_out/r06n_$name.err; rc=$?
  [ $rc -eq 0 ] || { tail -5 gpurun_out/r06n_$name.err; exit $rc; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/r06n_$name.json').read().strip().splitlines()[-1])
s=d['search']; nd=d.get('search_near_dup',{})
print('$name', s['qps'], s['tflops'], s['check']['match'], s['paths'], nd.get('qps'), nd.get('equal_to_full_exact_scan'))
"
done

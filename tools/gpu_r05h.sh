#!/bin/bash
# round-5 session h: attn_long_dma_kernel parity + L/14 timing (+ attention PMC passes with PMC=1)
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_encode.py -k "attention or l14" -q -x --timeout 300 --timeout-method thread > gpurun_out/h_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/h_pytest.log; [ $rc -eq 0 ] || exit $rc
for mode in ${MODES:-2 3}; do
  CLM_ATTN_LONG=$mode timeout -k 10 300 python -u tools/l14_run.py 4 > gpurun_out/h_l14_$mode.json 2> gpurun_out/h_l14_$mode.err || { tail -5 gpurun_out/h_l14_$mode.err; exit 1; }
  echo "mode $mode: $(cat gpurun_out/h_l14_$mode.json)"
done
[ -n "$PMC" ] && { rm -rf gpurun_out/apmc; bash tools/attn_pmc.sh || exit 1; }
exit 0

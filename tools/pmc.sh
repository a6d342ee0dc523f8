#!/bin/bash
# PMC passes (one counter group per pass, never combined with tracing domains) over the
# GEMM sweep shapes and one bench step. Output CSVs under gpurun_out/pmc/.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d gpurun_out/pmc/p$i -o run -- python bench.py --steps 2 --warmup 1 --no-search --no-cpu-baseline --sequential > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pmc pass $i ($grp) rc=$rc"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/pmc/p$i.log; exit $rc; }
done

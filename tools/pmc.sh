#!/bin/bash
# PMC passes (one counter group per pass, never combined with tracing domains) over the
# sequential bench step, with CLM_GEMM_CONCURRENT=1 so every GEMM runs the tile config the timed
# two-stream step picks (128 x 192 RESID tiles, not the alone-on-the-chip 160 x 128).
# Output CSVs under gpurun_out/pmc/; summarise with
#   python tools/pmc_summary.py gpurun_out/pmc r<round>_v<version>
# Each pass stays within one pass's hardware budget (MI355X_MICROARCH.md: 8 SQ, 4 TCC with
# FETCH_SIZE = 3 and WRITE_SIZE = 2, 2 GRBM) and runs under its own time limit.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F16 GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  CLM_GEMM_CONCURRENT=1 timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d gpurun_out/pmc/p$i -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-search --no-cpu-baseline --no-l14 --no-parity-mode --no-varlen --no-index-build --no-unmerged --no-encode-item --sequential \
    > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pmc pass $i ($grp) rc=$rc"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/pmc/p$i.log; exit $rc; }
done

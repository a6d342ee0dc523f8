#!/bin/bash
# Stall breakdown of single encoder GEMMs: SQ wait/active cycles, MFMA busy, L2 hit/miss.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/stalls
i=0
for shape in "12800 3072 768 1 0" "12800 3072 768 1 8" "12800 768 3072 2 7" "4096 4096 4096 0 4"; do
  for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
             "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAIT_INST_LDS SQ_INSTS_LDS" \
             "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d gpurun_out/stalls/s$i -o run -- python tools/gemm_one.py $shape 20 > gpurun_out/stalls/s$i.log 2>&1
    rc=$?; echo "stall $i [$shape] [$grp] rc=$rc"
    [ $rc -eq 0 ] || { tail -5 gpurun_out/stalls/s$i.log; exit $rc; }
  done
done

#!/bin/bash
# LDS / issue / stall counters of single encoder GEMMs (tools/gemm_one.py), one rocprofv3 --pmc
# pass per counter group; the counter list of the box first.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/ldspmc
timeout -k 10 60 rocprofv3 -L > gpurun_out/ldspmc/counters.txt 2>&1
i=0
for shape in "12800 768 3072 2 3" "12800 3072 768 1 9" "12800 2304 768 0 1"; do
  for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
             "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VMEM SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d gpurun_out/ldspmc/s$i -o run -- python tools/gemm_one.py $shape 20 > gpurun_out/ldspmc/s$i.log 2>&1
    rc=$?; echo "pmc $i [$shape] rc=$rc"
    [ $rc -eq 0 ] || { tail -5 gpurun_out/ldspmc/s$i.log; exit $rc; }
  done
done

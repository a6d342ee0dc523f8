#!/bin/bash
# PMC passes over the configs[3] leg (tools/l14_run.py) for attn_long_kernel: wave-cycle split
# (active / waiting / issue-stalled), MFMA busy, LDS instructions and bank conflicts, VALU share.
# One counter group per pass (8 SQ + 2 GRBM at most), no tracing domains besides --kernel-trace,
# each pass under its own limit. Summarise with  python tools/attn_pmc_summary.py gpurun_out/apmc
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/apmc
timeout -s KILL 60 rocprofv3 -L > gpurun_out/apmc/counters.txt 2>&1 || true
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d gpurun_out/apmc/p$i -o run -- \
    python3 tools/l14_run.py 1 ${L14_DTYPE:-mixed} > gpurun_out/apmc/p$i.log 2>&1
  rc=$?; echo "attn pmc pass $i ($grp) rc=$rc"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/apmc/p$i.log; exit $rc; }
done

#!/bin/bash
# PMC of the configs[4] search leg (filter GEMM on G2 tiles): L2 hit rate, fetch, MFMA busy; one counter group per pass
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/spmc
i=0
for grp in "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" "FETCH_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d gpurun_out/spmc/p$i -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-l14 --no-parity-mode --no-varlen --no-index-build \
    --no-unmerged --no-trace --no-persist --no-near-dup > gpurun_out/spmc/p$i.log 2>&1 || exit 1
  echo "pass $i ok"
done

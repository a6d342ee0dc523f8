#!/bin/bash
# In-pipeline GEMM config sweep: force each tile config (CLM_GEMM_CFG) for every GEMM of the
# sequential encode and trace per-shape durations. CFGS="4 15 ..."
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/tc
for cfg in $CFGS; do
  CLM_GEMM_CFG=$cfg timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tc/c$cfg -o run -- python bench.py --sequential --no-search --no-cpu-baseline --steps 6 --warmup 2 > gpurun_out/tc/c$cfg.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/tc/c$cfg.log; exit $rc; }
  python tools/trace_gemm_shapes.py $(find gpurun_out/tc/c$cfg -name "*kernel_trace.csv" | head -1) c$cfg | tail -1
done

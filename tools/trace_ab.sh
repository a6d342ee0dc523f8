#!/bin/bash
# Kernel traces of the sequential encode pipeline per libclm build: LIBS="name=path ..."
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/tr
for spec in $LIBS; do
  name=${spec%%=*}; path=${spec#*=}
  CLM_LIB=$path timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr/$name -o run -- python bench.py --sequential --no-search --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/tr/$name.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/tr/$name.log; exit $rc; }
  python tools/trace_gemm_shapes.py $(find gpurun_out/tr/$name -name "*kernel_trace.csv" | head -1) $name
done

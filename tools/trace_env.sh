#!/bin/bash
# Per-shape GEMM durations in the sequential encode pipeline per environment setting:
# ENVS="name:VAR=val,VAR2=val ..."
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/te
for spec in $ENVS; do
  name=${spec%%:*}; vars=${spec#*:}
  for kv in $(echo "$vars" | tr ',' ' '); do export "$kv"; done
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/te/$name -o run -- python bench.py --sequential --no-search --no-cpu-baseline --steps 6 --warmup 2 > gpurun_out/te/$name.log 2>&1
  rc=$?
  for kv in $(echo "$vars" | tr ',' ' '); do unset "${kv%%=*}"; done
  [ $rc -eq 0 ] || { tail -5 gpurun_out/te/$name.log; exit $rc; }
  python tools/trace_gemm_shapes.py $(find gpurun_out/te/$name -name "*kernel_trace.csv" | head -1) $name | tail -1
done

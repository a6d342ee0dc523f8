#!/bin/bash
# round-5 session b: kernel traces of the pair step, two-stream vs grouped
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/tl
for spec in S:CLM_PAIR_GROUPED=0 G:CLM_PAIR_GROUPED=1; do
  name=${spec%%:*}; kv=${spec#*:}
  export "$kv"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl/$name -o run -- python bench.py --no-search --no-cpu-baseline --no-l14 --no-varlen --no-index-build --no-unmerged --no-parity-mode --no-trace --steps 10 --warmup 2 > gpurun_out/tl/$name.log 2>&1 || { tail -5 gpurun_out/tl/$name.log; exit 1; }
  echo "== $name"; python tools/timeline.py $(find gpurun_out/tl/$name -name "*kernel_trace.csv" | head -1) 5 | head -30
done

#!/bin/bash
# kernel traces of the headline pair step per variant: SPECS="name:VAR=val,...|bench args" (args after |)
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/tl
IFS=';' read -ra ARR <<< "$SPECS"
for spec in "${ARR[@]}"; do
  name=${spec%%:*}; rest=${spec#*:}; envs=${rest%%|*}; args=""
  [ "$rest" != "$envs" ] && args=${rest#*|}
  rm -rf gpurun_out/tl/$name
  env $(echo "$envs" | tr ',' ' ') timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl/$name -o run -- python bench.py --no-search --no-cpu-baseline --no-l14 --no-varlen --no-index-build --no-unmerged --no-parity-mode --no-trace --steps 10 --warmup 2 $args > gpurun_out/tl/$name.log 2>&1 || { tail -5 gpurun_out/tl/$name.log; exit 1; }
  echo "== $name"; python tools/timeline.py $(find gpurun_out/tl/$name -name "*kernel_trace.csv" | head -1) 5 | head -${LINES_OUT:-24}
done

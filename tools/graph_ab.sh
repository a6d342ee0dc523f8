#!/bin/bash
# pair step with vs without the hipGraph replay (two tower streams either way), + a kernel trace of the no-graph step
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/gab
for rep in 1 2; do for m in graph nograph; do
  extra=""; [ $m = nograph ] && extra="--no-graph"
  timeout -k 10 200 python bench.py $extra --no-search --no-cpu-baseline --no-l14 --no-varlen --no-index-build --no-unmerged --no-parity-mode --no-trace > gpurun_out/gab/$m.$rep.json 2> gpurun_out/gab/$m.$rep.err || { tail -5 gpurun_out/gab/$m.$rep.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/gab/$m.$rep.json')); print('$m', $rep, d['value'], d['ms_per_step'])"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gab/tr -o run -- python3 bench.py --no-graph --steps 6 --warmup 2 --no-search --no-cpu-baseline --no-l14 --no-varlen --no-index-build --no-unmerged --no-parity-mode --no-trace > gpurun_out/gab/tr.json 2> gpurun_out/gab/tr.err

#!/bin/bash
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/split
for rep in 1 2; do for sp in 1 2; do
  timeout -k 10 200 python bench.py --split $sp --no-search --no-cpu-baseline --no-l14 --no-varlen --no-index-build --no-unmerged --no-parity-mode --no-trace > gpurun_out/split/s$sp.$rep.json 2> gpurun_out/split/s$sp.$rep.err || { tail -5 gpurun_out/split/s$sp.$rep.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/split/s$sp.$rep.json')); print('split $sp', $rep, d['value'], d['ms_per_step'])"
done; done

#!/bin/bash
# kernel stats of the search leg (configs[4])
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/sprof2
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sprof2 -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-l14 --no-parity-mode --no-varlen --no-index-build \
  --no-unmerged --no-trace --no-persist --no-near-dup > gpurun_out/sprof2/s.json 2> gpurun_out/sprof2/s.err

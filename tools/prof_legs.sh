#!/bin/bash
# kernel stats of the search (configs[4]) and L/14 (configs[3]) legs
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/prof_legs
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_legs/s -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-l14 --no-parity-mode --no-varlen --no-index-build \
  --no-unmerged --no-trace --no-persist > gpurun_out/prof_legs/s.json 2> gpurun_out/prof_legs/s.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_legs/l -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-search --no-parity-mode --no-varlen --no-index-build \
  --no-unmerged --no-trace > gpurun_out/prof_legs/l.json 2> gpurun_out/prof_legs/l.err

#!/bin/bash
# scratch GPU session script (the command of the last gpurun call)
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/split
timeout -k 10 400 python -u -m pytest tests/test_gpu_encode.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t2.log 2>&1; rc=$?; tail -2 gpurun_out/t2.log; [ $rc -eq 0 ] || exit $rc
ARMS="A=A B=B" BENCH_ARGS="--sequential" bash tools/ab_lib.sh || exit 1
cp ab/libclm_A.so clip-lora-match_amd/libclm.so
for sp in 2 3; do
  timeout -k 10 200 python bench.py --no-search --no-cpu-baseline --no-l14 --no-varlen --no-index-build --no-unmerged --no-parity-mode --split $sp > gpurun_out/split/s$sp.json 2> gpurun_out/split/s$sp.err || { tail -3 gpurun_out/split/s$sp.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/split/s$sp.json')); print('A split $sp', d['value'], d['ms_per_step'])"
done
ARMS="A=A B=B" bash tools/ab_lib.sh

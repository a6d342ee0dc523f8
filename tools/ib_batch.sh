#!/bin/bash
# configs[2] index build vs encode batch size
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/ib
for b in 1280 1536 2048 2560 512; do
  timeout -k 10 240 python bench.py --index-batch $b --steps 3 --warmup 1 --no-search --no-cpu-baseline --no-l14 --no-varlen --no-unmerged --no-parity-mode --no-trace > gpurun_out/ib/b$b.json 2> gpurun_out/ib/b$b.err || { tail -5 gpurun_out/ib/b$b.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ib/b$b.json'))['index_build']; print('batch $b', d['images_per_s'], d['encode_images_per_s'], d['index_fold_sha256'])"
done

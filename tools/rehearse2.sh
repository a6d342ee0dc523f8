#!/bin/bash
# world-2 rehearsal of bench.py on one GPU (gloo): every N>1 leg (sharded index build with the fp16
# exchange, row-sharded search + top-k merge, pair step with the embedding all_gather)
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/reh
CLM_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 5 --warmup 2 --search-rows 2000000 --search-queries 4096 --index-images 131072 --no-cpu-baseline > gpurun_out/reh/w2.json 2> gpurun_out/reh/w2.err
rc=$?; tail -c 1500 gpurun_out/reh/w2.json; exit $rc

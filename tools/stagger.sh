#!/bin/bash
# stagger A/B: odd workgroups of gemm_kernel start n x s_sleep(127) late (debug 64 | n << 8)
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
PROBE_DBG=576,1088,1600,2112 timeout -k 10 400 python -u tools/pp_probe.py 1 l_qkv,l_fc1,sq8k > gpurun_out/stagger.jsonl 2>&1

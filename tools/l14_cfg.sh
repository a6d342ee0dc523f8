#!/bin/bash
# L/14 qkv / fc1 / out / fc2 GEMMs: gemm_kernel 256x256 (1) vs G2 tiles (8, 9, 10)
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 400 python -u tools/pp_probe.py 1,8,9,10 l_qkv,l_fc1 > gpurun_out/l14_cfg.jsonl 2>&1

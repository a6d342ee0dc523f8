#!/bin/bash
# W32 (32x32x16 MFMA) GEMM probe: exactness on integer data, then timing vs the picked configs
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
PROBE_INT=1 PROBE_TIME=0 timeout -k 10 120 python -u tools/pp_probe.py 12,13,14,15,16 odd,v_fc1,t_fc1,v_fc2,t_fc2,v_out,t_out,v_qkv > gpurun_out/w32_int.jsonl 2>&1 || exit 1
timeout -k 10 300 python -u tools/pp_probe.py 12,13,14,15,16 v_fc1,t_fc1,v_fc2,t_fc2,v_out,t_out,v_qkv,t_qkv > gpurun_out/w32_time.jsonl 2>&1 || exit 1
timeout -k 10 120 python -u tools/bf16_bisect.py > gpurun_out/bf16_bisect.jsonl 2>&1

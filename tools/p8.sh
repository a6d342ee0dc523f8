#!/bin/bash
# P8 (256 x 256 phase-staggered) GEMM: exactness on integer data, timing vs the picked configs, search leg
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
PROBE_INT=1 PROBE_TIME=0 timeout -k 10 120 python -u tools/pp_probe.py 12,1 odd,v_qkv,v_fc1,v_fc2,t_fc1,l_fc2 > gpurun_out/p8_int.jsonl 2>&1 || exit 1
timeout -k 10 300 python -u tools/pp_probe.py 12,1 v_qkv,v_fc1,t_fc1,l_qkv,l_fc1,l_fc2,sq8k > gpurun_out/p8_time.jsonl 2>&1 || exit 1
timeout -k 10 500 python -u tools/search_ab.py default: p8:CLM_GEMM_CFG=12 noepi:CLM_GEMM_DEBUG=1 p8noepi:CLM_GEMM_CFG=12,CLM_GEMM_DEBUG=1 > gpurun_out/p8_search.txt 2>&1

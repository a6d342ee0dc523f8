#!/bin/bash
# configs[4] search vs the threshold sample size (S = k N / CLM_SAMPLE_DIV)
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 600 python -u tools/search_ab.py default: d128:CLM_SAMPLE_DIV=128 d512:CLM_SAMPLE_DIV=512 d1024:CLM_SAMPLE_DIV=1024 d64:CLM_SAMPLE_DIV=64 > gpurun_out/search_sdiv.txt 2>&1

#!/bin/bash
# configs[4] search with the filter / sample GEMM tile forced (CLM_GEMM_CFG)
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 900 python -u tools/search_ab.py default: c8:CLM_GEMM_CFG=8 c9:CLM_GEMM_CFG=9 c10:CLM_GEMM_CFG=10 c11:CLM_GEMM_CFG=11 c5:CLM_GEMM_CFG=5 c6:CLM_GEMM_CFG=6 > gpurun_out/search_cfg.txt 2>&1

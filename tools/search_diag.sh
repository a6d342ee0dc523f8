#!/bin/bash
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 600 python -u tools/search_ab.py default: noepi:CLM_GEMM_DEBUG=1 boundonly:CLM_GEMM_DEBUG=2 noskip:CLM_FILTER_SKIP=0 > gpurun_out/search_diag.txt 2>&1

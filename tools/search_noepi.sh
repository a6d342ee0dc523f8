#!/bin/bash
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 600 python -u tools/search_ab.py default: noepi:CLM_GEMM_DEBUG=1 nostore:CLM_GEMM_DEBUG=2 default2: > gpurun_out/search_noepi.txt 2>&1

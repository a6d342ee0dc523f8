#!/bin/bash
# L/14 RESID GEMMs (out_proj, fc2; M = 73,856, N = 1024): tile configs vs the picked one
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
PROBE_INT=0 timeout -k 10 500 python -u tools/pp_probe.py 1,3,4,5,7,8,10 l_fc2,l_out > gpurun_out/l14_resid.jsonl 2>&1

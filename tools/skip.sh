#!/bin/bash
# FILTER skip test (GemmArgs::cbound): search parity tests, then the configs[4] search A/B
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_search.py > gpurun_out/skip_tests.log 2>&1 || exit 1
timeout -k 10 500 python -u tools/search_ab.py default: noskip:CLM_FILTER_SKIP=0 noepi:CLM_GEMM_DEBUG=1 > gpurun_out/skip_search.txt 2>&1
export TMPDIR=/tmp && mkdir -p gpurun_out/sprof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sprof -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-l14 --no-parity-mode --no-varlen --no-index-build \
  --no-unmerged --no-trace --no-persist --no-near-dup > gpurun_out/sprof/s.json 2> gpurun_out/sprof/s.err

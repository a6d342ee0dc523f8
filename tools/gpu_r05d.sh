#!/bin/bash
# round-5 session d: unmerged LoRA through the MFMA down-projection -- parity, then A/B merged vs unmerged
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_dropin.py -x -v --timeout 200 --timeout-method thread -k "unmerged or varlen or tiny or golden or pruning" > gpurun_out/r05d_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAIL|Error|assert" gpurun_out/r05d_pytest.log | head -20; tail -3 gpurun_out/r05d_pytest.log; [ $rc -eq 0 ] || exit $rc
REPS=2 BENCH_ARGS="--no-trace" ARMS="M=cur U=cur|--lora-mode=unmerged" bash tools/ab.sh

#!/bin/bash
# round-5 session g: fused attention with 16-row-aligned sequence staging -- parity, PMC LDS conflicts, A/B
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_encode.py -x -v --timeout 200 --timeout-method thread -k "fused or varlen or golden or grouped or pair" > gpurun_out/r05g_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAIL|Error|assert" gpurun_out/r05g_pytest.log | head -20; tail -3 gpurun_out/r05g_pytest.log; [ $rc -eq 0 ] || exit $rc
for lib in old new; do
  cp ab/libclm_$lib.so clip-lora-match_amd/libclm.so
  CLM_GEMM_CONCURRENT=1 timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcfa/$lib -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-search --no-cpu-baseline --no-l14 --no-parity-mode --no-varlen --no-index-build --no-unmerged --sequential --no-trace > gpurun_out/pmcfa_$lib.log 2>&1 || { tail -5 gpurun_out/pmcfa_$lib.log; cp ab/libclm_new.so clip-lora-match_amd/libclm.so; exit 1; }
done
cp ab/libclm_new.so clip-lora-match_amd/libclm.so
REPS=3 BENCH_ARGS="--no-trace" ARMS="old=old new=new" bash tools/ab.sh

#!/bin/bash
# A/B of two prebuilt libraries (ab/libclm_A.so, ab/libclm_B.so, with ab/_capi_{A,B}.py if present) on the bench, alternating in one
# session; the library in place at the end is B. ENV: extra environment for both arms.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/abl
for rep in 1 2 3; do
  for v in A B; do
    cp ab/libclm_$v.so clip-lora-match_amd/libclm.so
    [ -f ab/_capi_$v.py ] && cp ab/_capi_$v.py clip-lora-match_amd/_capi.py
    env ${ENV:-} timeout -k 10 300 python bench.py --no-search --no-cpu-baseline --no-l14 --no-varlen --no-index-build --no-unmerged --no-parity-mode ${BENCH_ARGS:-} > gpurun_out/abl/$v.$rep.json 2> gpurun_out/abl/$v.$rep.err
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/abl/$v.$rep.err; cp ab/libclm_B.so clip-lora-match_amd/libclm.so; [ -f ab/_capi_B.py ] && cp ab/_capi_B.py clip-lora-match_amd/_capi.py; exit $rc; }
    python -c "import json; d=json.load(open('gpurun_out/abl/$v.$rep.json')); print('$v', $rep, d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_step'])"
  done
done
cp ab/libclm_B.so clip-lora-match_amd/libclm.so
[ -f ab/_capi_B.py ] && cp ab/_capi_B.py clip-lora-match_amd/_capi.py
true

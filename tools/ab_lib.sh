#!/bin/bash
# A/B of prebuilt libraries on the bench, alternating in one session. ARMS = space-separated
# "name=lib[:VAR=val,VAR=val]" (lib X = ab/libclm_X.so with ab/_capi_X.py if present); default
# "A=A B=B". The library in place at the end is B.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/abl
restore() { cp ab/libclm_B.so clip-lora-match_amd/libclm.so; [ -f ab/_capi_B.py ] && cp ab/_capi_B.py clip-lora-match_amd/_capi.py; true; }
for rep in 1 2 3; do
  for arm in ${ARMS:-A=A B=B}; do
    name=${arm%%=*}; rest=${arm#*=}; lib=${rest%%:*}; envs=""
    [ "$rest" != "$lib" ] && envs=$(echo "${rest#*:}" | tr ',' ' ')
    cp ab/libclm_$lib.so clip-lora-match_amd/libclm.so
    [ -f ab/_capi_$lib.py ] && cp ab/_capi_$lib.py clip-lora-match_amd/_capi.py
    env $envs timeout -k 10 300 python bench.py --no-search --no-cpu-baseline --no-l14 --no-varlen --no-index-build --no-unmerged --no-parity-mode ${BENCH_ARGS:-} > gpurun_out/abl/$name.$rep.json 2> gpurun_out/abl/$name.$rep.err
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/abl/$name.$rep.err; restore; exit $rc; }
    python -c "import json; d=json.load(open('gpurun_out/abl/$name.$rep.json')); print('$name', $rep, d['value'], d['ms_per_step'], d.get('roofline',{}).get('achieved'))"
  done
done
restore

#!/bin/bash
# Same-session A/B of the pair-step bench: ARMS = space-separated "name=lib[:VAR=val,VAR=val][|bench args]",
# lib "cur" = the library in place, lib X = ab/libclm_X.so (with ab/_capi_X.py if present);
# default "A=A B=B". REPS rounds (default 3) alternate the arms; BENCH_ARGS are appended. The
# library in place at the end is the one that was in place at the start.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/ab ab
cp clip-lora-match_amd/libclm.so ab/libclm_cur.so
cp clip-lora-match_amd/_capi.py ab/_capi_cur.py
restore() { cp ab/libclm_cur.so clip-lora-match_amd/libclm.so; cp ab/_capi_cur.py clip-lora-match_amd/_capi.py; }
for rep in $(seq 1 ${REPS:-3}); do
  for arm in ${ARMS:-A=A B=B}; do
    name=${arm%%=*}; rest=${arm#*=}; args=""
    case "$rest" in *"|"*) args=${rest#*|}; rest=${rest%%|*};; esac
    lib=${rest%%:*}; envs=""
    [ "$rest" != "$lib" ] && envs=$(echo "${rest#*:}" | tr ',' ' ')
    cp ab/libclm_$lib.so clip-lora-match_amd/libclm.so
    [ -f ab/_capi_$lib.py ] && cp ab/_capi_$lib.py clip-lora-match_amd/_capi.py
    env $envs timeout -k 10 300 python bench.py --no-search --no-cpu-baseline --no-l14 --no-varlen --no-index-build --no-unmerged --no-parity-mode ${BENCH_ARGS:-} $args > gpurun_out/ab/$name.$rep.json 2> gpurun_out/ab/$name.$rep.err
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/ab/$name.$rep.err; restore; exit $rc; }
    python -c "import json; d=json.load(open('gpurun_out/ab/$name.$rep.json')); print('$name', $rep, d['value'], d['ms_per_step'], d.get('roofline',{}).get('achieved'))"
  done
done
restore

#!/bin/bash
# A/B of environment settings on the bench (alternating, same box): ENVS="name:VAR=val,VAR2=val ..."
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/abe
for rep in 1 2; do
  for spec in $ENVS; do
    name=${spec%%:*}; vars=${spec#*:}
    env $(echo "$vars" | tr ',' ' ') timeout -k 10 300 python bench.py --no-search --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/abe/$name.$rep.json 2> gpurun_out/abe/$name.$rep.err
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/abe/$name.$rep.err; exit $rc; }
    python -c "import json; d=json.load(open('gpurun_out/abe/$name.$rep.json')); print('$name', $rep, d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_step'], 'l14', d.get('l14',{}).get('images_per_s'))"
  done
done

#!/bin/bash
# A/B of libclm builds on the bench (alternating, same box): LIBS="name=path ..." BENCH_ARGS=...
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for spec in $LIBS; do
    name=${spec%%=*}; path=${spec#*=}
    CLM_LIB=$path timeout -k 10 300 python bench.py --no-search --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab/$name.$rep.json 2> gpurun_out/ab/$name.$rep.err
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/ab/$name.$rep.err; exit $rc; }
    python -c "import json,sys; d=json.load(open('gpurun_out/ab/$name.$rep.json')); print('$name', $rep, d['value'], d['ms_per_step'], d.get('roofline',{}).get('achieved'), 'l14', d.get('l14',{}).get('images_per_s'), d.get('l14',{}).get('kernel_ms'))"
  done
done

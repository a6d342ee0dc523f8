#!/bin/bash
# scratch GPU session script (the command of the last gpurun call): batched search with the nt cache policy on the
# filter GEMM's index-row DMA (A = HEAD, NT = k_gemm2.hip built with -DCLM_FILTER_W_AUX=2); search legs, 3 rounds
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/ab
cp clip-lora-match_amd/libclm.so ab/libclm_cur.so
for rep in 1 2 3; do
  for arm in A NT; do
    cp ab/libclm_$arm.so clip-lora-match_amd/libclm.so
    timeout -k 10 400 python bench.py --no-cpu-baseline --no-l14 --no-varlen --no-index-build --no-unmerged --no-parity-mode \
      --no-trace --no-encode-item --no-single --no-persist > gpurun_out/ab/f$arm.$rep.json 2> gpurun_out/ab/f$arm.$rep.err
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/ab/f$arm.$rep.err; cp ab/libclm_cur.so clip-lora-match_amd/libclm.so; exit $rc; }
    python -c "
import json; d=json.load(open('gpurun_out/ab/f$arm.$rep.json')); s=d['search']
print('$arm', $rep, d['value'], s['qps'], s['tflops'], s['check']['match'], s.get('near_dup', {}).get('qps'))"
  done
done
cp ab/libclm_cur.so clip-lora-match_amd/libclm.so

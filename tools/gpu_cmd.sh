#!/bin/bash
# scratch GPU session script (the command of the last gpurun call): single-query scan (scan16) with the
# non-temporal (nt) cache policy on its LDS-DMA index stream: A = HEAD, NT = k_search.hip built with
# -DCLM_SCAN_AUX=2; search + single-query legs, 3 rounds alternating
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/ab
cp clip-lora-match_amd/libclm.so ab/libclm_cur.so
for rep in 1 2 3; do
  for arm in A NT; do
    cp ab/libclm_$arm.so clip-lora-match_amd/libclm.so
    timeout -k 10 400 python bench.py --no-cpu-baseline --no-l14 --no-varlen --no-index-build --no-unmerged --no-parity-mode \
      --no-trace --no-encode-item --no-near-dup --no-persist > gpurun_out/ab/s$arm.$rep.json 2> gpurun_out/ab/s$arm.$rep.err
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/ab/s$arm.$rep.err; cp ab/libclm_cur.so clip-lora-match_amd/libclm.so; exit $rc; }
    python -c "
import json; d=json.load(open('gpurun_out/ab/s$arm.$rep.json')); s=d['search']; t=s['single']
print('$arm', $rep, d['value'], s['qps'], t['ms_per_query'], t['device_ms_per_query'], t['device_hbm_frac'], [t['per_call_batch'][k]['ms_per_call'] for k in ('1','2','4','8','16')], t['equal_to_exact_scan'])"
  done
done
cp ab/libclm_cur.so clip-lora-match_amd/libclm.so

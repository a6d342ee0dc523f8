#!/bin/bash
# scratch GPU session script (the command of the last gpurun call): single-query scan shape with the nt policy:
# waves per CU x ring depth (A = 1 x 4, the default; B = 2 x 4; C = 2 x 2; D = 4 x 2); search legs, 2 rounds
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/ab
for rep in 1 2; do
  for arm in A B C D; do
    case $arm in A) envs="";; B) envs="CLM_SCAN_NW=2 CLM_SCAN_D=4";; C) envs="CLM_SCAN_NW=2 CLM_SCAN_D=2";; D) envs="CLM_SCAN_NW=4 CLM_SCAN_D=2";; esac
    env $envs timeout -k 10 400 python bench.py --no-cpu-baseline --no-l14 --no-varlen --no-index-build --no-unmerged --no-parity-mode \
      --no-trace --no-encode-item --no-near-dup --no-persist > gpurun_out/ab/w$arm.$rep.json 2> gpurun_out/ab/w$arm.$rep.err
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/ab/w$arm.$rep.err; exit $rc; }
    python -c "
import json; d=json.load(open('gpurun_out/ab/w$arm.$rep.json')); t=d['search']['single']
print('$arm', $rep, t['ms_per_query'], t['device_ms_per_query'], t['device_hbm_frac'], [t['per_call_batch'][k]['ms_per_call'] for k in ('1','2','4','8','16')], t['equal_to_exact_scan'])"
  done
done

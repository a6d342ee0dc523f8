#!/bin/bash
# one probe run: tools/resln_probe.py [shapes] -> gpurun_out/resln_probe.jsonl (+ a readable table)
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 300 python tools/resln_probe.py ${SHAPES:-} > gpurun_out/resln_probe.jsonl 2> gpurun_out/resln_probe.err
rc=$?
python -c "
import sys,json
for l in open('gpurun_out/resln_probe.jsonl'):
  d=json.loads(l); print(d['shape'], d['variant'], d['us'], d['tflops'])
"
tail -3 gpurun_out/resln_probe.err
exit $rc

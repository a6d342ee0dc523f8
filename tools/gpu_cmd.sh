#!/bin/bash
# scratch GPU session script (the command of the last gpurun call): the default bench line three times on one
# box (run-to-run spread of every leg)
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
for r in 1 2 3; do
  timeout -k 10 900 python -u bench.py --no-trace > gpurun_out/r06t_bench$r.json 2> gpurun_out/r06t_bench$r.err; rc=$?
  echo "bench $r rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r06t_bench$r.err; exit $rc; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/r06t_bench$r.json').read().strip().splitlines()[-1])
print($r, d['value'], d['ms_per_step'], d['search']['qps'], d['l14']['images_per_s'], d['index_build']['images_per_s'], d['search']['single']['ms_per_query'])
"
done

#!/bin/bash
# round-3 session: GPU tests, RESID tile-candidate probe, rocprof kernel stats of both dtypes
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${DO_TEST:-1}" ] && [ "${DO_TEST:-1}" != 0 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${PROBE_CFGS:-}" ]; then
  PROBE_VARIANTS="${PROBE_VARIANTS:-blas,full,noepi}" timeout -k 10 600 python tools/gemm_probe.py "$PROBE_CFGS" "${PROBE_SHAPES:-v_out,t_out,v_fc2,t_fc2}" > gpurun_out/probe.jsonl 2> gpurun_out/probe.err
  rc=$?; echo "probe rc=$rc"; cat gpurun_out/probe.jsonl; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${DO_PROF:-}" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py ${PROF_ARGS:---no-search --no-cpu-baseline --no-l14 --no-varlen --no-index-build --no-unmerged} > gpurun_out/prof.log 2>&1
  rc=$?; echo "prof rc=$rc"; head -c 400 gpurun_out/prof.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${DO_BENCH:-}" ]; then
  timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; echo "bench rc=$rc"; head -c 1500 gpurun_out/bench.json; [ $rc -eq 0 ] || exit $rc
fi

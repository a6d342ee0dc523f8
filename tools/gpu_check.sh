#!/bin/bash
# One GPU session: parity tests, smoke, short bench, rocprof kernel stats.
# Stops at the first GPU fault / abort / timeout (exit codes other than 0/1).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
STAGES=${STAGES:-"test smoke bench prof"}
for st in $STAGES; do
  case $st in
    test)
      timeout -k 10 900 python -m pytest tests -m gpu -q -rf --timeout 600 ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
      rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log; ok $rc || exit $rc ;;
    smoke)
      timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
      rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc ;;
    bench)
      timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
      rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err; [ $rc -eq 0 ] || exit $rc ;;
    splits)
      for sp in 1 2 3 4; do
        timeout -k 10 300 python bench.py --no-search --no-cpu-baseline --split $sp > gpurun_out/bench_split$sp.json 2> gpurun_out/bench_split$sp.err
        rc=$?; echo "split $sp rc=$rc"; cat gpurun_out/bench_split$sp.json; [ $rc -eq 0 ] || exit $rc
      done ;;
    sweep)
      timeout -k 10 600 python tools/gemm_sweep.py > gpurun_out/sweep.jsonl 2> gpurun_out/sweep.err
      rc=$?; echo "sweep rc=$rc"; cat gpurun_out/sweep.jsonl | head -80; tail -3 gpurun_out/sweep.err; [ $rc -eq 0 ] || exit $rc ;;
    split)
      timeout -k 10 600 python tools/gemm_split.py > gpurun_out/split.jsonl 2> gpurun_out/split.err
      rc=$?; echo "split rc=$rc"; cat gpurun_out/split.jsonl; tail -3 gpurun_out/split.err; [ $rc -eq 0 ] || exit $rc ;;
    stalls)
      timeout -k 10 1200 bash tools/gemm_stalls.sh; rc=$?; echo "stalls rc=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    pmc)
      timeout -k 10 1500 bash tools/pmc.sh; rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    prof)
      export TMPDIR=/tmp
      timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --no-cpu-baseline ${PROF_ARGS:-} > gpurun_out/prof.log 2>&1
      rc=$?; echo "prof rc=$rc"; tail -3 gpurun_out/prof.log
      find gpurun_out/prof -name "*stats*" | head; [ $rc -eq 0 ] || exit $rc ;;
  esac
done

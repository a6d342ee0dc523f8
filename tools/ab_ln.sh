set -o pipefail
cd /root/repo
mkdir -p gpurun_out
CLM_LN_ROWS=4 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_encode.py > gpurun_out/ln4_tests.log 2>&1 || { tail -20 gpurun_out/ln4_tests.log; exit 1; }
tail -2 gpurun_out/ln4_tests.log
for r in 2 4 2 4; do CLM_LN_ROWS=$r timeout -k 10 120 python tools/ln_bench.py | sed "s/^/rows=$r /" || exit 1; done
ENVS="r2:CLM_LN_ROWS=2 r4:CLM_LN_ROWS=4" BENCH_ARGS="--no-l14 --no-parity-mode" timeout -k 10 900 bash tools/ab_env.sh

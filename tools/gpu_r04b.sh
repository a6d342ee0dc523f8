cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_encode.py -q -x -k "mixed" --timeout 120 --timeout-method thread > gpurun_out/mixed_tests.log 2>&1; rc=$?; tail -3 gpurun_out/mixed_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/pmc.sh && python3 tools/pmc_summary.py gpurun_out/pmc r04_v3 > gpurun_out/pmc_summary.log 2>&1

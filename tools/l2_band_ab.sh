cd /root/repo
export TMPDIR=/tmp
for b in 1 0; do
  CLM_GEMM_BAND=$b timeout -k 10 240 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/l2ab/b$b -o run -- python3 bench.py --steps 2 --warmup 1 --no-search --no-cpu-baseline --no-l14 --no-parity-mode --no-varlen --sequential > gpurun_out/l2ab/b$b.log 2>&1 || exit $?
  echo "band $b done"
done

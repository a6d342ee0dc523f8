#!/bin/bash
# attention parity tests + L/14 (configs[3]) timing per variant (VARIANTS="name:VAR=v,VAR=v;..."),
# + attention PMC passes with PMC=1
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_encode.py -k "attention or l14" -q -x --timeout 300 --timeout-method thread > gpurun_out/l14_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/l14_pytest.log; [ $rc -eq 0 ] || exit $rc
IFS=';' read -ra ARR <<< "${VARIANTS:-cur:X=0}"
for spec in "${ARR[@]}"; do
  name=${spec%%:*}; envs=${spec#*:}
  env $(echo "$envs" | tr ',' ' ') timeout -k 10 300 python -u tools/l14_run.py 4 > gpurun_out/l14_$name.json 2> gpurun_out/l14_$name.err || { tail -5 gpurun_out/l14_$name.err; exit 1; }
  echo "$name: $(python -c "import json;d=json.load(open('gpurun_out/l14_$name.json'));print(d['images_per_s'], d['attn_tflops'], d['kernel_ms'])")"
done
[ -n "$PMC" ] && { rm -rf gpurun_out/apmc; bash tools/attn_pmc.sh || exit 1; }
exit 0

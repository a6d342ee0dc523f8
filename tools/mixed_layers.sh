#!/bin/bash
# mixed dtype with bf16 text layers (bit mask): pair step and parity vs the goldens
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/ml
for m in 0x0 0xfff 0x3ff 0xff 0x3f 0xffc 0xff0 0xf00 0x0ff 0x00f; do
  CLM_MIXED_TEXT_BF16=$m timeout -k 10 200 python bench.py --no-search --no-cpu-baseline --no-l14 --no-varlen --no-index-build --no-unmerged --no-parity-mode --no-trace > gpurun_out/ml/$m.json 2> gpurun_out/ml/$m.err || { tail -5 gpurun_out/ml/$m.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ml/$m.json')); print('$m', d['value'], d['ms_per_step'], d['parity']['max_score_err'], d['parity']['max_one_minus_cos'])"
done

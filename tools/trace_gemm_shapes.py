"""Per-GEMM-shape durations inside the real encode pipeline, from a rocprofv3 kernel trace of
`bench.py --sequential` (one stream, towers back to back). Every step launches, in order, the
vision patch GEMM, 12 x (qkv, out, fc1, fc2) vision GEMMs, then 12 x (qkv, out, fc1, fc2)
text GEMMs; the GEMM dispatches are split into steps of 97 and averaged per (tower, op).
usage: python tools/trace_gemm_shapes.py <kernel_trace.csv> [label]"""
import csv
import json
import sys
from collections import defaultdict

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "gemm" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
per = 97
nsteps = len(rows) // per
ops = ["qkv", "out", "fc1", "fc2"]
acc = defaultdict(list)
names = {}
for s in range(max(0, nsteps - 8), nsteps):   # the last (steady-state) steps
    seq = rows[s * per:(s + 1) * per]
    for i, r in enumerate(seq):
        if i == 0:
            key = "v_patch"
        elif i < 49:
            key = "v_" + ops[(i - 1) % 4]
        else:
            key = "t_" + ops[(i - 49) % 4]
        acc[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
        names[key] = r["Kernel_Name"].split("(")[0].replace("void clm::(anonymous namespace)::", "")
tot = 0.0
out = {}
for k in ["v_patch", "v_qkv", "v_out", "v_fc1", "v_fc2", "t_qkv", "t_out", "t_fc1", "t_fc2"]:
    v = acc.get(k, [])
    if not v:
        continue
    avg = sum(v) / len(v)
    n = 1 if k == "v_patch" else 12
    tot += avg * n
    out[k] = round(avg, 2)
    print(f"{k:8s} {avg:8.2f} us  x{n:2d}  {names[k]}")
print(f"GEMM total per step: {tot / 1000:.3f} ms")
if len(sys.argv) > 2:
    print(json.dumps({"label": sys.argv[2], "per_shape_us": out, "gemm_ms_per_step": round(tot / 1000, 4)}))

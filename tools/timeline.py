"""Timeline of one encode_pair step from a rocprofv3 kernel trace of `bench.py` (graph mode,
two tower streams): busy union, idle gaps, and time with one vs two kernels in flight.
usage: python tools/timeline.py <kernel_trace.csv>"""
import csv
import sys
from collections import Counter

rows = [r for r in csv.DictReader(open(sys.argv[1]))]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
enc = [r for r in rows if "clm::" in r["Kernel_Name"] and "topk" not in r["Kernel_Name"]
       and "rows_to_f16" not in r["Kernel_Name"] and "sample_rows" not in r["Kernel_Name"]]
# one step = one patchify launch; take the last full step of the timed graph replays
starts = [i for i, r in enumerate(enc) if "patchify" in r["Kernel_Name"]]
i0, i1 = starts[-6], starts[-5]
step = enc[i0:i1]
t0 = int(step[0]["Start_Timestamp"])
ev = []
for r in step:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    ev.append((s, 1, r))
    ev.append((e, -1, r))
ev.sort(key=lambda x: (x[0], x[1]))
level, last, hist = 0, 0, Counter()
for t, d, r in ev:
    hist[min(level, 3)] += t - last
    level += d
    last = t
span = last
kind = Counter()
for r in step:
    n = r["Kernel_Name"]
    k = "gemm" if "gemm" in n else "attn" if "attn" in n else "ln" if "ln" in n else "other"
    kind[k] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
print(f"step span {span / 1e3:.1f} us, kernels {len(step)}")
print("time with 0/1/2/3+ kernels in flight (us):", {k: round(v / 1e3, 1) for k, v in sorted(hist.items())})
print("kernel time by kind (us):", {k: round(v / 1e3, 1) for k, v in kind.items()})

"""Timeline of encode_pair steps from a rocprofv3 kernel trace of `bench.py` (graph replay):
busy union, idle gaps, time with one vs two kernels in flight, and per-kernel time per step.
usage: python tools/timeline.py <kernel_trace.csv> [steps (default 5)]"""
import csv
import re
import sys
from collections import Counter, defaultdict

rows = [r for r in csv.DictReader(open(sys.argv[1]))]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
enc = [r for r in rows if "clm::" in r["Kernel_Name"] and "topk" not in r["Kernel_Name"]
       and "rows_to_f16" not in r["Kernel_Name"] and "sample_rows" not in r["Kernel_Name"]]
# one step = one patchify launch; take the last full steps of the timed graph replays
starts = [i for i, r in enumerate(enc) if "patchify" in r["Kernel_Name"]]
nst = int(sys.argv[2]) if len(sys.argv) > 2 else 5
# the timed replays: the most frequent launch sequence among the steps (the bench's other passes --
# warm-up shapes, the profiled sequential pass, parity -- launch different sequences)
steps = [enc[starts[j]:starts[j + 1]] for j in range(len(starts) - 1)]
sig = Counter(tuple(sorted(r["Kernel_Name"] for r in st)) for st in steps)
top = sig.most_common(1)[0][0]
steps = [st for st in steps if tuple(sorted(r["Kernel_Name"] for r in st)) == top][-nst:]
spans, hist, per = [], Counter(), defaultdict(lambda: [0, 0])
for step in steps:
    t0 = int(step[0]["Start_Timestamp"])
    ev = []
    for r in step:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        ev.append((s, 1))
        ev.append((e, -1))
        name = re.sub(r"\(clm::.*$|\(float const.*$|\(void const.*$|\(int.*$", "", r["Kernel_Name"])
        name = name.replace("void clm::(anonymous namespace)::", "").replace("clm::(anonymous namespace)::", "")
        per[name][0] += e - s
        per[name][1] += 1
    ev.sort()
    level, last = 0, 0
    for t, d in ev:
        hist[min(level, 3)] += t - last
        level += d
        last = t
    spans.append(last)
n = len(spans)
print(f"steps {n}, mean span {sum(spans) / n / 1e3:.1f} us")
print("time per step with 0/1/2/3+ kernels in flight (us):", {k: round(v / n / 1e3, 1) for k, v in sorted(hist.items())})
for name, (t, c) in sorted(per.items(), key=lambda kv: -kv[1][0]):
    print(f"{t / n / 1e3:9.1f} us/step {c // n:4d} launches {t / c / 1e3:8.2f} us avg  {name}")

"""Tabulate tools/gemm_probe.py output: one line per shape, us per variant.
usage: python tools/probe_table.py gpurun_out/probe.jsonl"""
import json
import sys
from collections import defaultdict

d = defaultdict(dict)
for line in open(sys.argv[1]):
    if line.startswith("{"):
        r = json.loads(line)
        d[r["shape"]][r["variant"]] = r["us"]
for s, v in d.items():
    print(f"{s:7s}", " ".join(f"{k}={x}" for k, x in v.items()))

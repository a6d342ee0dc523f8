"""Time the config-4 search leg (10k fp16 queries x 10M x 512 fp16 index, k = 5) once per
environment setting given on the command line as NAME:VAR=val,... (each in a child process)."""
import json
import os
import subprocess
import sys

CODE = r'''
import os, sys, json, torch
sys.path.insert(0, os.getcwd())
import bench
dev = torch.device("cuda", 0)
r = bench.search_leg(int(os.environ.get("ROWS", "10000000")), 10000, 5, dev)[0]
r2 = bench.search_leg(int(os.environ.get("ROWS", "10000000")), 10000, 5, dev)[0]
print(json.dumps({"s1": r["seconds"], "s2": r2["seconds"], "qps": max(r["qps"], r2["qps"])}))
'''
for spec in sys.argv[1:]:
    name, _, kv = spec.partition(":")
    env = dict(os.environ)
    for item in filter(None, kv.split(",")):
        k, _, v = item.partition("=")
        env[k] = v
    out = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=600)
    if out.returncode:
        print(out.stderr[-2000:])
        sys.exit(out.returncode)
    print(name, out.stdout.strip().splitlines()[-1], flush=True)

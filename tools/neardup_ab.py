"""Time the near-duplicate search leg (bench.near_dup_search_leg) once per environment setting
given as NAME:VAR=val,... (each in a child process)."""
import os
import subprocess
import sys

CODE = r'''
import os, sys, json, torch
sys.path.insert(0, os.getcwd())
import bench
dev = torch.device("cuda", 0)
r = [bench.near_dup_search_leg(dev) for _ in range(3)]
print(json.dumps({"qps": [x["qps"] for x in r], "equal": [x["equal_to_full_exact_scan"] for x in r],
                  "paths": r[-1]["paths_timed_block"]}))
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

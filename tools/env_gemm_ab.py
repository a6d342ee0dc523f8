"""GEMM timing per environment setting (each in a child process, since the library reads its
knobs once): python tools/env_gemm_ab.py NAME:VAR=val,... -> JSON lines of µs per launch for
the encoder shapes at the heuristic config and config 4, full epilogue and main loop only."""
import json
import os
import subprocess
import sys

CODE = r'''
import json, os, sys, torch
sys.path.insert(0, os.getcwd())
from clip_lora_match_amd import _capi as C
B = 256
SHAPES = {"v_qkv": (B*50, 2304, 768, 0), "v_out": (B*50, 768, 768, 2), "v_fc1": (B*50, 3072, 768, 1),
          "v_fc2": (B*50, 768, 3072, 2), "t_qkv": (B*77, 1536, 512, 0), "t_out": (B*77, 512, 512, 2),
          "t_fc1": (B*77, 2048, 512, 1), "t_fc2": (B*77, 512, 2048, 2), "sq4096": (4096, 4096, 4096, 0)}
dev = torch.device("cuda", 0); L = C.lib(); st = torch.cuda.current_stream()
res = {}
for name, (M, N, K, epi) in SHAPES.items():
    A = (torch.rand((M, K), device=dev) * 2 - 1).to(torch.bfloat16)
    W = ((torch.rand((N, K), device=dev) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
    out = torch.zeros((M, N), device=dev, dtype=torch.float32 if epi == 2 else torch.bfloat16)
    bias = torch.zeros(N, device=dev)
    for cfg in [int(c) for c in os.environ.get("AB_CFGS", "-1,4").split(",")]:
        for dbg in (0, 1):
            L.clm_debug_set(dbg)
            run = lambda: C.check(L.clm_gemm(0, C.CLM_BF16, epi, cfg, C.ptr(A), K, C.ptr(W), K, M, N, K, C.ptr(out), N,
                                             C.ptr(bias), None, None, C.stream_of(dev)))
            run(); ts = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(10): run()
                e1.record(st); e1.synchronize(); ts.append(e0.elapsed_time(e1) / 10 * 1e3)
            res[f"{name}.c{cfg}{'.noepi' if dbg else ''}"] = round(sorted(ts)[2], 2)
    L.clm_debug_set(0)
print(json.dumps(res))
'''
for spec in sys.argv[1:] or ["default:"]:
    name, _, kv = spec.partition(":")
    env = dict(os.environ)
    for item in filter(None, kv.split(",")):
        k, _, v = item.partition("=")
        env[k] = v
    out = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=600)
    print(name, out.stdout.strip().splitlines()[-1] if out.returncode == 0 else out.stderr[-2000:], flush=True)

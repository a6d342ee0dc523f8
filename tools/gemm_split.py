"""Main-loop vs epilogue split: time each encoder GEMM shape with its auto tile, with and
without the epilogue (CLM_GEMM_DEBUG=1 in a child process), and at K x 4 (fixed-cost fit)."""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CODE = r'''
import os, sys, json, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(sys.argv[1]))))
from clip_lora_match_amd import _capi as C
shapes = json.loads(sys.argv[2])
dev = torch.device("cuda", 0); L = C.lib(); st = torch.cuda.current_stream()
res = {}
for name, (M, N, K, epi) in shapes.items():
    A = (torch.rand((M, K), device=dev) * 2 - 1).to(torch.bfloat16)
    W = ((torch.rand((N, K), device=dev) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
    out = torch.zeros((M, N), device=dev, dtype=torch.float32 if epi == 2 else torch.bfloat16)
    bias = torch.zeros(N, device=dev)
    run = lambda: C.check(L.clm_gemm(0, C.CLM_BF16, epi, -1, C.ptr(A), K, C.ptr(W), K, M, N, K, C.ptr(out), N,
                                     C.ptr(bias), None, None, C.stream_of(dev)))
    run(); torch.cuda.synchronize()
    best = 1e9
    for r in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(10): run()
        e1.record(st); e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / 10 * 1e3)
    res[name] = best
print(json.dumps(res))
'''
B = 256
SHAPES = {"v_qkv": (B * 50, 2304, 768, 0), "v_out": (B * 50, 768, 768, 2), "v_fc1": (B * 50, 3072, 768, 1),
          "v_fc2": (B * 50, 768, 3072, 2), "t_qkv": (B * 77, 1536, 512, 0), "t_out": (B * 77, 512, 512, 2),
          "t_fc1": (B * 77, 2048, 512, 1), "t_fc2": (B * 77, 512, 2048, 2)}
SHAPES4 = {k + "_K4": (M, N, K * 4, e) for k, (M, N, K, e) in SHAPES.items()}


def run(env_extra, shapes):
    env = dict(os.environ, **env_extra)
    out = subprocess.run([sys.executable, "-c", CODE, os.path.join(HERE, "x"), json.dumps(shapes)], env=env,
                         capture_output=True, text=True, timeout=300)
    if out.returncode:
        print(out.stderr[-2000:], file=sys.stderr)
        raise SystemExit(out.returncode)
    return json.loads(out.stdout.strip().splitlines()[-1])


full = run({}, SHAPES)
noepi = run({"CLM_GEMM_DEBUG": "1"}, SHAPES)
k4 = run({}, SHAPES4)
for k in SHAPES:
    print(json.dumps({"shape": k, "full_us": round(full[k], 2), "mainloop_only_us": round(noepi[k], 2),
                      "k_x4_us": round(k4[k + "_K4"], 2),
                      "fixed_us_fit": round(full[k] - (k4[k + "_K4"] - full[k]) / 3, 2)}))

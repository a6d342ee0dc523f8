"""GEMM probe: per encoder shape, time (a) torch.mm bf16 (hipBLASLt) as a same-box reference,
(b) clm_gemm per tile config with the real epilogue, (c) main loop only (debug bit 1),
(d) epilogue computed but every store dropped (debug bit 2), (e) K = 64 (fixed cost),
(f) one tile per workgroup instead of the persistent grid (debug bit 4), (g) no bias vector.
All variants of one shape run interleaved in ONE process (median of rounds), random operands.
usage: python tools/gemm_probe.py [cfg,cfg,...] [shape,shape,...] -> one JSON line per (shape, variant)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from clip_lora_match_amd import _capi as C  # noqa: E402

B = 256
SHAPES = {"v_qkv": (B * 50, 2304, 768, 0), "v_out": (B * 50, 768, 768, 2), "v_fc1": (B * 50, 3072, 768, 1),
          "v_fc2": (B * 50, 768, 3072, 2), "t_qkv": (B * 77, 1536, 512, 0), "t_out": (B * 77, 512, 512, 2),
          "t_fc1": (B * 77, 2048, 512, 1), "t_fc2": (B * 77, 512, 2048, 2), "sq4096": (4096, 4096, 4096, 0),
          "sq8k": (8192, 8192, 8192, 0),
          # configs[3] ViT-L/14@336 at batch 128 (M = 128 x 577)
          "l_qkv": (128 * 577, 3072, 1024, 0), "l_out": (128 * 577, 1024, 1024, 2),
          "l_fc1": (128 * 577, 4096, 1024, 1), "l_fc2": (128 * 577, 1024, 4096, 2),
          # the pruned last layer: B pooled rows
          "pv_out": (B, 768, 768, 2), "pv_fc1": (B, 3072, 768, 1), "pv_fc2": (B, 768, 3072, 2),
          "pt_out": (B, 512, 512, 2), "pt_fc1": (B, 2048, 512, 1), "pt_fc2": (B, 512, 2048, 2)}
cfgs = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [-1]
only = sys.argv[2].split(",") if len(sys.argv) > 2 else [k for k in SHAPES if k[0] in "vt"]
dev = torch.device("cuda", 0)
L = C.lib()
st = torch.cuda.current_stream()
sptr = C.stream_of(dev)


def timed(fn, reps=10, rounds=5):
    ts = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            fn()
        e1.record(st)
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) / reps * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


for name in only:
    M, N, K, epi = SHAPES[name]
    A = (torch.rand((M, K), device=dev) * 2 - 1).to(torch.bfloat16)
    W = ((torch.rand((N, K), device=dev) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
    out = torch.zeros((M, N), device=dev, dtype=torch.float32 if epi == 2 else torch.bfloat16)
    bias = torch.zeros(N, device=dev)
    ob = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
    out2 = torch.zeros_like(out)

    def ours(cfg, dbg, k=K, use_bias=True):
        def f():
            L.clm_debug_set(dbg)
            C.check(L.clm_gemm(0, C.CLM_BF16, epi, cfg, C.ptr(A), K, C.ptr(W), K, M, N, k, C.ptr(out), N,
                               C.ptr(bias) if use_bias else None, None, None, sptr))
        return f

    variants = {"blas": lambda: torch.mm(A, W.t(), out=ob), "fill_out": lambda: out.fill_(1.0),
                "copy_out": lambda: out.copy_(out2)}
    for cfg in cfgs:
        variants[f"c{cfg}_full"] = ours(cfg, 0)
        variants[f"c{cfg}_np"] = ours(cfg, 4)
        variants[f"c{cfg}_noepi"] = ours(cfg, 1)
        variants[f"c{cfg}_nostore"] = ours(cfg, 2)
        variants[f"c{cfg}_nobias"] = ours(cfg, 0, K, False)
        variants[f"c{cfg}_k64"] = ours(cfg, 0, 64)
        variants[f"c{cfg}_k64nobias"] = ours(cfg, 0, 64, False)
        variants[f"c{cfg}_k64noepi"] = ours(cfg, 1, 64)
        variants[f"c{cfg}_k64nostore"] = ours(cfg, 2, 64)
    keep = os.environ.get("PROBE_VARIANTS")   # e.g. "blas,full": suffixes to keep
    if keep:
        ks = keep.split(",")
        variants = {k: v for k, v in variants.items() if k in ks or k.split("_", 1)[-1] in ks}
    for fn in variants.values():
        fn()
    torch.cuda.synchronize()
    res = {k: [] for k in variants}
    for _ in range(3):
        for k, fn in variants.items():
            res[k].append(timed(fn))
    L.clm_debug_set(0)
    flop = 2.0 * M * N * K
    for k, v in res.items():
        t = sorted(v)[1]
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "variant": k, "us": round(t, 2),
                          "tflops": None if "k64" in k or "_out" in k else round(flop / t / 1e6, 1)}), flush=True)

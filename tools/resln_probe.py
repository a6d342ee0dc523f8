"""Probe of the fused residual GEMM + LayerNorm (k_resln.hip) per encoder shape, against the
two-launch path it replaces (RESID GEMM at the heuristic tile + ln4 LayerNorm): full kernel per
row tiling, main loop only (debug bit 1), residual update without LayerNorm (debug bit 2), W operand through
the LDS ring instead of straight to registers (debug bit 16).
Interleaved in one process, median of rounds, random operands.
usage: python tools/resln_probe.py [shape,...] -> one JSON line per (shape, variant)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from clip_lora_match_amd import _capi as C  # noqa: E402

B = 256
SHAPES = {"v_out": (B * 50, 768, 768), "v_fc2": (B * 50, 768, 3072), "t_out": (B * 77, 512, 512),
          "t_fc2": (B * 77, 512, 2048), "pv_out": (B, 768, 768), "pt_out": (B, 512, 512)}
only = sys.argv[1].split(",") if len(sys.argv) > 1 else list(SHAPES)
dev = torch.device("cuda", 0)
L = C.lib()
st = torch.cuda.current_stream()
sp = C.stream_of(dev)
DT = C.CLM_F16


def timed(fn, reps=10, rounds=7):
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
    M, N, K = SHAPES[name]
    A = (torch.rand((M, K), device=dev) * 2 - 1).half()
    W = ((torch.rand((N, K), device=dev) * 2 - 1) / K ** 0.5).half()
    h = torch.randn((M, N), device=dev) * 0.01
    bias, gam, bet = torch.zeros(N, device=dev), torch.ones(N, device=dev), torch.zeros(N, device=dev)
    y = torch.empty((M, N + 64), device=dev, dtype=torch.half)

    def rl(bm, dbg):
        def f():
            L.clm_debug_set(dbg)
            C.check(L.clm_gemm_resid_ln(0, DT, C.ptr(A), K, C.ptr(W), K, M, N, K, C.ptr(h), N, C.ptr(bias), C.ptr(gam),
                                        C.ptr(bet), 1e-5, C.ptr(y), y.stride(0), bm, sp))
        return f

    def resid():
        L.clm_debug_set(0)
        C.check(L.clm_gemm(0, DT, C.CLM_EPI_RESID, -1, C.ptr(A), K, C.ptr(W), K, M, N, K, C.ptr(h), N, C.ptr(bias),
                           None, None, sp))

    def ln():
        C.check(L.clm_layernorm(0, DT, C.ptr(h), N, M, N, C.ptr(gam), C.ptr(bet), 1e-5, C.ptr(y), y.stride(0), sp))

    variants = {"resid": resid, "ln": ln}
    for bm in (32, 64, 80):
        variants[f"rl{bm}"] = rl(bm, 0)          # W fragments straight to registers
        variants[f"rl{bm}_noepi"] = rl(bm, 1)
        variants[f"rl{bm}_noln"] = rl(bm, 2)
        variants[f"rl{bm}L"] = rl(bm, 16)        # W through the LDS ring (debug bit 4)
        variants[f"rl{bm}L_noepi"] = rl(bm, 17)
    for f in variants.values():
        f()
    torch.cuda.synchronize()
    res = {k: [] for k in variants}
    for _ in range(3):
        for k, f in variants.items():
            res[k].append(timed(f))
    L.clm_debug_set(0)
    for k, v in res.items():
        v.sort()
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "variant": k, "us": round(v[1], 2),
                          "tflops": round(2.0 * M * N * K / v[1] / 1e6, 1)}), flush=True)

"""PP GEMM probe: per encoder shape, check the PP configs (12-16, k_gemm3.hip) bit for bit against
the picked gemm_kernel / G2 config on the same random fp16 operands and epilogue, then time full /
main-loop-only (debug bit 1) / epilogue without its stores (debug bit 2) of every config, interleaved in ONE process (median of rounds).
usage: python tools/pp_probe.py [cfg,cfg,...] [shape,shape,...] -> one JSON line per (shape, variant)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from clip_lora_match_amd import _capi as C  # noqa: E402

B = 256
SHAPES = {"v_qkv": (B * 50, 2304, 768, 0), "v_out": (B * 50, 768, 768, 2), "v_fc1": (B * 50, 3072, 768, 1),
          "v_fc2": (B * 50, 768, 3072, 2), "t_qkv": (B * 77, 1536, 512, 0), "t_out": (B * 77, 512, 512, 2),
          "t_fc1": (B * 77, 2048, 512, 1), "t_fc2": (B * 77, 512, 2048, 2), "odd": (1000, 200, 192, 1),
          "l_fc1": (128 * 577, 4096, 1024, 1), "l_fc2": (128 * 577, 1024, 4096, 2),
          "l_qkv": (128 * 577, 3072, 1024, 0), "l_out": (128 * 577, 1024, 1024, 2), "sq8k": (8192, 8192, 8192, 0)}
cfgs = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [12, 13, 14, 15, 16]
only = sys.argv[2].split(",") if len(sys.argv) > 2 else ["v_fc1", "t_fc1", "v_fc2", "t_fc2", "v_out", "t_out", "v_qkv"]
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


torch.manual_seed(0)
INT = os.environ.get("PROBE_INT", "0") == "1"
TIME = os.environ.get("PROBE_TIME", "1") == "1"
for name in only:
    M, N, K, epi = SHAPES[name]
    if INT:   # small integers: every sum exact in fp32, so any MFMA shape / K order gives the same bits
        A = torch.randint(-2, 3, (M, K), device=dev).half()
        W = torch.randint(-2, 3, (N, K), device=dev).half()
        h0 = torch.randint(-8, 9, (M, N), device=dev).float() if epi == 2 else None
        bias = torch.randint(-4, 5, (N,), device=dev).float()
    else:
        A = (torch.rand((M, K), device=dev) * 2 - 1).half()
        W = ((torch.rand((N, K), device=dev) * 2 - 1) / K ** 0.5).half()
        h0 = torch.randn((M, N), device=dev) if epi == 2 else None
        bias = torch.randn(N, device=dev) * 0.1
    odt = torch.float32 if epi == 2 else torch.float16

    def run(cfg, out, dbg=0):
        L.clm_debug_set(dbg)
        C.check(L.clm_gemm(0, C.CLM_F16, epi, cfg, C.ptr(A), K, C.ptr(W), K, M, N, K, C.ptr(out), N,
                           C.ptr(bias), None, None, sptr))

    def fresh():
        return h0.clone() if epi == 2 else torch.zeros((M, N), device=dev, dtype=odt)

    ref = fresh()
    run(-1, ref)
    torch.cuda.synchronize()
    for cfg in cfgs:
        o = fresh()
        run(cfg, o)
        torch.cuda.synchronize()
        same = torch.equal(o.view(torch.int16 if odt == torch.float16 else torch.int32),
                           ref.view(torch.int16 if odt == torch.float16 else torch.int32))
        diff = (o.float() - ref.float()).abs().max().item()
        print(json.dumps({"shape": name, "cfg": cfg, "bit_equal_to_picked": same, "max_abs_diff": diff}), flush=True)
    if name == "odd" or not TIME:
        continue
    bufs = {}
    variants = {"blas": lambda: torch.mm(A, W.t())}
    for cfg in [-1] + cfgs:
        bufs[cfg] = fresh()
        variants[f"c{cfg}_full"] = (lambda c: lambda: run(c, bufs[c]))(cfg)
        variants[f"c{cfg}_noepi"] = (lambda c: lambda: run(c, bufs[c], 1))(cfg)
        variants[f"c{cfg}_nostore"] = (lambda c: lambda: run(c, bufs[c], 2))(cfg)
        for dv in filter(None, os.environ.get("PROBE_DBG", "").split(",")):   # extra debug-flag variants
            variants[f"c{cfg}_dbg{dv}"] = (lambda c, v: lambda: run(c, bufs[c], v))(cfg, int(dv))
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
                          "tflops": round(flop / t / 1e6, 1)}), flush=True)

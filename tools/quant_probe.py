"""Wave-quantization probe: one GEMM shape and tile config timed at several row counts M (the
persistent grid's rounds = ceil(tiles / slots)), interleaved in one process, random operands.
usage: python tools/quant_probe.py N K epi cfg M1,M2,... -> one JSON line per M"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from clip_lora_match_amd import _capi as C  # noqa: E402

N, K, epi, cfg = (int(x) for x in sys.argv[1:5])
Ms = [int(x) for x in sys.argv[5].split(",")]
dev = torch.device("cuda", 0)
L = C.lib()
st = torch.cuda.current_stream()
sptr = C.stream_of(dev)
Mx = max(Ms)
A = (torch.rand((Mx, K), device=dev) * 2 - 1).to(torch.bfloat16)
W = ((torch.rand((N, K), device=dev) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
out = torch.zeros((Mx, N), device=dev, dtype=torch.float32 if epi in (2, 4) else torch.bfloat16)
bias = torch.rand(N, device=dev)
res = {M: [] for M in Ms}
for _ in range(5):
    for M in Ms:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(20):
            C.check(L.clm_gemm(0, C.CLM_BF16, epi, cfg, C.ptr(A), K, C.ptr(W), K, M, N, K, C.ptr(out), N,
                               C.ptr(bias), None, None, sptr))
        e1.record(st)
        e1.synchronize()
        res[M].append(e0.elapsed_time(e1) / 20 * 1e3)
for M in Ms:
    us = sorted(res[M])[2]
    print(json.dumps({"N": N, "K": K, "epi": epi, "cfg": cfg, "M": M, "us": round(us, 2),
                      "tflops": round(2 * M * N * K / us / 1e6, 1)}), flush=True)

"""Epilogue cost probe for the quick-GELU fc1 GEMMs: the same shape and tile config timed with the
GELU epilogue, the plain STORE epilogue (bias + pack, no GELU) and the main loop only (debug bit 1),
interleaved in one process on random operands.
usage: python tools/epi_probe.py [cfg] -> one JSON line per shape"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from clip_lora_match_amd import _capi as C  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else -1
dev = torch.device("cuda", 0)
L = C.lib()
st = torch.cuda.current_stream()
sptr = C.stream_of(dev)
for name, (M, N, K) in {"v_fc1": (12800, 3072, 768), "t_fc1": (19712, 2048, 512)}.items():
    A = (torch.rand((M, K), device=dev) * 2 - 1).to(torch.bfloat16)
    W = ((torch.rand((N, K), device=dev) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
    out = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
    bias = torch.rand(N, device=dev)

    def run(epi, dbg):
        L.clm_debug_set(dbg)
        C.check(L.clm_gemm(0, C.CLM_BF16, epi, cfg, C.ptr(A), K, C.ptr(W), K, M, N, K, C.ptr(out), N,
                           C.ptr(bias), None, None, sptr))

    res = {}
    for _ in range(5):
        for lab, epi, dbg in (("gelu", 1, 0), ("store", 0, 0), ("mainloop", 1, 1)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(20):
                run(epi, dbg)
            e1.record(st)
            e1.synchronize()
            res.setdefault(lab, []).append(e0.elapsed_time(e1) / 20 * 1e3)
    L.clm_debug_set(0)
    print(json.dumps({"shape": name, "cfg": cfg, **{k: round(sorted(v)[2], 2) for k, v in res.items()}}), flush=True)

"""Run one GEMM shape/config repeatedly (for rocprofv3 --pmc stall analysis).
usage: python tools/gemm_one.py M N K epi cfg reps"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from clip_lora_match_amd import _capi as C  # noqa: E402

M, N, K, epi, cfg, reps = (int(x) for x in sys.argv[1:7])
dev = torch.device("cuda", 0)
A = (torch.rand((M, K), device=dev) * 2 - 1).to(torch.bfloat16)
W = ((torch.rand((N, K), device=dev) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
out = torch.zeros((M, N), device=dev, dtype=torch.float32 if epi == C.CLM_EPI_RESID else torch.bfloat16)
bias = torch.zeros(N, device=dev)
L = C.lib()
for _ in range(reps):
    C.check(L.clm_gemm(0, C.CLM_BF16, epi, cfg, C.ptr(A), K, C.ptr(W), K, M, N, K, C.ptr(out), N, C.ptr(bias),
                       None, None, C.stream_of(dev)))
torch.cuda.synchronize()
print("ok")

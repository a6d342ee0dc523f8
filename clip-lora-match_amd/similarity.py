"""Drop-in for src/embedding/similarity.py on the gfx950 kernels.

  cosine_similarity  similarity.py:10-33  normalise both sides, (1,d) @ (N,d)^T -> (N,)
  top_k_similar      similarity.py:36-58  topk(min(k, N)) -> (values (k,), indices (k,))

Scores come from the fp16-operand MFMA GEMM with fp32 accumulation and fp32
norms of the source rows (within 1e-3 of the fp32 CPU reference; typically
~1e-5); top-k ties are ordered (score desc, index asc).
"""
from __future__ import annotations

from typing import Tuple

import torch

from . import _capi as C
from .search import CosineIndex, _pad_dim


def cosine_similarity(query: torch.Tensor, candidates: torch.Tensor) -> torch.Tensor:
    C.require_gpu()
    q = torch.as_tensor(query)
    if q.dim() == 1:
        q = q.unsqueeze(0)
    c = torch.as_tensor(candidates)
    if c.dim() != 2 or q.dim() != 2 or q.shape[-1] != c.shape[-1]:
        raise ValueError(f"shape mismatch: query {tuple(q.shape)} vs candidates {tuple(c.shape)}")
    out_dev = c.device
    dev = torch.device("cuda", torch.cuda.current_device())
    d = q.shape[-1]
    dp = (d + 63) // 64 * 64
    qg = _pad_dim(q.float().to(dev), dp).contiguous()
    cg = _pad_dim(c.float().to(dev), dp).contiguous()
    out = torch.empty((qg.shape[0], cg.shape[0]), dtype=torch.float32, device=dev)
    C.check(C.lib().clm_cosine_scores(dev.index, C.ptr(qg), qg.shape[0], C.ptr(cg), cg.shape[0], dp, C.ptr(out),
                                      C.stream_of(dev)), "clm_cosine_scores")
    return out.squeeze(0).to(out_dev)


def top_k_similar(query: torch.Tensor, candidates: torch.Tensor, k: int = 5) -> Tuple[torch.Tensor, torch.Tensor]:
    c = torch.as_tensor(candidates)
    q = torch.as_tensor(query)
    if q.dim() == 1:
        q = q.unsqueeze(0)
    if c.dim() != 2 or q.shape[-1] != c.shape[-1]:
        raise ValueError(f"shape mismatch: query {tuple(q.shape)} vs candidates {tuple(c.shape)}")
    k = min(int(k), c.shape[0])
    if k < 0:
        raise RuntimeError("selected index k out of range")
    if k == 0:
        return torch.empty(0), torch.empty(0, dtype=torch.int64)
    idx = CosineIndex(c.shape[1], capacity=c.shape[0])
    try:
        # the reference normalises the fp32 candidates first (similarity.py:30); store those rows
        cn = c.float()
        cn = cn / cn.norm(p=2, dim=-1, keepdim=True)
        idx.append(cn)
        s, i = idx.search(q.float(), k)
    finally:
        idx.close()
    return s[0].to(c.device), i[0].to(c.device)

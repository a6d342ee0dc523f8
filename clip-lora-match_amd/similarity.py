"""Drop-in for src/embedding/similarity.py on the gfx950 kernels.

  cosine_similarity  similarity.py:10-33  normalise both sides, (1,d) @ (N,d)^T -> (N,)
  top_k_similar      similarity.py:36-58  topk(min(k, N)) -> (values (k,), indices (k,))

Scores are exact: the fp64 cosine of the caller's fp32 vectors, rounded once to
fp32 (the reference's fp32 matmul of fp32-normalised rows differs from it only by
its own summation rounding, ~1e-7). top_k_similar bounds its candidates with the
fp16 MFMA pass and re-scores them exactly (clm_index_search); ties are ordered
(score desc, index asc).
"""
from __future__ import annotations

from typing import Tuple

import torch

from . import _capi as C
from .search import CosineIndex


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
    qg = q.float().to(dev).contiguous()
    cg = c.float().to(dev).contiguous()
    out = torch.empty((qg.shape[0], cg.shape[0]), dtype=torch.float32, device=dev)
    C.check(C.lib().clm_cosine_scores(dev.index, C.ptr(qg), qg.shape[0], C.ptr(cg), cg.shape[0], q.shape[-1],
                                      C.ptr(out), C.stream_of(dev)), "clm_cosine_scores")
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
        # the reference normalises the fp32 candidates first (similarity.py:30): store those rows
        # (the exact re-score reads them as given)
        cn = c.float()
        cn = cn / cn.norm(p=2, dim=-1, keepdim=True)
        idx.append(cn)
        s, i = idx.search(q.float(), k)
    finally:
        idx.close()
    return s[0].to(c.device), i[0].to(c.device)

"""Batch data parallelism for the encode / index-build / search path over the
GPUs of one node: one process per GPU, torch.distributed with the "nccl"
backend (RCCL on ROCm) over xGMI.

The reference has no parallelism at all; this adds exactly the
exchange steps the path has:

* index build (scripts/rebuild_index.py:64-96 generalised to N GPUs): rank r
  encodes rows [shard_range(n, r, world)) and one all_gather of the fp32 (or
  fp16) embeddings gives every rank the whole index in global order;
* sharded search: each rank keeps rows [start, stop) of the HBM index with
  global offset `start`, searches its shard locally (GEMM + exact top-k), one
  all_gather of the [nq, k] (score, index) lists, then the same
  (score desc, index asc) merge -- top-k of a union equals top-k of the
  per-shard top-ks, so the result is identical to the single-GPU order.

The collective plumbing takes injectable local-search / merge functions so it
is testable with the gloo backend on CPU (tests/test_distributed_cpu.py); the
product defaults are the GPU index and the clm_topk_merge kernel.
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import torch
import torch.distributed as dist


def shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous balanced shard [start, stop) of n rows for `rank` of `world`."""
    if world <= 0 or not (0 <= rank < world) or n < 0:
        raise ValueError("bad shard arguments")
    base, rem = divmod(n, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def all_gather_rows(local: torch.Tensor, n_total: int, group=None) -> torch.Tensor:
    """Concatenate every rank's shard (shard_range layout, uneven sizes allowed) on every rank."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    start, stop = shard_range(n_total, rank, world)
    if local.shape[0] != stop - start:
        raise ValueError(f"rank {rank} holds {local.shape[0]} rows, shard is {stop - start}")
    width = (n_total + world - 1) // world
    buf = torch.zeros((width,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    buf[: local.shape[0]] = local
    out = torch.empty((world * width,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, buf, group=group)
    pieces = []
    for r in range(world):
        s, e = shard_range(n_total, r, world)
        pieces.append(out[r * width: r * width + (e - s)])
    return torch.cat(pieces, 0)


def gather_candidates(scores: torch.Tensor, idx: torch.Tensor, group=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """[nq, k] per rank -> [nq, world*k] on every rank (rank-major within a row)."""
    world = dist.get_world_size(group)
    nq, k = scores.shape
    s_all = torch.empty((world * nq, k), dtype=scores.dtype, device=scores.device)
    i_all = torch.empty((world * nq, k), dtype=idx.dtype, device=idx.device)
    dist.all_gather_into_tensor(s_all, scores.contiguous(), group=group)
    dist.all_gather_into_tensor(i_all, idx.contiguous(), group=group)
    s_all = s_all.view(world, nq, k).permute(1, 0, 2).reshape(nq, world * k)
    i_all = i_all.view(world, nq, k).permute(1, 0, 2).reshape(nq, world * k)
    return s_all, i_all


def merge_topk_gpu(scores: torch.Tensor, idx: torch.Tensor, parts: int, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """(score desc, index asc) merge of `parts` candidate lists per row on the GPU (clm_topk_merge)."""
    from . import _capi as C
    nq, n_in = scores.shape
    k_in = n_in // parts
    s = scores.contiguous()
    i = idx.contiguous()
    os_ = torch.empty((nq, k), dtype=torch.float32, device=s.device)
    oi = torch.empty((nq, k), dtype=torch.int64, device=s.device)
    C.check(C.lib().clm_topk_merge(s.device.index, C.ptr(s), C.ptr(i), nq, parts, k_in, k, C.ptr(os_), C.ptr(oi),
                                   C.stream_of(s.device)), "clm_topk_merge")
    return os_, oi


class ShardedIndex:
    """Row-sharded cosine index: this rank holds rows [start, stop) of n_total."""

    def __init__(self, dim: int, n_total: int, group=None, device=None,
                 local_factory: Optional[Callable] = None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.dim = dim
        self.n_total = n_total
        self.start, self.stop = shard_range(n_total, self.rank, self.world)
        if local_factory is None:
            from .search import CosineIndex
            local_factory = lambda: CosineIndex(dim, capacity=max(self.stop - self.start, 1), device=device)  # noqa
        self.local = local_factory()
        self.local.set_offset(self.start)

    def append_shard(self, rows: torch.Tensor) -> None:
        if rows.shape[0] != self.stop - self.start:
            raise ValueError("rows must be exactly this rank's shard")
        self.local.append(rows)

    def search(self, queries: torch.Tensor, k: int,
               merge: Callable = merge_topk_gpu) -> Tuple[torch.Tensor, torch.Tensor]:
        s, i = self.local.search(queries, k)
        if self.world == 1:
            return s, i
        s_all, i_all = gather_candidates(s, i, self.group)
        return merge(s_all, i_all, self.world, k)


def build_index_sharded(encode_rows: Callable[[int, int], torch.Tensor], n_total: int, batch: int,
                        group=None, exchange: Optional[Callable[[torch.Tensor], torch.Tensor]] = None,
                        restore: Optional[Callable[[torch.Tensor], torch.Tensor]] = None) -> torch.Tensor:
    """Index build over N GPUs: encode_rows(start, stop) encodes global rows [start, stop)
    (e.g. a slice of images or captions) on this rank's GPU; returns all n_total embeddings
    on every rank (one all_gather). exchange / restore (optional) map the local rows to the form
    that crosses the links and the gathered rows back (index_build's fp16 exchange: half the
    bytes of the fp32 rows)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    start, stop = shard_range(n_total, rank, world)
    outs = [encode_rows(s, min(s + batch, stop)) for s in range(start, stop, batch)]
    local = torch.cat(outs, 0) if outs else encode_rows(start, start)   # [0, D] for an empty shard
    if exchange is not None:
        local = exchange(local)
    rows = all_gather_rows(local, n_total, group)
    return restore(rows) if restore is not None else rows

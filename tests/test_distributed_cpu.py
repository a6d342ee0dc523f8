"""N>1 path with the gloo backend on CPU (world_size 2 and 3): shard layout,
uneven all-gather of embeddings (index build), sharded search candidate
exchange + merge == single-process oracle top-k. The per-shard search and the
merge are injected CPU oracle functions; on GPUs they are the HIP index and
the clm_topk_merge kernel (tests/test_gpu_distributed.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from clip_lora_match_amd.distributed import (ShardedIndex, all_gather_rows, build_index_sharded,
                                             shard_range)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _OracleShard:
    """CPU stand-in for CosineIndex with the same interface (test-only)."""

    def __init__(self):
        self.rows = None
        self.offset = 0

    def set_offset(self, o):
        self.offset = o

    def append(self, rows):
        self.rows = rows.float()

    def search(self, q, k):
        from oracle import search_ref as S
        out_s = np.full((q.shape[0], k), -np.inf, np.float32)
        out_i = np.full((q.shape[0], k), -1, np.int64)
        if self.rows is not None and self.rows.shape[0]:
            s, i = S.search(q.numpy(), self.rows.numpy(), k)   # like the GPU index: pad (-inf, -1)
            out_s[:, :s.shape[1]], out_i[:, :i.shape[1]] = s, i + self.offset
        return torch.from_numpy(out_s), torch.from_numpy(out_i)


def _oracle_merge(s_all, i_all, parts, k):
    from oracle import search_ref as S
    s = s_all.numpy().astype(np.float64)
    order = np.lexsort((i_all.numpy(), -s), axis=-1)[:, :k]
    return torch.from_numpy(np.take_along_axis(s, order, 1)), torch.from_numpy(np.take_along_axis(i_all.numpy(), order, 1))


def _worker(rank, world, port, n, dim, nq, k, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(0)
        full = rng.standard_normal((n, dim)).astype(np.float32)
        # index build: every rank "encodes" its shard (identity here), one all_gather
        got = build_index_sharded(lambda s, e: torch.from_numpy(full[s:e] * 2.0), n, batch=7)
        assert torch.equal(got, torch.from_numpy(full * 2.0))
        # the fp16 exchange form (index_build exchange="fp16"): the rows cross the links as fp16 and
        # are restored after the gather -- equal to the same round trip done without ranks
        got16 = build_index_sharded(lambda s, e: torch.from_numpy(full[s:e]), n, batch=5,
                                    exchange=lambda r: r.to(torch.float16), restore=lambda r: r.float() * 3.0)
        assert got16.dtype == torch.float32
        assert torch.equal(got16, torch.from_numpy(full).to(torch.float16).float() * 3.0)
        # sharded search
        idx = ShardedIndex(dim, n, local_factory=_OracleShard)
        idx.append_shard(torch.from_numpy(full[idx.start:idx.stop]))
        qs = torch.from_numpy(rng.standard_normal((nq, dim)).astype(np.float32))
        s, i = idx.search(qs, k, merge=_oracle_merge)
        from oracle import search_ref as S
        es, ei = S.search(qs.numpy(), full, k)
        assert np.array_equal(i.numpy(), ei), (i, ei)
        assert np.allclose(s.numpy(), es, atol=1e-6)
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 101), (3, 64), (2, 1), (4, 3), (8, 37)])
def test_sharded_build_and_search_gloo(world, n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, 32, 5, min(4, n), q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] == "ok" for r in res), res


def test_shard_range_partition():
    for n in (0, 1, 7, 100, 1_000_003):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[r][1] == spans[r + 1][0] for r in range(world - 1))
            sizes = [e - s for s, e in spans]
            assert max(sizes) - min(sizes) <= 1

"""Worker of tests/test_gpu_distributed.py::test_rccl_collectives: one rank of a job whose process
group is RCCL ("nccl") for device tensors and gloo for host tensors. It runs every collective the
product and bench.py issue -- all_gather_rows (index build), gather_candidates + the GPU top-k merge
(sharded search), a float64 MAX all_reduce and barrier (bench timing), broadcast_object_list
(rank-0 write status in index_build.rebuild_index) -- and writes a JSON verdict per rank.
On a 1-GPU box the job has one rank, so RCCL's init and collective entry points run without a peer;
the driver's 8-GPU node runs the same calls over xGMI."""
import json
import os
import sys

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from clip_lora_match_amd.distributed import (all_gather_rows, gather_candidates, merge_topk_gpu,  # noqa: E402
                                             shard_range)


def main(out_dir):
    local = int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist.init_process_group("cpu:gloo,cuda:nccl", device_id=dev)
    rank, world = dist.get_rank(), dist.get_world_size()
    res = {"rank": rank, "world": world, "backend": str(dist.get_backend())}
    # index build: uneven shards of 1001 rows, every rank gets all rows in global order
    n, d = 1001, 512
    g = torch.Generator(device="cpu").manual_seed(5)
    full = torch.randn((n, d), generator=g).to(dev)
    a, b = shard_range(n, rank, world)
    got = all_gather_rows(full[a:b].contiguous(), n)
    res["all_gather_rows_equal"] = bool(torch.equal(got, full))
    # sharded search: per-rank [nq, k] lists (global indices), gathered and merged on the GPU
    nq, k = 64, 10
    sc = torch.randn((world * nq, k), generator=g).sort(dim=1, descending=True).values.to(dev)
    ix = torch.randint(0, 1 << 40, (world * nq, k), generator=g).to(dev)
    s_loc, i_loc = sc[rank * nq:(rank + 1) * nq].contiguous(), ix[rank * nq:(rank + 1) * nq].contiguous()
    s_all, i_all = gather_candidates(s_loc, i_loc)
    res["gather_candidates_equal"] = bool(
        torch.equal(s_all, sc.view(world, nq, k).permute(1, 0, 2).reshape(nq, world * k))
        and torch.equal(i_all, ix.view(world, nq, k).permute(1, 0, 2).reshape(nq, world * k)))
    s_m, i_m = merge_topk_gpu(s_all, i_all, world, k)
    res["merge_sorted"] = bool((s_m[:, :-1] >= s_m[:, 1:]).all())
    # bench timing: barrier + float64 MAX all_reduce of a per-rank value on the device
    dist.barrier()
    t = torch.tensor([1.5 + rank], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    res["max_all_reduce"] = float(t.item()) == 0.5 + world
    # index_build's rank-0 status broadcast
    status = [f"ok from {rank}"]
    dist.broadcast_object_list(status, src=0)
    res["broadcast_object"] = status[0] == "ok from 0"
    # host tensors take the gloo side of the same group
    h = torch.tensor([rank], dtype=torch.int64)
    dist.all_reduce(h)
    res["host_all_reduce"] = int(h.item()) == world * (world - 1) // 2
    torch.cuda.synchronize()
    with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])

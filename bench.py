#!/usr/bin/env python
"""Benchmark: ViT-B/32 + LoRA r=8 encode of 224px images + 77-token captions
(BASELINE.json configs[1]) on N GPUs, plus an optional cosine top-k search leg
(configs[4] shape).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...)

One step = every rank encodes its own batch (default 256 images + 256 captions,
bf16 operands, LoRA merged) into L2-normalised fp32 embeddings; for N > 1 the
step ends with the index-build exchange: an RCCL all-gather of every rank's
embeddings over xGMI (scripts/rebuild_index.py builds the whole index), so per
-GPU work is fixed as N grows ("weak" scaling). Inputs are resident in HBM
before the timed region. Prints ONE JSON line on rank 0.

value = image+text pairs encoded per second over all ranks.
roofline = the MFMA GEMM kernel (dominant: ~97% of the step's FLOPs), timed
live with HIP events on its launch stream in a separate profiled pass.
cpu_baseline = transformers CLIPModel fp32 on the host cores (the arithmetic
models/clip_model.py runs) with the restated PEFT LoRA, on a bounded sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import clip_lora_match_amd as clm  # noqa: E402
from clip_lora_match_amd import synthetic as syn  # noqa: E402
from clip_lora_match_amd import weights as W  # noqa: E402
from clip_lora_match_amd.engine import ClipLoraModel  # noqa: E402

MFMA_PEAK_TFLOPS = 2500.0   # dense bf16/fp16 MFMA, MI355X (MI355X_MICROARCH.md chip table)
HBM_PEAK_GBS = 8000.0


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def pruned_last_layer() -> bool:
    """libclm runs the last layer's out_proj / LN2 / fc1 / fc2 on the pooled rows only unless
    $CLM_NO_PRUNE=1 (capi.cpp run_layers); the FLOP / byte counts below follow it."""
    return os.environ.get("CLM_NO_PRUNE", "0") in ("", "0")


def flops_per_pair(cfg, pruned=None) -> dict:
    """Algorithmic FLOPs per image / caption (2 x MAC of every GEMM + full-T^2 attention,
    LoRA unmerged), SURVEY §8(d). With the last layer pruned, its out_proj / fc1 / fc2 (and
    their LoRA) count one pooled row instead of T."""
    pruned = pruned_last_layer() if pruned is None else pruned
    r = cfg.lora_r

    def lora_tok(d, mlp, targets):   # per token and layer: x.A^T (r x fin) + (.)B^T (fout x r)
        dims = {"q_proj": (d, d), "k_proj": (d, d), "v_proj": (d, d), "out_proj": (d, d),
                "fc1": (d, mlp), "fc2": (mlp, d)}
        return sum(2 * r * (dims[t][0] + dims[t][1]) for t in cfg.lora_targets if t in dims and t in targets)

    def tower(d, L, mlp, T):
        qkv = ("q_proj", "k_proj", "v_proj")
        rest = ("out_proj", "fc1", "fc2")
        front = 2 * T * d * 3 * d + 4 * T * T * d + lora_tok(d, mlp, qkv) * T   # q/k/v + attention
        back = 2 * d * (d + 2 * mlp) + lora_tok(d, mlp, rest)                     # per row
        return L * front + (L - 1) * T * back + (1 if pruned else T) * back
    v, t = cfg.vision, cfg.text
    P = cfg.num_patches
    img = tower(v.hidden, v.layers, v.mlp, P + 1) \
        + 2 * P * (cfg.channels * cfg.patch ** 2) * v.hidden + 2 * v.hidden * cfg.proj_dim
    txt = tower(t.hidden, t.layers, t.mlp, cfg.max_pos) + 2 * t.hidden * cfg.proj_dim
    return {"image": float(img), "caption": float(txt)}


def gemm_algorithmic_bytes(cfg, B) -> float:
    """Compulsory HBM bytes of one step's GEMMs: A read once, W read once, output written once
    (fp32 residual read + written for out_proj / fc2), bf16 operands; the pruned last layer's
    out_proj / fc1 / fc2 on B rows."""
    tot = 0.0
    for tw, T in ((cfg.vision, cfg.vision_seq), (cfg.text, cfg.max_pos)):
        d, f = tw.hidden, tw.mlp

        def front(M):
            return M * d * 2 + 3 * d * d * 2 + M * 3 * d * 2                    # qkv

        def back(M):
            return (M * d * 2 + d * d * 2 + M * d * 8                            # out (+ fp32 residual RMW)
                    + M * d * 2 + f * d * 2 + M * f * 2                          # fc1
                    + M * f * 2 + d * f * 2 + M * d * 8)                         # fc2 (+ residual RMW)
        M = B * T
        tot += tw.layers * front(M) + (tw.layers - 1) * back(M) + back(B if pruned_last_layer() else M)
    P = B * cfg.num_patches
    tot += P * cfg.channels * cfg.patch ** 2 * 2 + cfg.vision.hidden * cfg.channels * cfg.patch ** 2 * 2 + \
        B * cfg.vision_seq * cfg.vision.hidden * 4
    return tot


def cpu_baseline(cfg, sd, lora, budget_s: float):
    """transformers CLIPModel fp32 on the host cores + restated PEFT LoRA (oracle/hf_ref.py)."""
    from oracle import hf_ref as H
    cores = len(os.sched_getaffinity(0))
    threads = max(1, min(cores, int(os.environ.get("OMP_NUM_THREADS", cores))))
    torch.set_num_threads(threads)
    m = H.hf_model(cfg, sd, lora)
    n = 16
    imgs = syn.images_u8(n, cfg.image_size, 777)
    ids = syn.captions(n, cfg.max_pos, cfg.bos_token_id, cfg.eos_token_id, 778)
    pv = H.pixel_values(cfg, imgs)
    H.encode(m, cfg, pv[:2], ids[:2])  # warm
    done, t0 = 0, time.perf_counter()
    while True:
        H.encode(m, cfg, pv, ids)
        done += n
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    # the reference's own call pattern: one image / one caption per call (clip_model.py:89-150)
    t1 = time.perf_counter()
    for i in range(4):
        H.encode(m, cfg, pv[i:i + 1], ids[i:i + 1])
    dt1 = time.perf_counter() - t1
    return {"value": done / dt, "unit": "pairs/s", "cores": threads, "kind": "reference",
            "sample": f"{done} image+caption pairs in batches of {n} ({dt:.1f} s), transformers "
                      f"{__import__('transformers').__version__} CLIPModel fp32 + PEFT-equivalent LoRA hooks, "
                      f"torch CPU {threads} threads; reference per-item loop (batch 1): {4 / dt1:.2f} pairs/s"}


def search_leg(rows: int, queries: int, k: int, device, world: int = 1, rank: int = 0):
    """BASELINE configs[4]: 10k fp16 queries vs a rows x 512 fp16 index in HBM, top-k.
    world > 1: the index is row-sharded (rank r holds shard_range(rows, r, world)
    with global offsets), queries are replicated, each rank searches its shard, one all_gather of
    the [nq, k] lists and the (score desc, index asc) merge on the GPU give every rank the global
    top-k. The timed region spans local search + gather + merge, max over ranks."""
    from clip_lora_match_amd.distributed import shard_range
    from clip_lora_match_amd.search import CosineIndex
    dim = 512
    start, stop = shard_range(rows, rank, world)
    idx = CosineIndex(dim, capacity=max(stop - start, 1), device=device)
    g = torch.Generator(device=device).manual_seed(7 + 1000 * rank)
    chunk = 1 << 20
    for r0 in range(start, stop, chunk):
        n = min(chunk, stop - r0)
        x = torch.randn((n, dim), generator=g, device=device)
        idx.append((x / x.norm(dim=-1, keepdim=True)).half())
        del x
    if world > 1:
        idx.set_offset(start)
        g = torch.Generator(device=device).manual_seed(8)   # replicated queries
    q = torch.randn((queries, dim), generator=g, device=device)
    q = (q / q.norm(dim=-1, keepdim=True)).half()

    def run(qq):
        s, i = idx.search(qq, k)
        if world > 1:
            from clip_lora_match_amd.distributed import gather_candidates, merge_topk_gpu
            s_all, i_all = gather_candidates(s, i)
            s, i = merge_topk_gpu(s_all, i_all, world, k)
        return s, i

    run(q[:64])
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    s, i = run(q)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=device)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t.item())
    idx.close()
    flops = 2.0 * queries * rows * dim
    out = {"qps": queries / dt, "seconds": dt, "rows": rows, "queries": queries, "k": k, "dim": dim,
           "index_dtype": "fp16", "tflops": flops / dt / 1e12}
    if world > 1:
        out.update({"n_gpus": world, "shard_rows": stop - start,
                    "parallelism": "row-sharded index, replicated queries, all_gather(top-k) + GPU merge"})
    return out


def l14_leg(device, batch: int = 128, steps: int = 3, warmup: int = 1):
    """BASELINE configs[3]: ViT-L/14@336 + LoRA r=16 on q,k,v,out,fc1,fc2 (merged), bf16, image
    tower, batch 128 (576 patches + CLS per image: the large-tile MFMA path). Synthetic weights
    and uint8 336x336 images; inputs resident in HBM; one JSON sub-object."""
    cfg = clm.get_preset("ViT-L/14@336")
    sd, lora = W.synthetic_state_dict(cfg, 0), W.synthetic_lora(cfg, 1)
    m = ClipLoraModel(cfg, device=device, compute_dtype="bfloat16", lora_mode="merged", max_batch=batch)
    m.load_tensors(sd)
    m.load_tensors(lora)
    m.finalize()
    del sd, lora
    imgs = torch.from_numpy(syn.images_u8(batch, cfg.image_size, 4321)).to(device)
    out = torch.empty((batch, cfg.proj_dim), dtype=torch.float32, device=device)
    for _ in range(warmup):
        m.encode_pixels(imgs, out=out)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        m.encode_pixels(imgs, out=out)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    m.prof_enable(True)
    m.encode_pixels(imgs, out=out)
    torch.cuda.synchronize()
    prof = m.prof_read()
    m.prof_enable(False)
    m.close()
    fp = flops_per_pair(cfg)["image"]
    g_ms, g_flops, _ = prof["gemm"]
    return {"config": "ViT-L/14@336 + LoRA r=16 (q,k,v,out,fc1,fc2) merged, bf16, batch 128, image tower",
            "images_per_s": round(batch / dt, 1), "ms_per_step": round(dt * 1e3, 3),
            "step_tflops": round(batch * fp / dt / 1e12, 1),
            "gemm_tflops": round(g_flops / (g_ms * 1e-3) / 1e12, 1),
            "kernel_ms": {k: round(v[0], 3) for k, v in prof.items()}}


def pmc_traffic():
    """HBM bytes per GEMM launch from the newest committed PMC summary (tools/pmc_summary.py),
    or None when no counter run has been recorded."""
    import glob
    files = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "*_pmc_summary.json")))
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    return d.get("gemm_mean_hbm_bytes_per_launch"), os.path.basename(files[-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--dtype", default="bfloat16", choices=["bfloat16", "float16"])
    ap.add_argument("--lora-mode", default="merged", choices=["merged", "unmerged"])
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--search-rows", type=int, default=10_000_000)
    ap.add_argument("--search-queries", type=int, default=10_000)
    ap.add_argument("--no-search", action="store_true")
    ap.add_argument("--no-l14", action="store_true", help="skip the ViT-L/14@336 (configs[3]) leg")
    ap.add_argument("--sequential", action="store_true", help="towers back to back on one stream, no graph")
    ap.add_argument("--split", type=int, default=0, help="sub-batches per tower in encode_pair (0 = library default)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # modulo: a rehearsal may put several ranks on one GPU; on a full node this is LOCAL_RANK itself
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        # RCCL over xGMI; CLM_DIST_BACKEND=gloo only to rehearse N ranks on one GPU (RCCL refuses that)
        backend = os.environ.get("CLM_DIST_BACKEND", "nccl")
        dist.init_process_group(backend, **({"device_id": dev} if backend == "nccl" else {}))

    cfg = clm.get_preset("ViT-B/32")   # LoRA r=8, alpha=16 on q,k,v,out (config/lora_config.yaml)
    sd = W.synthetic_state_dict(cfg, 0)
    lora = W.synthetic_lora(cfg, 1)
    B = args.batch
    model = ClipLoraModel(cfg, device=dev, compute_dtype=args.dtype, lora_mode=args.lora_mode, max_batch=B)
    model.load_tensors(sd)
    model.load_tensors(lora)
    model.finalize()

    imgs = torch.from_numpy(syn.images_u8(B, cfg.image_size, 1234 + rank * B)).to(dev)
    ids = torch.from_numpy(syn.captions(B, cfg.max_pos, cfg.bos_token_id, cfg.eos_token_id, 99 + rank)).to(dev)
    emb = torch.empty((2 * B, cfg.proj_dim), dtype=torch.float32, device=dev)
    profiling = [False]
    gathered = torch.empty((world * 2 * B, cfg.proj_dim), dtype=torch.float32, device=dev) if world > 1 else None

    def step():
        if args.sequential or profiling[0]:   # profiled pass: one stream, so kernel spans don't overlap
            model.encode_pixels(imgs, out=emb[:B])
            model.encode_ids(ids, out=emb[B:])
        else:   # towers concurrently on two streams, replayed from a captured hipGraph
            model.encode_pair(imgs, ids, out_img=emb[:B], out_txt=emb[B:], graph=not profiling[0],
                               split=args.split)
        if world > 1:
            torch.distributed.all_gather_into_tensor(gathered, emb)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t.item())
    ms_step = dt / args.steps * 1e3
    pairs_s = world * B / (dt / args.steps)

    # profiled pass (outside the timed region): HIP events around every kernel launch
    model.prof_enable(True)
    profiling[0] = True
    nprof = 3
    for _ in range(nprof):
        step()
    torch.cuda.synchronize()
    prof = model.prof_read()
    model.prof_enable(False)
    gemm_ms, gemm_flops, gemm_n = prof["gemm"]
    fp = flops_per_pair(cfg)
    traffic, traffic_src = pmc_traffic()
    gemm_bytes = gemm_algorithmic_bytes(cfg, B) * nprof
    step_flops = B * (fp["image"] + fp["caption"])

    result = {
        "metric": "image+text embeds/sec & cosine top-k QPS, ViT-B/32+LoRA, 1/2/4/8 MI355X",
        "value": round(pairs_s, 1),
        "unit": "image+text pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16" if args.dtype == "bfloat16" else "fp16",
        "data": "synthetic (seeded uint8 224x224 RGB images, 77-token id captions; deterministic synthetic weights)",
        "config": {"workload": "ViT-B/32 + LoRA r=8 alpha=16 (q,k,v,out, both towers) encode + L2-normalise",
                   "execution": "sequential" if args.sequential else
                       f"image / text towers concurrently on 2 HIP streams (sub-batches per tower: {args.split or 1})"
                       " + hipGraph replay",
                   "per_gpu_batch": B, "global_batch": world * B, "seq_len": cfg.max_pos,
                   "image_size": cfg.image_size, "lora_mode": args.lora_mode,
                   "parallelism": f"dp{world}" + (" + all_gather(embeddings)" if world > 1 else "")},
        "embeds_per_s": round(2 * pairs_s, 1),
        "step_tflops_per_gpu": round(step_flops / (ms_step * 1e-3) / 1e12, 2),
        "roofline": {
            "kernel": "gemm_kernel / gemm2_kernel (MFMA 16x16x32, all encoder GEMMs)",
            "bound": "mfma",
            "achieved": round(gemm_flops / (gemm_ms * 1e-3) / 1e12, 2),
            "peak": MFMA_PEAK_TFLOPS,
            "unit": "TFLOP/s",
            "frac": round(gemm_flops / (gemm_ms * 1e-3) / 1e12 / MFMA_PEAK_TFLOPS, 4),
            "traffic": traffic,
            "traffic_unit": "bytes per launch (PMC: 2*FETCH_SIZE + WRITE_SIZE, gfx950-corrected)",
            "traffic_source": traffic_src,
            "algorithmic_bytes_per_launch": round(gemm_bytes / max(gemm_n, 1)),
            "avg_launch_us": round(gemm_ms / gemm_n * 1e3, 2),
            "launches_per_step": gemm_n // nprof,
            "kernel_ms_per_step": {k: round(v[0] / nprof, 4) for k, v in prof.items()},
        },
    }
    if not args.no_search:   # every rank takes part when the index is sharded (world > 1)
        try:
            sr = search_leg(args.search_rows, args.search_queries, 5, dev, world, rank)
        except Exception as e:  # report, never hide
            sr = {"error": repr(e)}
        if rank == 0:
            result["search"] = sr
    if rank == 0 and world == 1 and not args.no_l14:
        try:
            result["l14"] = l14_leg(dev)
        except Exception as e:  # report, never hide
            result["l14"] = {"error": repr(e)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(cfg, sd, lora, args.cpu_budget)
    if rank == 0:
        print(json.dumps(result), flush=True)
    model.close()
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()

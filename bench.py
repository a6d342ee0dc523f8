#!/usr/bin/env python
"""Benchmark: ViT-B/32 + LoRA r=8 encode of 224px images + 77-token captions
(BASELINE.json configs[1]) on N GPUs, plus the cosine top-k search leg (configs[4]),
the ViT-L/14@336 leg (configs[3]) and the reference CPU path timed beside them.

  python bench.py [--gpus N] [--steps K] [--warmup W]

--gpus N > 1 without a torch.distributed launcher around it: bench.py starts its own N ranks
(python -m torch.distributed.run, 127.0.0.1) before touching the GPU and exits with their
status. On a box with fewer than N GPUs the ranks rehearse over gloo (RCCL refuses two ranks
per device) and the line says so ("rehearsal"). Every rank checks that the process group really
has N ranks.

One step = every rank encodes its own batch (default 256 images + 256 captions, bf16 operands,
LoRA merged) into L2-normalised fp32 embeddings; for N > 1 the step ends with the index-build
exchange: an RCCL all-gather of every rank's embeddings over xGMI (scripts/rebuild_index.py
builds the whole index), so per-GPU work is fixed as N grows ("weak" scaling). Inputs are
resident in HBM before the timed region. Prints ONE JSON line on rank 0.

value = image+text pairs encoded per second over all ranks.
roofline = the MFMA GEMM kernels (~97% of the step's FLOPs), from a rocprofv3 kernel trace of the
timed step's own form (a child process under rocprofv3 replaying the same two-stream hipGraph
step): achieved = GEMM FLOPs per step / time with a GEMM kernel running; `dominant` = the GEMM
kernel with the most time per step, with its FLOPs and algorithmic bytes per launch; traffic / MFMA
busy from the newest committed rocprofv3 PMC summary (tools/pmc.sh + tools/pmc_summary.py, run
with the timed step's tile configs).
dtype: "mixed" by default -- bf16 operands (BASELINE configs[1]'s wording) in the vision tower,
fp16 in the text tower, which carries the bf16 error (include/clm.h CLM_COMPUTE_MIXED): the bf16
assignment whose scores meet north_star's 1e-3 bar against the fp32 reference (the `parity` object
measures it on every run, ~6e-4). All-fp16 and all-bf16 operands are the `dtype_legs`, each with its
own parity figure (fp16 ~2.8e-4; bf16 ~1.7e-3: over the bar).
cpu_baseline = the reference's arithmetic on the host cores: transformers CLIPModel fp32 + the
restated PEFT LoRA (batched 64 and per item), and search_with_embedding's fp32 q @ E^T + topk
per single query over the fp16-upcast, re-normalised 10 M-row index (a bounded query subset).
"""
from __future__ import annotations

import argparse
import json
import os
import re
import socket
import subprocess
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import clip_lora_match_amd as clm  # noqa: E402
from clip_lora_match_amd import synthetic as syn  # noqa: E402
from clip_lora_match_amd import weights as W  # noqa: E402
from clip_lora_match_amd.engine import ClipLoraModel  # noqa: E402

MFMA_PEAK_TFLOPS = 2500.0   # dense bf16/fp16 MFMA, MI355X (MI355X_MICROARCH.md chip table)
# what the chip sustains on a pure back-to-back v_mfma_f32_16x16x32_f16 stream with random operands
# (tools/mfma_probe.hip, 256-1024 workgroups of 8 waves: 1.98-2.03 PF/s; the clock drops under
# MFMA load), profiles/r03_v10_mfma_peak_probe.jsonl; reported beside the list peak, not used for frac
MFMA_SUSTAINED_TFLOPS = 2028.0
HBM_PEAK_GBS = 8000.0
DTYPE_LABEL = {"bfloat16": "bf16", "float16": "fp16", "mixed": "bf16 (vision) + fp16 (text)"}
METRIC = "image+text embeds/sec & cosine top-k QPS, ViT-B/32+LoRA, 1/2/4/8 MI355X"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--dtype", default="mixed", choices=["bfloat16", "float16", "mixed"])
    ap.add_argument("--lora-mode", default="merged", choices=["merged", "unmerged"])
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds of CPU encode timing")
    ap.add_argument("--cpu-search-budget", type=float, default=20.0, help="seconds of CPU search timing")
    ap.add_argument("--cpu-search-queries", type=int, default=100)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--search-rows", type=int, default=10_000_000)
    ap.add_argument("--search-queries", type=int, default=10_000)
    ap.add_argument("--no-search", action="store_true")
    ap.add_argument("--no-l14", action="store_true", help="skip the ViT-L/14@336 (configs[3]) leg")
    ap.add_argument("--no-parity-mode", action="store_true", help="skip the other-dtype (bf16 / fp16) step")
    ap.add_argument("--no-varlen", action="store_true", help="skip the mixed-length caption (varlen) leg")
    ap.add_argument("--no-unmerged", action="store_true", help="skip the unmerged (hot-swappable) LoRA leg")
    ap.add_argument("--no-index-build", action="store_true", help="skip the configs[2] index-build leg")
    ap.add_argument("--index-images", type=int, default=1_000_000, help="images of the configs[2] index build")
    ap.add_argument("--index-batch", type=int, default=1280,
                    help="encode batch of the configs[2] leg (1280: profiles/r04_v8_index_batch_sweep.txt)")
    ap.add_argument("--no-persist", action="store_true", help="skip the search index shard save / load timing")
    ap.add_argument("--no-near-dup", action="store_true", help="skip the near-duplicate-rows search leg")
    ap.add_argument("--no-single", action="store_true", help="skip the one-query-per-call search leg")
    ap.add_argument("--no-encode-item", action="store_true", help="skip the per-item encode_image / encode_text leg")
    ap.add_argument("--sequential", action="store_true", help="towers back to back on one stream, no graph")
    ap.add_argument("--split", type=int, default=0, help="sub-batches per tower in encode_pair (0 = library default)")
    ap.add_argument("--no-trace", action="store_true", help="skip the rocprofv3 kernel trace of the headline step")
    ap.add_argument("--trace-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--no-graph", action="store_true", help="two tower streams without the hipGraph replay (A/B)")
    return ap.parse_args(argv)


def maybe_spawn(args) -> None:
    """--gpus N > 1 outside a launcher: run N ranks under torch.distributed.run as a child
    process and exit with its status. Nothing here touches the GPU (device_count does not
    initialise it), so the ranks start from a clean process."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return
    ndev = torch.cuda.device_count()
    env = dict(os.environ)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    if ndev < args.gpus:
        env["CLM_DIST_BACKEND"] = "gloo"
        env["CLM_REHEARSAL"] = f"{args.gpus} ranks on {ndev} GPU(s) over gloo: timings are not a scaling measurement"
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    log("bench: launching", " ".join(cmd))
    sys.exit(subprocess.call(cmd, env=env))


def pruned_last_layer() -> bool:
    """libclm runs the last layer's out_proj / LN2 / fc1 / fc2 on the pooled rows only unless
    $CLM_NO_PRUNE=1 (capi.cpp run_layers); the FLOP / byte counts below follow it."""
    return os.environ.get("CLM_NO_PRUNE", "0") in ("", "0")


def flops_per_pair(cfg, pruned=None, lora_merged=False) -> dict:
    """Algorithmic FLOPs per image / caption (2 x MAC of every GEMM + full-T^2 attention),
    SURVEY §8(d). LoRA unmerged adds its down/up products; merged LoRA costs nothing (the
    LoRA column is subtracted). With the last layer pruned, its out_proj / fc1 / fc2 (and
    their LoRA) count one pooled row instead of T."""
    pruned = pruned_last_layer() if pruned is None else pruned
    r = 0 if lora_merged else cfg.lora_r

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


def cpu_encode_baseline(cfg, sd, lora, budget_s: float):
    """transformers CLIPModel fp32 on the host cores + restated PEFT LoRA (oracle/hf_ref.py):
    the arithmetic of models/clip_model.py encode_image / encode_text. Batched 64 (BASELINE.md
    §4) for a time budget, and the reference's own per-item calls (batch 1) for 16 + 16 items."""
    from oracle import hf_ref as H
    cores = len(os.sched_getaffinity(0))
    threads = max(1, min(cores, int(os.environ.get("OMP_NUM_THREADS", cores))))
    torch.set_num_threads(threads)
    m = H.hf_model(cfg, sd, lora)
    n = 64
    imgs = syn.images_u8(n, cfg.image_size, 777)
    ids = syn.captions(n, cfg.max_pos, cfg.bos_token_id, cfg.eos_token_id, 778)
    pv = H.pixel_values(cfg, imgs)
    H.encode_images(m, pv[:2])
    H.encode_texts(m, cfg, ids[:2])
    ti = tt = 0.0
    batches = 0
    while True:
        t0 = time.perf_counter()
        H.encode_images(m, pv)
        t1 = time.perf_counter()
        H.encode_texts(m, cfg, ids)
        t2 = time.perf_counter()
        ti, tt, batches = ti + t1 - t0, tt + t2 - t1, batches + 1
        if ti + tt > budget_s:
            break
    per = 16
    t0 = time.perf_counter()
    for i in range(per):
        H.encode_images(m, pv[i:i + 1])
    t1 = time.perf_counter()
    for i in range(per):
        H.encode_texts(m, cfg, ids[i:i + 1])
    t2 = time.perf_counter()
    pi, pt = per / (t1 - t0), per / (t2 - t1)
    bi, bt = batches * n / ti, batches * n / tt
    return {"batched64": {"images_per_s": round(bi, 2), "texts_per_s": round(bt, 2),
                          "pairs_per_s": round(batches * n / (ti + tt), 2), "batches": batches,
                          "seconds": round(ti + tt, 2)},
            "per_item": {"images_per_s": round(pi, 2), "texts_per_s": round(pt, 2),
                         "pairs_per_s": round(per / (t2 - t0), 2), "calls": 2 * per},
            "threads": threads, "impl": f"transformers {__import__('transformers').__version__} CLIPModel fp32 "
                                        "+ PEFT-equivalent LoRA hooks (oracle/hf_ref.py)"}


def cpu_search_baseline(host16: torch.Tensor, queries16: torch.Tensor, k: int, max_queries: int, budget_s: float,
                        gpu_idx: torch.Tensor):
    """TextSearchIndex semantics on the host cores (search.py:36,68,93-99): the fp16 index upcast
    to fp32 and re-normalised once, then per single query q / ||q||, sims = q @ E^T, topk(k).
    Also checks the GPU's top-k for the same queries (indices equal up to fp32 near-ties)."""
    t_prep = time.perf_counter()
    E = host16.float()
    E /= E.norm(dim=-1, keepdim=True)
    t_prep = time.perf_counter() - t_prep
    done, t0 = 0, time.perf_counter()
    match = 0
    for qi in range(min(max_queries, queries16.shape[0])):
        q = queries16[qi:qi + 1].float()
        q = q / q.norm(dim=-1, keepdim=True)
        sims = q @ E.T
        vals, idx = torch.topk(sims, k, dim=-1)
        done += 1
        # parity of this query: GPU indices vs the reference's, allowing fp32 near-ties (2e-6)
        g = gpu_idx[qi]
        if torch.equal(idx[0], g):
            match += 1
        else:
            cand = torch.unique(torch.cat([idx[0], g]))
            ex = (E[cand].double() @ q[0].double())
            exd = dict(zip(cand.tolist(), ex.tolist()))
            sa = torch.tensor([exd[int(i)] for i in idx[0]])
            sb = torch.tensor([exd[int(i)] for i in g])
            if float((sa - sb).abs().max()) <= 2e-6:
                match += 1
        if time.perf_counter() - t0 > budget_s and done >= 10:
            break
    dt = time.perf_counter() - t0
    del E
    return {"qps": round(done / dt, 3), "ms_per_query": round(dt / done * 1e3, 2), "queries": done,
            "sample": f"the first {done} of {queries16.shape[0]} queries, one at a time (a {budget_s:.0f} s budget: "
                      f"SURVEY §8(d)'s 100-query subset takes ~{100 * dt / done:.0f} s here; --cpu-search-budget "
                      "raises it)",
            "rows": host16.shape[0], "k": k, "prep_s": round(t_prep, 2),
            "gpu_topk_matches_reference": f"{match}/{done}",
            "impl": "torch CPU fp32: index.float() / ||row|| once; per query q/||q||, q @ E^T, topk"}


def _topk_ordered(s: torch.Tensor, i: torch.Tensor, k: int):
    """top k of each row by (score desc, index asc): stable sort by index, then by score"""
    o = torch.argsort(i, dim=1, stable=True)
    s, i = torch.gather(s, 1, o), torch.gather(i, 1, o)
    o = torch.argsort(-s, dim=1, stable=True)[:, :k]
    return torch.gather(s, 1, o), torch.gather(i, 1, o)


def shard_roundtrip(idx, q, k) -> dict:
    """The index persisted as a raw shard (CosineIndex.save_shard: fp16 rows + fp32 inverse norms,
    streamed through a pinned buffer) and loaded back into HBM (load_shard), timed; the reloaded
    index must answer the same queries bit for bit."""
    import shutil
    import tempfile
    from clip_lora_match_amd.search import CosineIndex
    d = tempfile.mkdtemp(prefix="clm_shard_")
    try:
        path = os.path.join(d, "index.clmidx")
        s0, i0 = idx.search(q, k)
        t0 = time.perf_counter()
        idx.save_shard(path)
        t1 = time.perf_counter()
        re, _ = CosineIndex.load_shard(path, device=idx.device)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        s1, i1 = re.search(q, k)
        same = bool(torch.equal(s0, s1) and torch.equal(i0, i1))
        nbytes = os.path.getsize(path)
        re.close()
    finally:
        shutil.rmtree(d, ignore_errors=True)
    return {"bytes": nbytes, "save_s": round(t1 - t0, 3), "load_s": round(t2 - t1, 3),
            "save_gb_s": round(nbytes / (t1 - t0) / 1e9, 2), "load_gb_s": round(nbytes / (t2 - t1) / 1e9, 2),
            "reloaded_search_identical": same, "where": "a temporary file (the box's /tmp)"}


def single_query_leg(idx, q, chk_s, chk_i, k: int, calls: int = 64) -> dict:
    """The reference's own search call pattern on the configs[4] index: ONE query per call through
    the drop-in TextSearchIndex.search_with_embedding(q, 5) (search.py:93-99; SeekerService.search_items
    calls it per request, seeker_service.py:183-186), with the CPU float32 query tensor the reference's
    encode_* returns. The small batch takes the one-pass streaming search (capi.cpp search_small:
    the fp16 index read once, scan16_kernel). HBM bound: the 10 M x 512 fp16 rows + fp32 inverse
    norms per query. Also the device-level call (CosineIndex.search, device queries) and nq = 1..16
    per call, and equality with the exact fp64 scan (scores and indices) on the check queries."""
    from clip_lora_match_amd.search import TextSearchIndex
    tsi = TextSearchIndex.from_gpu_index(idx)
    n, dim = len(idx), idx.dim
    nbytes = n * dim * 2 + n * 4
    qs_cpu = q[:calls].float().cpu()
    for j in range(3):
        tsi.search_with_embedding(qs_cpu[j], k)
    torch.cuda.synchronize()
    st0 = idx.stats()
    t0 = time.perf_counter()
    res = [tsi.search_with_embedding(qs_cpu[j], k) for j in range(calls)]
    t_call = (time.perf_counter() - t0) / calls
    st1 = idx.stats()
    nchk = min(chk_i.shape[0], calls)
    ci, cs = chk_i.cpu(), chk_s.cpu()
    eq = sum(1 for j in range(nchk) if [r.index for r in res[j]] == ci[j].tolist()
             and [r.score for r in res[j]] == cs[j].tolist())
    qd = q[:calls].contiguous()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for j in range(calls):
        idx.search(qd[j:j + 1], k)
    e1.record()
    torch.cuda.synchronize()
    t_dev = e0.elapsed_time(e1) * 1e-3 / calls
    per_nq = {}
    for nq in (1, 2, 4, 8, 16):
        reps = 12
        idx.search(qd[:nq], k)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(reps):
            idx.search(qd[:nq], k)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t1) / reps
        per_nq[str(nq)] = {"ms_per_call": round(dt * 1e3, 3), "qps": round(nq / dt, 1),
                           "hbm_frac": round(nbytes / dt / (HBM_PEAK_GBS * 1e9), 4)}
    served = {key: st1[key] - st0[key] for key in st1}
    return {"ms_per_query": round(t_call * 1e3, 3), "qps": round(1.0 / t_call, 1),
            "hbm_bytes_per_query": nbytes,
            "hbm_frac": round(nbytes / t_call / (HBM_PEAK_GBS * 1e9), 4),
            "device_ms_per_query": round(t_dev * 1e3, 3),
            "device_hbm_frac": round(nbytes / t_dev / (HBM_PEAK_GBS * 1e9), 4),
            "calls": calls, "k": k, "rows": n,
            "equal_to_exact_scan": f"{eq}/{nchk}",
            "paths": served, "per_call_batch": per_nq,
            "api": "TextSearchIndex.search_with_embedding(q, 5), q a CPU float32 (512,) tensor, results as "
                   "SearchResult lists; device_*: CosineIndex.search on a device query, HIP events",
            "hbm_frac_def": "(N x 512 x 2 B fp16 rows + N x 4 B inverse norms) / time per query / 8 TB/s"}


def search_leg(rows: int, queries: int, k: int, device, world: int = 1, rank: int = 0, keep_host: bool = False,
               persist_shard: bool = False, single: bool = False):
    """BASELINE configs[4]: 10k fp16 query embeddings vs a rows x 512 fp16 index in HBM, top-k
    by exact cosine (fp16 MFMA pass + exact re-score of the candidates).
    world > 1: the index is row-sharded (rank r holds shard_range(rows, r, world)
    with global offsets), queries are replicated, each rank searches its shard, one all_gather of
    the [nq, k] lists and the (score desc, index asc) merge on the GPU give every rank the global
    top-k. The timed region spans local search + gather + merge, max over ranks.
    Every rank reports whether its shard built; all skip together if one failed (no rank is left
    waiting in a collective)."""
    from clip_lora_match_amd import _capi as C
    from clip_lora_match_amd.distributed import shard_range
    from clip_lora_match_amd.search import CosineIndex
    dim = 512
    start, stop = shard_range(rows, rank, world)
    err = None
    idx = None
    host16 = None
    nchk = min(32, queries)
    chk_s = chk_i = None
    try:
        idx = CosineIndex(dim, capacity=max(stop - start, 1), device=device)
        if world > 1:
            idx.set_offset(start)
        gq = torch.Generator(device=device).manual_seed(8)   # queries: replicated on every rank
        q = torch.randn((queries, dim), generator=gq, device=device)
        q = (q / q.norm(dim=-1, keepdim=True)).half()
        qchk = q[:nchk].float().contiguous()
        if keep_host:
            host16 = torch.empty((stop - start, dim), dtype=torch.float16)
        # rows by GLOBAL position: chunk c = rows [c * 2^20, (c + 1) * 2^20) comes from seed 7 + c, so
        # every world size searches the same index (each rank generates the chunks its shard overlaps)
        chunk = 1 << 20
        for c0 in range((start // chunk) * chunk, stop, chunk):
            g = torch.Generator(device=device).manual_seed(7 + c0 // chunk)
            x = torch.randn((min(chunk, rows - c0), dim), generator=g, device=device)
            a, b = max(start, c0) - c0, min(stop, c0 + chunk) - c0
            xh = (x[a:b] / x[a:b].norm(dim=-1, keepdim=True)).half()
            del x
            idx.append(xh)
            if host16 is not None:
                host16[c0 + a - start: c0 + b - start] = xh.cpu()
            # independent check path: exact fp64 cosines (clm_cosine_scores) of the first queries
            # against this piece, folded into a running top-k by (score desc, global index asc)
            xf = xh.float().contiguous()
            sc = torch.empty((nchk, xf.shape[0]), dtype=torch.float32, device=device)
            C.check(C.lib().clm_cosine_scores(device.index, C.ptr(qchk), nchk, C.ptr(xf), xf.shape[0], dim, C.ptr(sc),
                                              C.stream_of(device)), "clm_cosine_scores")
            ts, ti = torch.topk(sc, min(k, xf.shape[0]), dim=1)
            ti = ti + (c0 + a)
            if chk_s is not None:
                ts, ti = torch.cat([chk_s, ts], 1), torch.cat([chk_i, ti], 1)
            chk_s, chk_i = _topk_ordered(ts, ti, k)
            del xh, xf, sc
    except Exception as e:   # reported, never hidden
        err = repr(e)
    if world > 1:
        ok = torch.tensor([0 if err else 1], dtype=torch.int32, device=device)
        torch.distributed.all_reduce(ok, op=torch.distributed.ReduceOp.MIN)
        if int(ok.item()) == 0:
            return {"error": err or "another rank failed to build its shard"}, None, None, None
    elif err:
        return {"error": err}, None, None, None

    def run(qq):
        s, i = idx.search(qq, k)
        if world > 1:
            from clip_lora_match_amd.distributed import gather_candidates, merge_topk_gpu
            s_all, i_all = gather_candidates(s, i)
            s, i = merge_topk_gpu(s_all, i_all, world, k)
        return s, i

    run(q)   # untimed pass of the same shape: the index's search workspace is sized here
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
    st = idx.stats()
    persist = None
    if persist_shard and world == 1:
        persist = shard_roundtrip(idx, q[:256], k)
    # the check subset: gather every rank's exact top-k, order the union, compare with the fast path
    if world > 1:
        from clip_lora_match_amd.distributed import gather_candidates
        chk_s, chk_i = gather_candidates(chk_s.contiguous(), chk_i.contiguous())
    chk_s, chk_i = _topk_ordered(chk_s, chk_i, k)
    single_res = None
    if single and world == 1:
        try:
            single_res = single_query_leg(idx, q, chk_s, chk_i, k)
        except Exception as e:   # reported, never hidden
            single_res = {"error": repr(e)}
    idx.close()
    match = int((torch.eq(chk_i, i[:nchk]).all(1) & torch.eq(chk_s, s[:nchk]).all(1)).sum())
    import hashlib
    flops = 2.0 * queries * rows * dim
    out = {"qps": round(queries / dt, 1), "seconds": round(dt, 4), "rows": rows, "queries": queries, "k": k,
           "dim": dim, "index_dtype": "fp16", "tflops": round(flops / dt / 1e12, 1),
           "scores": "exact cosine (fp16 MFMA candidate pass + fp64 re-score), order (score desc, index asc)",
           "paths": st,
           "check": {"queries": nchk, "match": f"{match}/{nchk}",
                     "method": "first queries re-scored exactly (fp64 clm_cosine_scores) against every row, "
                               "per-rank top-k gathered and ordered (score desc, index asc): indices and scores equal"},
           "rows_seeded": "by global row (2^20-row chunks, seed 7 + chunk): the same index at every world size",
           "topk_sha256": hashlib.sha256(i.cpu().numpy().tobytes()).hexdigest()[:16]}
    if persist is not None:
        out["persist"] = persist
    if single_res is not None:
        out["single"] = single_res
    if world > 1:
        out.update({"n_gpus": world, "shard_rows": stop - start,
                    "parallelism": "row-sharded index, replicated queries, all_gather(top-k) + GPU merge"})
    return out, host16, q.cpu(), i.cpu()


def near_dup_search_leg(device, rows: int = 1_000_000, groups: int = 64, group_rows: int = 8192,
                        queries: int = 1024, k: int = 5):
    """Search over near-duplicate rows (a finder index built from one description
    template puts thousands of rows inside the candidate window): `groups` tie groups of
    `group_rows` rows (center + 1e-3 noise) spread through `rows` Gaussian rows, queries at the
    group centers plus random ones. Every query near a center overflows its candidate list
    (> 2048 candidates); an overflowed list of up to 8192 / k chunks of 4,096 is rebuilt whole by a
    second filter pass over just those queries and re-scored chunk-wise (rescore_wide + topk_merge);
    only longer lists go through the exact scan, all of them in one scan. Reports QPS, the path
    counts (`overflow`: sampled / exact / overflowed queries) and whether the result equals the full
    exact scan of every query (CLM_SEARCH_FULL, untimed)."""
    from clip_lora_match_amd.search import CosineIndex
    dim = 512
    g = torch.Generator(device=device).manual_seed(91)
    x = torch.randn((rows, dim), generator=g, device=device)
    centers = torch.randn((groups, dim), generator=g, device=device)
    stride = rows // groups
    for j in range(groups):
        a = j * stride
        x[a:a + group_rows] = centers[j] + 1e-3 * torch.randn((group_rows, dim), generator=g, device=device)
    x = (x / x.norm(dim=-1, keepdim=True)).half()
    idx = CosineIndex(dim, capacity=rows, device=device)
    idx.append(x)
    del x
    nc = groups * max((queries - 64) // groups, 0)   # center queries; the last >= 64 are random
    q = torch.cat([centers.repeat(max(nc // groups, 1), 1)[:nc],
                   torch.randn((queries - nc, dim), generator=g, device=device)])
    q = (q / q.norm(dim=-1, keepdim=True)).half()
    idx.search(q, k)   # untimed: workspace sizing
    torch.cuda.synchronize()
    before = idx.stats()
    t0 = time.perf_counter()
    s, i = idx.search(q, k)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    after = idx.stats()
    os.environ["CLM_SEARCH_FULL"] = "1"
    try:
        s_ref, i_ref = idx.search(q, k)
    finally:
        os.environ.pop("CLM_SEARCH_FULL", None)
    idx.close()
    return {"qps": round(queries / dt, 1), "seconds": round(dt, 4), "rows": rows, "queries": queries, "k": k,
            "tie_groups": groups, "group_rows": group_rows,
            "paths_timed_block": {key: after[key] - before.get(key, 0) for key in after},
            "equal_to_full_exact_scan": bool(torch.equal(i, i_ref) and torch.equal(s, s_ref))}


def encode_item_leg(device, dtype: str, calls: int = 32) -> dict:
    """The reference's per-item API (models/clip_model.py:89-150; embed_image / embed_text call it per
    item): encode_image(path) on a 640 x 480 JPEG (host decode with PIL, GPU bicubic resize + centre
    crop, batch-1 encode, CPU float32 result) and encode_text(str) (host BPE tokenizer -- the committed
    fixture vocabulary, no CLIP vocab ships here -- batch-1 encode), through load_clip_model with the
    synthetic B/32 weights and LoRA r=8 on q,k,v,out. Also the GPU encode alone at batch 1 on resident
    pixels / ids, so the host share (decode, tokenize, copies) is visible."""
    import shutil
    import tempfile
    import yaml
    from PIL import Image
    from clip_lora_match_amd.clip_model import encode_image, encode_text, load_clip_model
    d = tempfile.mkdtemp(prefix="clm_item_")
    try:
        cfgp = os.path.join(d, "clip_config.yaml")
        with open(cfgp, "w") as f:
            yaml.safe_dump({"model": {"name": "openai/clip-vit-base-patch32", "device": "cuda",
                                      "tokenizer_dir": os.path.join(REPO, "tests", "golden", "clip_bpe")},
                            "preprocess": {"image_size": 224}}, f)
        import contextlib
        with contextlib.redirect_stdout(sys.stderr):   # the loader's progress prints: stdout is the JSON line
            model, proc, dv = load_clip_model(cfgp, use_lora=True, lora_weights_path="synthetic",
                                              weights_dir="synthetic", max_batch=1, compute_dtype=dtype)
        paths = []
        for i in range(4):
            p = os.path.join(d, f"item{i}.jpg")
            Image.fromarray(syn.images_u8(1, 480, 300 + i)[0]).resize((640, 480)).save(p, quality=90)
            paths.append(p)
        caps = ["a black leather wallet with a student card", "blue umbrella left near the library entrance",
                "dompet hitam ditemukan di kantin", "silver laptop charger with a frayed cable"]
        for j in range(4):
            encode_image(paths[j], model, proc, dv)
            encode_text(caps[j], model, proc, dv)
        t0 = time.perf_counter()
        for j in range(calls):
            encode_image(paths[j % 4], model, proc, dv)
        t1 = time.perf_counter()
        for j in range(calls):
            encode_text(caps[j % 4], model, proc, dv)
        t2 = time.perf_counter()
        px = proc.images_u8([paths[0]], dv)
        ids = proc.token_ids([caps[0]]).to(dv)
        for _ in range(3):
            model.encode_pixels(px)
            model.encode_ids(ids)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        for _ in range(calls):
            model.encode_pixels(px)
            torch.cuda.synchronize()
        t4 = time.perf_counter()
        for _ in range(calls):
            model.encode_ids(ids)
            torch.cuda.synchronize()
        t5 = time.perf_counter()
        model.close()
    finally:
        shutil.rmtree(d, ignore_errors=True)
    ms = lambda a, b: round((b - a) / calls * 1e3, 3)   # noqa: E731
    return {"encode_image_ms": ms(t0, t1), "encode_text_ms": ms(t1, t2),
            "gpu_encode_image_ms": ms(t3, t4), "gpu_encode_text_ms": ms(t4, t5),
            "images_per_s": round(calls / (t1 - t0), 1), "texts_per_s": round(calls / (t2 - t1), 1),
            "calls": calls, "dtype": DTYPE_LABEL.get(dtype, dtype), "text_tokens": int(ids.shape[1]),
            "api": "clip_model.encode_image(path) / encode_text(str), one item per call (CPU float32 out); "
                   "gpu_*: ClipLoraModel.encode_pixels / encode_ids at batch 1 on resident inputs, synchronised",
            "image": "640 x 480 JPEG (quality 90), shortest-edge 224 bicubic + centre crop on the GPU"}


def l14_leg(device, batch: int = 128, steps: int = 3, warmup: int = 1, dtype: str = "float16"):
    """BASELINE configs[3]: ViT-L/14@336 + LoRA r=16 on q,k,v,out,fc1,fc2 (merged), bf16, image
    tower, batch 128 (576 patches + CLS per image: the large-tile MFMA path). Synthetic weights
    and uint8 336x336 images; inputs resident in HBM; one JSON sub-object."""
    cfg = clm.get_preset("ViT-L/14@336")
    sd, lora = W.synthetic_state_dict(cfg, 0), W.synthetic_lora(cfg, 1)
    m = ClipLoraModel(cfg, device=device, compute_dtype=dtype, lora_mode="merged", max_batch=batch)
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
    fp = flops_per_pair(cfg, lora_merged=True)["image"]
    g_ms, g_flops, _ = prof["gemm"]
    a_ms, a_flops, _ = prof["attn"]
    return {"config": f"ViT-L/14@336 + LoRA r=16 (q,k,v,out,fc1,fc2) merged, "
                      f"{'bf16' if dtype in ('bfloat16', 'mixed') else 'fp16'} (the image tower's operands), batch 128",
            "images_per_s": round(batch / dt, 1), "ms_per_step": round(dt * 1e3, 3),
            "step_tflops": round(batch * fp / dt / 1e12, 1),
            "gemm_tflops": round(g_flops / (g_ms * 1e-3) / 1e12, 1),
            "attn_tflops": round(a_flops / (a_ms * 1e-3) / 1e12, 1),
            "kernel_ms": {k: round(v[0], 3) for k, v in prof.items()}}


def newest_profile(pattern: str):
    """The newest committed summary matching profiles/r<round>_v<version>_<pattern>, ordered by
    (round, version) numerically (a lexicographic sort would put v9 after v11)."""
    import glob
    best, key = None, None
    for f in glob.glob(os.path.join(REPO, "profiles", f"*_{pattern}")):
        m = re.fullmatch(r"r(\d+)_v(\d+)_" + re.escape(pattern), os.path.basename(f))
        if not m:   # e.g. r05_v5_attn_pmc_summary.json is not a "pmc_summary.json"
            continue
        kk = (int(m.group(1)), int(m.group(2)))
        if key is None or kk > key:
            best, key = f, kk
    return best


def pmc_summary():
    f = newest_profile("pmc_summary.json")
    if not f:
        return {}, None
    return json.load(open(f)), os.path.basename(f)


def gemm_launch_table(cfg, B: int) -> dict:
    """The GEMM launches of one encode_pair step in launch order per tower, as the library issues
    them (capi.cpp run_layers, fused q/k/v + attention, pruned last layer, merged LoRA):
    [(label, FLOPs, algorithmic HBM bytes)]. FLOPs: 2 x MAC (+ full-T^2 attention inside the fused
    q/k/v kernel); bytes: A + W read once, output written once (fp32 residual read +
    written for the RESID GEMMs; the fused kernel writes only O), 2-byte operands."""
    out = {}
    for name, tw, T in (("vision", cfg.vision, cfg.vision_seq), ("text", cfg.text, cfg.max_pos)):
        d, f, L = tw.hidden, tw.mlp, tw.layers
        M = B * T
        seq = []
        if name == "vision":
            Kp = cfg.channels * cfg.patch ** 2
            P = B * cfg.num_patches
            seq.append(("patch", 2.0 * P * d * Kp, P * Kp * 2 + d * Kp * 2 + P * d * 4))

        def layer(rows_back):
            return [("qkv_attn", 2.0 * M * 3 * d * d + 4.0 * B * T * T * d, M * d * 2 + 3 * d * d * 2 + M * d * 2),
                    ("out", 2.0 * rows_back * d * d, rows_back * d * 2 + d * d * 2 + rows_back * d * 8),
                    ("fc1", 2.0 * rows_back * f * d, rows_back * d * 2 + f * d * 2 + rows_back * f * 2),
                    ("fc2", 2.0 * rows_back * d * f, rows_back * f * 2 + d * f * 2 + rows_back * d * 8)]
        for _ in range(L - 1):
            seq += layer(M)
        last = layer(B if pruned_last_layer() else M)
        seq += [(lab + (".pooled" if lab != "qkv_attn" and pruned_last_layer() else ""), fl, by) for lab, fl, by in last]
        out[name] = seq
    return out


def _short_kernel(n: str) -> str:
    n = n.replace("clm::(anonymous namespace)::", "").replace("clm::", "").replace("void ", "")
    return re.sub(r"\(.*", "", n)


def parse_step_trace(csv_path: str, cfg, B: int, steps: int) -> dict:
    """Per-kernel durations of the TIMED step's form (both towers concurrently on two streams,
    hipGraph replay) from a rocprofv3 kernel trace: the towers' queues are told apart by their
    first kernel (patchify / text_lens), each queue is cut into steps there, the last `steps`
    steps are kept, and every GEMM launch is matched (by order) to gemm_launch_table for its
    FLOPs and bytes. Returns the GEMM family table, the dominant kernel, the union of GEMM busy
    time per step (<= the step span) and the step span itself."""
    import csv
    import statistics
    rows = list(csv.DictReader(open(csv_path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    queues = {}
    for r in rows:
        queues.setdefault(r["Queue_Id"], []).append(r)
    starters = {"vision": "patchify_fast_kernel", "text": "text_lens_kernel"}
    tower_q = {}
    for tower, key in starters.items():
        for qid, rs in queues.items():
            if any(key in r["Kernel_Name"] for r in rs):
                tower_q[tower] = qid
    if set(tower_q) != {"vision", "text"} or tower_q["vision"] == tower_q["text"]:
        raise RuntimeError(f"trace: tower queues not found ({tower_q})")
    table = gemm_launch_table(cfg, B)
    per_tower_steps = {}
    for tower, qid in tower_q.items():
        cur, st = None, []
        for r in queues[qid]:
            if starters[tower] in r["Kernel_Name"]:
                cur = []
                st.append(cur)
            if cur is not None:
                cur.append(r)
        per_tower_steps[tower] = st[-steps:]
    n = min(len(v) for v in per_tower_steps.values())
    fam, spans, busy, matched = {}, [], [], True
    for j in range(n):
        ivs, t0, t1 = [], None, None
        for tower in ("vision", "text"):
            ks = per_tower_steps[tower][-n + j]
            t0 = min([int(k["Start_Timestamp"]) for k in ks] + ([t0] if t0 is not None else []))
            t1 = max([int(k["End_Timestamp"]) for k in ks] + ([t1] if t1 is not None else []))
            gk = [k for k in ks if "gemm" in k["Kernel_Name"]]
            tab = table[tower]
            ok = len(gk) == len(tab)
            matched &= ok
            for i, k in enumerate(gk):
                a, b = int(k["Start_Timestamp"]), int(k["End_Timestamp"])
                ivs.append((a, b))
                name = _short_kernel(k["Kernel_Name"])
                lab, fl, by = tab[i] if ok else ("?", None, None)
                e = fam.setdefault(name, {"kernel": name, "launches": 0, "ns": 0, "flops": 0.0, "bytes": 0.0,
                                          "labels": set(), "towers": set()})
                e["launches"] += 1
                e["ns"] += b - a
                e["flops"] += fl or 0.0
                e["bytes"] += by or 0.0
                e["labels"].add(lab)
                e["towers"].add(tower)
        spans.append((t1 - t0) / 1e3)
        ivs.sort()
        u, cs, ce = 0, None, None
        for a, b in ivs:
            if ce is None or a > ce:
                if ce is not None:
                    u += ce - cs
                cs, ce = a, b
            else:
                ce = max(ce, b)
        if ce is not None:
            u += ce - cs
        busy.append(u / 1e3)
    fams = []
    for e in fam.values():
        us = e["ns"] / 1e3 / e["launches"]
        fl = e["flops"] / e["launches"] if matched else None
        by = e["bytes"] / e["launches"] if matched else None
        fams.append({"kernel": e["kernel"], "launches_per_step": e["launches"] // max(n, 1), "avg_us": round(us, 2),
                     "ms_per_step": round(e["ns"] / 1e6 / max(n, 1), 4), "labels": sorted(e["labels"]),
                     "towers": sorted(e["towers"]),
                     "flops_per_launch": fl, "tflops": round(fl / (us * 1e-6) / 1e12, 1) if fl else None,
                     "frac": round(fl / (us * 1e-6) / 1e12 / MFMA_PEAK_TFLOPS, 4) if fl else None,
                     "alg_bytes_per_launch": by,
                     "hbm_frac": round(by / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4) if by else None})
    fams.sort(key=lambda x: -x["ms_per_step"])
    step_gemm_flops = sum(fl for t in table.values() for _, fl, _ in t)
    med_busy, med_span = statistics.median(busy), statistics.median(spans)
    return {"steps": n, "matched_launch_table": matched, "step_span_ms": round(med_span / 1e3, 4),
            "gemm_busy_ms_per_step": round(med_busy / 1e3, 4),
            "gemm_kernel_ms_per_step_sum": round(sum(f["ms_per_step"] for f in fams), 4),
            "gemm_flops_per_step": step_gemm_flops,
            "gemm_tflops_over_busy": round(step_gemm_flops / (med_busy * 1e-6) / 1e12, 1),
            "families": fams}


def step_trace_leg(args, cfg) -> dict:
    """rocprofv3 --kernel-trace of the headline step itself: bench.py --trace-child runs the same
    model, batch, dtype and concurrent hipGraph step (warmup + steps) in a child process under
    rocprofv3 (the program right after `--`), and parse_step_trace reads the per-kernel durations.
    The roofline's `achieved` / `frac` and `dominant` come from this trace, not from a separate
    sequential pass."""
    import shutil
    import tempfile
    prof = shutil.which("rocprofv3")
    if not prof:
        return {"error": "rocprofv3 not found"}
    d = tempfile.mkdtemp(prefix="clm_trace_")
    steps = max(3, min(args.steps, 10))
    cmd = [prof, "--kernel-trace", "--stats", "--output-format", "csv", "-d", d, "-o", "trace", "--",
           sys.executable, os.path.abspath(__file__), "--trace-child", "--steps", str(steps), "--warmup", "2",
           "--batch", str(args.batch), "--dtype", args.dtype, "--lora-mode", args.lora_mode]
    try:
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=dict(os.environ, TMPDIR="/tmp"))
        if p.returncode != 0:
            return {"error": f"rocprofv3 rc={p.returncode}: {p.stderr[-600:]}"}
        import glob
        kt = glob.glob(os.path.join(d, "**", "trace_kernel_trace.csv"), recursive=True)
        ks = glob.glob(os.path.join(d, "**", "trace_kernel_stats.csv"), recursive=True)
        if not kt:
            return {"error": "no kernel trace written"}
        res = parse_step_trace(kt[0], cfg, args.batch, steps)
        res["command"] = "rocprofv3 --kernel-trace --stats -- python bench.py --trace-child " + \
            f"--steps {steps} --warmup 2 --batch {args.batch} --dtype {args.dtype}"
        keep = os.environ.get("CLM_TRACE_KEEP")   # copy the raw CSVs out (e.g. into gpurun_out/)
        if keep:
            os.makedirs(keep, exist_ok=True)
            for f in kt + ks:
                shutil.copy(f, keep)
        return res
    finally:
        shutil.rmtree(d, ignore_errors=True)


def trace_child(args) -> None:
    """The traced process: the headline step only (model, inputs and graph exactly as main())."""
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = clm.get_preset("ViT-B/32")
    B = args.batch
    model = ClipLoraModel(cfg, device=dev, compute_dtype=args.dtype, lora_mode=args.lora_mode, max_batch=B)
    model.load_tensors(W.synthetic_state_dict(cfg, 0))
    model.load_tensors(W.synthetic_lora(cfg, 1))
    model.finalize()
    imgs = torch.from_numpy(syn.images_u8(B, cfg.image_size, 1234)).to(dev)
    ids = torch.from_numpy(syn.captions(B, cfg.max_pos, cfg.bos_token_id, cfg.eos_token_id, 99,
                                        min_len=cfg.max_pos)).to(dev)
    emb = torch.empty((2 * B, cfg.proj_dim), dtype=torch.float32, device=dev)
    for _ in range(args.warmup + args.steps):
        model.encode_pair(imgs, ids, out_img=emb[:B], out_txt=emb[B:], graph=True, split=args.split)
    torch.cuda.synchronize()
    model.close()


def varlen_leg(model, cfg, dev, B, imgs, steps, warmup, rank=0):
    """Mixed-length captions (lengths uniform in [8, 77], padded to 77 with EOS as the CLIP
    tokenizer pads): the library's default varlen text path encodes each caption's live rows only
    (through its first EOS; causal tower, bit-identical embeddings, tests/test_gpu_encode.py::
    test_text_varlen_bit_identical) vs every padded row (clm_debug_set bit 32). Not the headline:
    the headline captions are full 77-token ones, where every row is live."""
    from clip_lora_match_amd import _capi as C
    ids = torch.from_numpy(syn.captions(B, cfg.max_pos, cfg.bos_token_id, cfg.eos_token_id, 4242 + rank)).to(dev)
    live = int(sum(min(int((r == cfg.eos_token_id).nonzero()[0]) + 1, cfg.max_pos) for r in ids.cpu()))
    oi = torch.empty((B, cfg.proj_dim), dtype=torch.float32, device=dev)
    ot = torch.empty_like(oi)
    res = {}
    try:
        for name, flag in (("varlen", 0), ("padded", 32)):
            C.lib().clm_debug_set(flag)
            for _ in range(warmup):
                model.encode_pair(imgs, ids, out_img=oi, out_txt=ot, graph=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                model.encode_pair(imgs, ids, out_img=oi, out_txt=ot, graph=True)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / steps
            res[name] = {"value": round(B / dt, 1), "ms_per_step": round(dt * 1e3, 4)}
    finally:
        C.lib().clm_debug_set(0)
    return {"unit": "image+text pairs/s", "captions": "lengths uniform in [8, 77], padded to 77",
            "live_text_rows": live, "padded_text_rows": B * cfg.max_pos, **res,
            "note": "varlen = each caption's rows through its first EOS (the pooled row) only; same embeddings"}


def other_dtype_leg(cfg, sd, lora, dev, B, imgs, ids, steps, warmup, lora_mode, dtype):
    """The same encode step with the other 16-bit operand type, and its parity against the goldens."""
    m = ClipLoraModel(cfg, device=dev, compute_dtype=dtype, lora_mode=lora_mode, max_batch=B)
    m.load_tensors(sd)
    m.load_tensors(lora)
    m.finalize()
    oi = torch.empty((B, cfg.proj_dim), dtype=torch.float32, device=dev)
    ot = torch.empty_like(oi)
    for _ in range(warmup):
        m.encode_pair(imgs, ids, out_img=oi, out_txt=ot, graph=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        m.encode_pair(imgs, ids, out_img=oi, out_txt=ot, graph=True)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    par = parity_vs_golden(m, cfg, dev)
    m.close()
    name = {"bfloat16": "bf16", "float16": "fp16", "mixed": "mixed (bf16 vision tower, fp16 text tower)"}[dtype]
    return {"dtype": name, "value": round(B / dt, 1), "unit": "image+text pairs/s",
            "ms_per_step": round(dt * 1e3, 4), "parity": {k: par[k] for k in ("max_score_err", "max_one_minus_cos")},
            "note": "16-bit GEMM / attention operands, fp32 accumulate, residual stream, LayerNorm and softmax"}


def parity_vs_golden(model, cfg, dev) -> dict:
    """The timed model's error against the transformers fp32 goldens (tests/golden/enc_b32_lora_64.npz:
    CLIPModel + LoRA hooks on 64 seeded 224^2 images + 64 full captions, B/32 synthetic weights),
    computed outside the timed region: the max |score| error over the whole 128 x 128 matrix
    (img.img, img.txt, txt.txt) and the max 1 - cos per embedding."""
    g = np.load(os.path.join(REPO, "tests", "golden", "enc_b32_lora_64.npz"), allow_pickle=False)
    imgs = torch.from_numpy(syn.images_u8(int(g["n_img"]), cfg.image_size, int(g["img_seed"]))).to(dev)
    ids = torch.from_numpy(g["ids"]).to(dev)
    a = torch.cat([model.encode_pixels(imgs), model.encode_ids(ids)]).double().cpu().numpy()
    b = np.concatenate([g["emb_img"], g["emb_txt"]]).astype(np.float64)
    cos = np.sum(a * b, 1) / (np.linalg.norm(a, axis=1) * np.linalg.norm(b, axis=1))
    return {"max_score_err": float(np.abs(a @ a.T - b @ b.T).max()), "max_one_minus_cos": float(np.max(1 - cos)),
            "bar": {"score": 1e-3, "source": "north_star: cosine scores within 1e-3"},
            "reference": "transformers CLIPModel fp32 + LoRA hooks (tests/golden/enc_b32_lora_64.npz: 64 images + "
                         "64 captions, B/32 + LoRA r=8)"}


def lora_unmerged_leg(cfg, sd, lora, dev, B, imgs, ids, steps, warmup, dtype):
    """The same step with the LoRA adapters kept unmerged (hot-swappable, models/clip_model.py:65-79):
    the K-extension mode, Y = [X | X A^T] . [W | (alpha/r) B]^T, the down-projection X A^T written into
    the activation's extension columns by a skinny MFMA GEMM (64 x 64 tiles, GEMM config 12) per LoRA'd
    input (q/k/v after LN1, out_proj after attention; capi.cpp lora_down_gemm)."""
    m = ClipLoraModel(cfg, device=dev, compute_dtype=dtype, lora_mode="unmerged", max_batch=B)
    m.load_tensors(sd)
    m.load_tensors(lora)
    m.finalize()
    oi = torch.empty((B, cfg.proj_dim), dtype=torch.float32, device=dev)
    ot = torch.empty_like(oi)
    for _ in range(warmup):
        m.encode_pair(imgs, ids, out_img=oi, out_txt=ot, graph=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        m.encode_pair(imgs, ids, out_img=oi, out_txt=ot, graph=True)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    m.close()
    return {"lora_mode": "unmerged (K-extension)", "value": round(B / dt, 1), "unit": "image+text pairs/s",
            "ms_per_step": round(dt * 1e3, 4)}


# configs[2]'s all_gather form: fp32 rows as encoded (the reference's .pt content; 2.05 GB for 1 M x
# 512 at N > 1). The fp16 exchange (half the link bytes, rows re-normalised after the
# gather) is reported beside it as a variant: its all_gather time and how far it moves the rows.
EXCHANGE = "fp32"


def index_build_leg(dev, world: int, rank: int, n_images: int, batch: int, dtype: str) -> dict:
    """BASELINE configs[2] (scripts/rebuild_index.py:64-96 over images, batch-sharded): the product's
    index_build.encode_items over n_images synthetic 224^2 images generated on the device batch by
    batch (synthetic.DeviceImages: pixels a function of the global row, so every world size builds
    the same index), B/32 + LoRA merged; rank r encodes shard_range(n, r, world) and one all_gather
    (RCCL over xGMI at N > 1) gives every rank the index; rank 0 then writes the reference's .pt.
    Timed end to end (max over ranks): generate + encode + re-normalise + all_gather, and the .pt
    write. The all_gather alone is timed again afterwards on the same rows."""
    import shutil
    import tempfile
    from clip_lora_match_amd.distributed import all_gather_rows, shard_range
    from clip_lora_match_amd.index_build import _f16_exchange, _f16_restore, _save_index, encode_items, fold_sha256
    from clip_lora_match_amd.processor import ClipProcessor
    cfg = clm.get_preset("ViT-B/32")
    m = ClipLoraModel(cfg, device=dev, compute_dtype=dtype, lora_mode="merged", max_batch=batch)
    m.load_tensors(W.synthetic_state_dict(cfg, 0))
    m.load_tensors(W.synthetic_lora(cfg, 1))
    m.finalize()
    proc = ClipProcessor(cfg)
    src = syn.DeviceImages(n_images, cfg.image_size, seed=20240, device=dev)
    m.encode_pixels(src.batch(0, min(batch, n_images)))   # untimed warm-up
    names = [f"synthetic/{i:07d}.png" for i in range(n_images)]
    texts = [""] * n_images

    def sync():
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()

    def max_over_ranks(v: float) -> float:
        if world == 1:
            return v
        t = torch.tensor([v], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        return float(t.item())

    tmpdir = tempfile.mkdtemp(prefix="clm_index_") if rank == 0 else None
    try:
        sync()
        t0 = time.perf_counter()
        rows = encode_items(m, proc, images=src, batch_size=batch, exchange=EXCHANGE)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        if rank == 0:
            _save_index(rows.cpu(), texts, names, os.path.join(tmpdir, "index.pt"))
        sync()
        t2 = time.perf_counter()
        enc_s, total_s = max_over_ranks(t1 - t0), max_over_ranks(t2 - t0)
        gather_ms = {}
        if world > 1:
            a, b = shard_range(n_images, rank, world)
            for ex, dt in (("fp32", torch.float32), ("fp16", torch.float16)):
                local = rows[a:b].to(dt).contiguous()
                sync()
                tg = time.perf_counter()
                all_gather_rows(local, n_images)
                torch.cuda.synchronize()
                gather_ms[ex] = round(max_over_ranks(time.perf_counter() - tg) * 1e3, 3)
        sha = fold_sha256(rows)   # checksum of checksums of every row's bits
        # the fp16-exchange variant's rows (what every rank would keep): their distance from these
        r16 = _f16_restore(_f16_exchange(rows))
        f16_var = {"max_abs_component_diff": float((r16 - rows).abs().max()),
                   "max_1_minus_cos": float((1 - (r16.double() * rows.double()).sum(1)).max()),
                   "index_fold_sha256": fold_sha256(r16)}
        del r16
        pt_bytes = os.path.getsize(os.path.join(tmpdir, "index.pt")) if rank == 0 else None
    finally:
        m.close()
        if tmpdir:
            shutil.rmtree(tmpdir, ignore_errors=True)
    flops = n_images * flops_per_pair(cfg, lora_merged=True)["image"]
    out = {"config": "configs[2]: ViT-B/32 + LoRA r=8 index build over synthetic 224^2 images "
                     "(index_build.encode_items + rank 0's .pt write)",
           "images": n_images, "batch": batch, "dtype": DTYPE_LABEL[dtype],
           "images_per_s": round(n_images / total_s, 1), "seconds": round(total_s, 3),
           "encode_images_per_s": round(n_images / enc_s, 1), "encode_gather_s": round(enc_s, 3),
           "write_s": round(total_s - enc_s, 3), "pt_bytes": pt_bytes,
           "tflops": round(flops / enc_s / 1e12, 1), "index_fold_sha256": sha, "exchange": EXCHANGE,
           "fp16_exchange_variant": f16_var,
           "note": "index_fold_sha256 is equal at every world size when the sharded build is bit-identical "
                   "(tests/test_gpu_distributed.py builds the same 1 M rows and prints its world-1 fold); "
                   "fp16_exchange_variant: the same rows rounded to fp16 for the all_gather and re-normalised "
                   "in fp32 after it (index_build exchange='fp16'), compared with the fp32 rows"}
    if world > 1:
        out.update({"n_gpus": world, "all_gather_ms": gather_ms.get(EXCHANGE),
                    "all_gather_ms_fp16_variant": gather_ms.get("fp16"),
                    "all_gather_bytes": n_images * cfg.proj_dim * 4,
                    "parallelism": f"batch-sharded encode + all_gather({EXCHANGE} embeddings) over xGMI"})
    return out


def main():
    args = parse_args()
    if args.trace_child:
        trace_child(args)
        return
    maybe_spawn(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus} but the launcher started {world} rank(s)")
    # modulo: a rehearsal may put several ranks on one GPU; on a full node this is LOCAL_RANK itself
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    backend = None
    if world > 1:
        import torch.distributed as dist
        # RCCL over xGMI; CLM_DIST_BACKEND=gloo only to rehearse N ranks on fewer GPUs
        backend = os.environ.get("CLM_DIST_BACKEND", "nccl")
        dist.init_process_group(backend, **({"device_id": dev} if backend == "nccl" else {}))
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"process group has {dist.get_world_size()} ranks, --gpus {args.gpus}")

    cfg = clm.get_preset("ViT-B/32")   # LoRA r=8, alpha=16 on q,k,v,out (config/lora_config.yaml)
    sd = W.synthetic_state_dict(cfg, 0)
    lora = W.synthetic_lora(cfg, 1)
    B = args.batch
    model = ClipLoraModel(cfg, device=dev, compute_dtype=args.dtype, lora_mode=args.lora_mode, max_batch=B)
    model.load_tensors(sd)
    model.load_tensors(lora)
    model.finalize()

    imgs = torch.from_numpy(syn.images_u8(B, cfg.image_size, 1234 + rank * B)).to(dev)
    # full 77-token captions (every row live): the headline workload is the same with or without
    # the varlen text path; mixed lengths are the separate `varlen_text` leg
    ids = torch.from_numpy(syn.captions(B, cfg.max_pos, cfg.bos_token_id, cfg.eos_token_id, 99 + rank,
                                        min_len=cfg.max_pos)).to(dev)
    emb = torch.empty((2 * B, cfg.proj_dim), dtype=torch.float32, device=dev)
    profiling = [False]
    gathered = torch.empty((world * 2 * B, cfg.proj_dim), dtype=torch.float32, device=dev) if world > 1 else None

    def step():
        if args.sequential or profiling[0]:   # profiled pass: one stream, so kernel spans don't overlap
            model.encode_pixels(imgs, out=emb[:B])
            model.encode_ids(ids, out=emb[B:])
        else:   # towers concurrently on two streams, replayed from a captured hipGraph
            model.encode_pair(imgs, ids, out_img=emb[:B], out_txt=emb[B:], graph=not args.no_graph, split=args.split)
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
    fp = flops_per_pair(cfg, lora_merged=args.lora_mode == "merged")
    pmc, pmc_src = pmc_summary()
    gemm_bytes = gemm_algorithmic_bytes(cfg, B) * nprof
    step_flops = B * (fp["image"] + fp["caption"])
    trace = None
    if world == 1 and not args.no_trace and not args.sequential:
        try:
            trace = step_trace_leg(args, cfg)
        except Exception as e:  # report, never hide
            trace = {"error": repr(e)}
    seq_tf = gemm_flops / (gemm_ms * 1e-3) / 1e12
    traced = trace is not None and "error" not in trace and trace.get("matched_launch_table")
    if traced:
        # the traced replay runs slower than the timed one (profiler overhead): the GEMM share of the
        # traced step, applied to the timed step, gives the GEMM time inside ms_per_step
        frac_busy = trace["gemm_busy_ms_per_step"] / trace["step_span_ms"]
        trace["gemm_busy_frac_of_step"] = round(frac_busy, 4)
        trace["gemm_busy_ms_in_timed_step"] = round(frac_busy * ms_step, 4)
        trace["gemm_tflops_in_timed_step"] = round(trace["gemm_flops_per_step"] / (frac_busy * ms_step * 1e-3) / 1e12, 1)
    if traced:
        dom = dict(trace["families"][0])
        pk = (pmc.get("kernels") or {}).get(dom["kernel"], {})
        dom["pmc_hbm_bytes_per_launch"] = pk.get("hbm_bytes_per_launch")
        dom["pmc_mfma_busy_frac"] = pk.get("mfma_busy_frac")
        dom["pmc_l2_hit_rate"] = pk.get("l2_hit_rate")
        dom["pmc_source"] = pmc_src if pk else None
        ach = trace["gemm_tflops_over_busy"]
    else:
        dom, ach = None, seq_tf

    result = {
        "metric": METRIC,
        "value": round(pairs_s, 1),
        "unit": "image+text pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": DTYPE_LABEL[args.dtype],
        "data": "synthetic (seeded uint8 224x224 RGB images, full 77-token id captions; deterministic synthetic weights)",
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
            "kernel": "gemm_kernel / gemm2_kernel / gemm_attn_kernel (MFMA 16x16x32: every encoder GEMM; "
                      "the q/k/v GEMM fused with its attention, whose FLOPs it counts)",
            "bound": "mfma",
            "achieved": round(ach, 2),
            "peak": MFMA_PEAK_TFLOPS,
            "sustained_mfma_peak": {"value": MFMA_SUSTAINED_TFLOPS,
                                    "frac": round(ach / MFMA_SUSTAINED_TFLOPS, 4),
                                    "source": "tools/mfma_probe.hip: MFMA-only loop, random fp16 operands "
                                              "(profiles/r03_v10_mfma_peak_probe.jsonl)"},
            "unit": "TFLOP/s",
            "frac": round(ach / MFMA_PEAK_TFLOPS, 4),
            "dominant": dom,
            "traffic": (dom or {}).get("pmc_hbm_bytes_per_launch") or pmc.get("gemm_mean_hbm_bytes_per_launch"),
            "traffic_unit": "bytes per launch of the dominant kernel (PMC: 2*FETCH_SIZE + WRITE_SIZE, "
                            "gfx950-corrected, tools/pmc.sh with the timed step's tile configs)",
            "traffic_source": pmc_src,
            "mfma_busy_frac": pmc.get("gemm_mfma_busy_frac"),
            "mfma_busy_source": pmc_src if pmc.get("gemm_mfma_busy_frac") is not None else None,
            "mode": ("achieved = the step's GEMM FLOPs / the time at least one GEMM kernel runs, per step, from a "
                     "rocprofv3 kernel trace of the timed step's own form (two tower streams, hipGraph replay; "
                     "`trace`); dominant = the GEMM kernel with the most time per step in that trace")
                    if traced else "trace unavailable: per-kernel durations from the sequential profiled pass",
            "trace": trace,
            "sequential_pass": {"achieved": round(seq_tf, 2), "frac": round(seq_tf / MFMA_PEAK_TFLOPS, 4),
                                "avg_launch_us": round(gemm_ms / gemm_n * 1e3, 2),
                                "launches_per_step": gemm_n // nprof,
                                "algorithmic_bytes_per_launch": round(gemm_bytes / max(gemm_n, 1)),
                                "kernel_ms_per_step": {k: round(v[0] / nprof, 4) for k, v in prof.items()},
                                "mode": "HIP events on the launch stream around every GEMM, towers one after the "
                                        "other (no two kernels share the chip)"},
            "step_frac": round(step_flops / (ms_step * 1e-3) / 1e12 / MFMA_PEAK_TFLOPS, 4),
        },
    }
    if world > 1:
        result["dist"] = {"backend": backend, "world_size": torch.distributed.get_world_size()}
        if os.environ.get("CLM_REHEARSAL"):
            result["rehearsal"] = os.environ["CLM_REHEARSAL"]
    if world == 1 and not args.no_varlen:
        try:
            result["varlen_text"] = varlen_leg(model, cfg, dev, B, imgs, args.steps, args.warmup, rank)
        except Exception as e:  # report, never hide
            result["varlen_text"] = {"error": repr(e)}
    if rank == 0:
        try:
            result["parity"] = {"dtype": result["dtype"], **parity_vs_golden(model, cfg, dev)}
        except Exception as e:  # report, never hide
            result["parity"] = {"error": repr(e)}
    if rank == 0 and world == 1 and not args.no_unmerged and args.lora_mode == "merged":
        try:
            result["lora_unmerged"] = lora_unmerged_leg(cfg, sd, lora, dev, B, imgs, ids, args.steps, args.warmup,
                                                        args.dtype)
        except Exception as e:  # report, never hide
            result["lora_unmerged"] = {"error": repr(e)}
    if rank == 0 and world == 1 and not args.no_parity_mode:
        legs = {}
        for other in ("float16", "bfloat16", "mixed"):   # the same step with the other operand types
            if other == args.dtype:
                continue
            try:
                legs[DTYPE_LABEL[other]] = other_dtype_leg(cfg, sd, lora, dev, B, imgs, ids, args.steps, args.warmup,
                                                           args.lora_mode, other)
            except Exception as e:  # report, never hide
                legs[DTYPE_LABEL[other]] = {"error": repr(e)}
        result["dtype_legs"] = legs
    model.close()
    if not args.no_index_build:   # every rank takes part (batch-sharded + all_gather at N > 1)
        try:
            ib = index_build_leg(dev, world, rank, args.index_images, args.index_batch, args.dtype)
        except Exception as e:  # report, never hide
            ib = {"error": repr(e)}
        if rank == 0:
            result["index_build"] = ib
    host16 = qs_host = gpu_i = None
    if not args.no_search:   # every rank takes part when the index is sharded (world > 1)
        keep = rank == 0 and world == 1 and not args.no_cpu_baseline
        sr, host16, qs_host, gpu_i = search_leg(args.search_rows, args.search_queries, 5, dev, world, rank,
                                                keep_host=keep, persist_shard=not args.no_persist,
                                                single=not args.no_single)
        if rank == 0:
            result["search"] = sr
    if rank == 0 and world == 1 and not args.no_search and not args.no_near_dup:
        try:
            result["search_near_dup"] = near_dup_search_leg(dev)
        except Exception as e:  # report, never hide
            result["search_near_dup"] = {"error": repr(e)}
    if rank == 0 and world == 1 and not args.no_encode_item:
        try:
            result["encode_item"] = encode_item_leg(dev, args.dtype)
        except Exception as e:  # report, never hide
            result["encode_item"] = {"error": repr(e)}
    if rank == 0 and world == 1 and not args.no_l14:
        try:
            result["l14"] = l14_leg(dev, dtype=args.dtype)
        except Exception as e:  # report, never hide
            result["l14"] = {"error": repr(e)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        enc = cpu_encode_baseline(cfg, sd, lora, args.cpu_budget)
        cb = {"value": enc["batched64"]["pairs_per_s"], "unit": "image+text pairs/s",
              "cores": enc["threads"], "kind": "reference",
              "sample": f"{enc['batched64']['batches']} batches of 64 images + 64 captions "
                        f"({enc['batched64']['seconds']} s) of configs[1] (B/32 + LoRA r=8), {enc['impl']}, "
                        f"{enc['threads']} threads; per-item (the reference's encode_image/encode_text pattern): "
                        f"{enc['per_item']['pairs_per_s']} pairs/s over {enc['per_item']['calls']} calls",
              "encode": enc}
        if isinstance(result.get("encode_item"), dict) and "error" not in result["encode_item"]:
            result["encode_item"]["cpu_reference_per_item_ms"] = {
                "encode_image": round(1e3 / enc["per_item"]["images_per_s"], 2),
                "encode_text": round(1e3 / enc["per_item"]["texts_per_s"], 2),
                "note": "cpu_baseline.encode.per_item: transformers CLIPModel fp32 + LoRA hooks, batch 1, on "
                        "preprocessed pixel_values / token ids (no decode or tokenizer)"}
        if host16 is not None:
            cb["search"] = cpu_search_baseline(host16, qs_host, 5, args.cpu_search_queries, args.cpu_search_budget,
                                               gpu_i)
            cb["search"]["threads"] = enc["threads"]
        result["cpu_baseline"] = cb
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()

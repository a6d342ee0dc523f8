"""bench.py's host-side measurement logic on CPU: the GEMM launch table it attributes FLOPs with
(summed, it is the step's GEMM FLOPs of flops_per_pair) and the step-trace parser on a synthetic
two-queue rocprofv3 kernel trace; index_build.fold_sha256 (the configs[2] cross-world checksum)."""
import csv
import os
import sys

import pytest
import torch

from conftest import REPO

sys.path.insert(0, REPO)


@pytest.fixture(scope="module")
def bench():
    import bench as b
    return b


def test_launch_table_matches_flops_per_pair(bench):
    import clip_lora_match_amd as clm
    cfg = clm.get_preset("ViT-B/32")
    B = 256
    t = bench.gemm_launch_table(cfg, B)
    assert len(t["vision"]) == 1 + 4 * cfg.vision.layers and len(t["text"]) == 4 * cfg.text.layers
    fp = bench.flops_per_pair(cfg, lora_merged=True)
    proj = 2 * cfg.proj_dim * (cfg.vision.hidden + cfg.text.hidden)   # pool_project, not a GEMM launch
    gemm = sum(f for tw in t.values() for _, f, _ in tw)
    assert abs(gemm - (B * (fp["image"] + fp["caption"]) - B * proj)) / gemm < 1e-12


def _write_trace(path, cfg, B, bench, steps=3, overlap=True):
    """a synthetic kernel trace: per step, the vision queue (2) and text queue (3) run their kernels
    back to back; the two queues start together, so their kernels overlap in time"""
    t = bench.gemm_launch_table(cfg, B)
    rows = []
    cols = ["Kind", "Queue_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp"]
    t0 = 1_000_000
    for s in range(steps):
        span = 0
        for q, tower, first in ((2, "vision", "patchify_fast_kernel<false>"), (3, "text", "text_lens_kernel")):
            ts = t0
            for name, dur in [(first, 1000)] + [(f"void clm::(anonymous namespace)::gemm_kernel<{lab}>(clm::GemmArgs)",
                                                 10_000) for lab, _, _ in t[tower]] + [("ln4_kernel", 500)]:
                rows.append({"Kind": "KERNEL_DISPATCH", "Queue_Id": q, "Kernel_Name": name,
                             "Start_Timestamp": ts, "End_Timestamp": ts + dur})
                ts += dur + 100
            span = max(span, ts - t0)
            if not overlap:
                t0 = ts
        t0 += span + 5000
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=cols)
        w.writeheader()
        w.writerows(rows)
    return t


def test_parse_step_trace_two_queues(bench, tmp_path):
    import clip_lora_match_amd as clm
    cfg = clm.get_preset("ViT-B/32")
    p = tmp_path / "k.csv"
    t = _write_trace(p, cfg, 256, bench)
    r = bench.parse_step_trace(str(p), cfg, 256, 2)
    assert r["steps"] == 2 and r["matched_launch_table"]
    n_v, n_t = len(t["vision"]), len(t["text"])
    # every GEMM 10 us; the two queues overlap, so the busy union is the longer queue's GEMM span
    assert r["gemm_kernel_ms_per_step_sum"] == pytest.approx((n_v + n_t) * 0.010, rel=1e-6)
    assert r["gemm_busy_ms_per_step"] == pytest.approx(n_v * 10_000 / 1e6, rel=1e-6)   # gaps are not busy
    assert r["gemm_busy_ms_per_step"] <= r["step_span_ms"]
    fam = {f["kernel"]: f for f in r["families"]}
    out = fam["gemm_kernel<out>"]
    assert out["launches_per_step"] == cfg.vision.layers - 1 + cfg.text.layers - 1
    assert out["avg_us"] == pytest.approx(10.0)
    assert r["gemm_flops_per_step"] == pytest.approx(sum(f for tw in t.values() for _, f, _ in tw))


def test_fold_sha256_sees_every_bit():
    from clip_lora_match_amd.index_build import fold_sha256
    g = torch.Generator().manual_seed(3)
    a = torch.randn((1000, 512), generator=g)
    b = a.clone()
    assert fold_sha256(a) == fold_sha256(b)
    b[777, 301] = torch.nextafter(b[777, 301], torch.tensor(2.0))   # one ulp of one value
    assert fold_sha256(a) != fold_sha256(b)
    c = a.clone()
    c[[3, 4]] = a[[4, 3]]                                            # two rows swapped
    assert fold_sha256(a) != fold_sha256(c)

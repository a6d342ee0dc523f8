"""Multi-rank GPU paths on one MI355X: world 2 over gloo (RCCL refuses two ranks
per device; the driver's 8-GPU node runs the RCCL path). The product's own sharded index build
and row-sharded search with the GPU merge must equal the single-rank results bit for bit, and
bench.py --gpus 2 must start and report 2 ranks by itself. The RCCL entry points themselves run
in test_rccl_collectives (one rank per GPU the box has)."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_sharded_build_and_search_world2(tmp_path):
    out = tmp_path / "res.json"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(REPO, "tests", "dist_gpu_worker.py"),
           str(out), str(tmp_path)]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    r = json.loads(out.read_text())
    assert r["world"] == 2
    assert r["file_rows_min_max"] == [37, 37]     # both ranks read the complete file
    for key in ("build_img_equal", "build_txt_equal", "file_equal", "search_idx_equal", "search_scores_equal",
                "merge_roundtrip", "big_build_equal", "big_file_equal", "big_paths_ok", "synth_rows_stable",
                "big_f16_exchange_equal",
                "write_failure_raised_everywhere"):
        assert r[key], (key, r)
    assert r["planted_top1"] == [5, 150_000, 150_001, 299_999]
    assert r["big_file_rows"] == 65_536
    assert r["big_f16_exchange_device"].startswith("cuda")   # host_rows=False: device rows on every rank


N_1M = 1_000_000


# bench.py's configs[2] leg: the headline compute dtype and the fp32 all_gather exchange; its
# index_fold_sha256 line equals the world-1 checksum of this build (rows do not depend on the batch)
INDEX_DTYPE, INDEX_EXCHANGE = "mixed", "fp32"


@pytest.fixture(scope="module")
def index_1m(tmp_path_factory):
    """configs[2] at its stated size (rebuild_index over 1 M device-generated images at the bench's
    dtype and exchange), run once per world size {1, 2} by tests/dist_index_worker.py; results by world."""
    d = tmp_path_factory.mktemp("index_1m")
    return {"dir": d, "res": {}}


def _run_index_1m(index_1m, world):
    out = index_1m["dir"] / f"w{world}.json"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(REPO, "tests", "dist_index_worker.py"),
           str(out), str(index_1m["dir"]), str(N_1M), INDEX_EXCHANGE, INDEX_DTYPE]
    p = subprocess.run(cmd, env=dict(os.environ, MASTER_ADDR="127.0.0.1"), capture_output=True, text=True,
                       timeout=170)
    assert p.returncode == 0, p.stderr[-3000:]
    r = json.loads(out.read_text())
    index_1m["res"][world] = r
    return r


def test_index_build_1m_world1(index_1m):
    """BASELINE configs[2] at 1 M images on one rank: the returned rows are the file's, 1 M unit rows
    with every image path in place (scripts/rebuild_index.py:64-96)."""
    r = _run_index_1m(index_1m, 1)
    assert r["file_rows"] == N_1M and r["rows_shape"] == [N_1M, 512]
    assert r["rows_device"].startswith("cuda")   # host_rows=False: the gathered rows stay on the device
    assert r["file_sha"] == r["rows_sha"] and r["file_dtype"] == "torch.float32"
    assert r["paths_ok"] and r["texts_ok"] and r["unit_rows"] < 1e-6
    print(f"\nconfigs[2] 1 M build ({INDEX_DTYPE}, {INDEX_EXCHANGE} exchange): fold {r['rows_sha']}")


def test_index_build_1m_spot_vs_oracle(index_1m):
    """64 rows of the 1 M build (spread over the whole index) against the fp32 oracle
    (oracle.clip_ref.image_features + the reference's second normalise) on the same device-generated
    pixels: the headline dtype's bars, 1 - cos <= 1e-4 per row and pairwise scores within 1e-3."""
    if 1 not in index_1m["res"]:
        pytest.skip("needs the world-1 result (run the module)")
    import numpy as np
    import clip_lora_match_amd as clm
    from clip_lora_match_amd import synthetic as syn
    from clip_lora_match_amd import weights as W
    from oracle import clip_ref as R
    r = index_1m["res"][1]
    cfg = clm.get_preset("ViT-B/32")
    src = syn.DeviceImages(N_1M, cfg.image_size, seed=20240)
    px = np.stack([src.batch(i, i + 1).cpu().numpy()[0] for i in r["spot_rows"]])
    ref = R.image_features(W.synthetic_state_dict(cfg, 0), cfg, R.preprocess_u8(px, cfg.mean, cfg.std),
                           W.synthetic_lora(cfg, 1))
    ref = ref / np.linalg.norm(ref, axis=1, keepdims=True)
    got = np.asarray(r["spot_emb"], np.float64)
    cos = np.sum(got * ref, 1) / (np.linalg.norm(got, axis=1) * np.linalg.norm(ref, axis=1))
    err = np.max(np.abs(got @ got.T - ref @ ref.T))
    print(f"\n1 M build spot check: max 1 - cos {np.max(1 - cos):.2e}, max score error {err:.2e}")
    assert np.max(1 - cos) <= 1e-4 and err <= 1e-3


def test_index_build_1m_world2(index_1m):
    """The same build sharded over 2 ranks (gloo on one GPU; RCCL on the 8-GPU node): every rank
    gathers the same 1 M rows (on its device, host_rows=False), and the index is bit-identical to
    the world-1 build (fold checksum)."""
    if 1 not in index_1m["res"]:
        pytest.skip("needs the world-1 result (run the module)")
    r = _run_index_1m(index_1m, 2)
    r1 = index_1m["res"][1]
    assert r["file_rows"] == N_1M and r["paths_ok"] and r["texts_ok"]
    assert r["rank_shas"] == [r1["rows_sha"]] * 2
    assert r["file_sha"] == r1["file_sha"] == r1["rows_sha"]


def test_rccl_collectives(tmp_path):
    """Every collective of the product and bench.py through an RCCL ("nccl") process group on the
    box's GPU(s): one rank per visible GPU (one on a 1-GPU box)."""
    import torch
    world = max(torch.cuda.device_count(), 1)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(REPO, "tests", "rccl_worker.py"),
           str(tmp_path)]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=180)
    assert p.returncode == 0, p.stderr[-3000:]
    for r in range(world):
        res = json.loads((tmp_path / f"rank{r}.json").read_text())
        assert res["world"] == world and "nccl" in res["backend"], res
        for key in ("all_gather_rows_equal", "gather_candidates_equal", "merge_sorted", "max_all_reduce",
                    "broadcast_object", "host_all_reduce"):
            assert res[key], (key, res)


def test_bench_spawns_its_own_ranks(tmp_path):
    """bench.py --gpus 2 with no launcher around it starts 2 ranks itself (gloo rehearsal on a
    1-GPU box) and reports n_gpus 2 from a 2-rank process group."""
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--batch", "32", "--no-cpu-baseline", "--no-l14", "--no-parity-mode", "--search-rows", "600000",
           "--search-queries", "256"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    assert p.returncode == 0, p.stderr[-3000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1]
    r = json.loads(line)
    assert r["n_gpus"] == 2 and r["dist"]["world_size"] == 2
    assert r["search"]["n_gpus"] == 2 and r["search"]["qps"] > 0
    assert r["value"] > 0

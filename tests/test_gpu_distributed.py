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
                "write_failure_raised_everywhere"):
        assert r[key], (key, r)
    assert r["planted_top1"] == [5, 150_000, 150_001, 299_999]
    assert r["big_file_rows"] == 65_536


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

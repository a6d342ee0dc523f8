"""Single / small-batch search probe on the configs[4] index (10 M x 512 fp16, rows seeded as
bench.py's search leg): per nq, ms per call of CosineIndex.search(q[:nq], 5). Env knobs of the
library (CLM_SCAN_NW / CLM_SCAN_D) select the scan16 shape; run under rocprofv3 for kernel times.
  python tools/single_probe.py [--rows N] [--reps R] [--nq 1,16]"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from clip_lora_match_amd.search import CosineIndex  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=10_000_000)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--nq", default="1,2,4,8,16")
ap.add_argument("--dim", type=int, default=512)
a = ap.parse_args()
dev = torch.device("cuda", 0)
idx = CosineIndex(a.dim, capacity=a.rows)
chunk = 1 << 20
for c0 in range(0, a.rows, chunk):
    g = torch.Generator(device=dev).manual_seed(7 + c0 // chunk)
    x = torch.randn((min(chunk, a.rows - c0), a.dim), generator=g, device=dev)
    idx.append((x / x.norm(dim=-1, keepdim=True)).half())
    del x
gq = torch.Generator(device=dev).manual_seed(8)
q = torch.randn((64, a.dim), generator=gq, device=dev)
q = (q / q.norm(dim=-1, keepdim=True)).half()
nbytes = a.rows * a.dim * 2 + a.rows * 4
out = {"rows": a.rows, "dim": a.dim, "env": {k: v for k, v in os.environ.items() if k.startswith("CLM_")}}
for nq in [int(v) for v in a.nq.split(",")]:
    idx.search(q[:nq], 5)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for r in range(a.reps):
        idx.search(q[r % 4 * 16 // 4: r % 4 * 16 // 4 + nq] if nq <= 12 else q[:nq], 5)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.reps
    out[str(nq)] = {"ms": round(dt * 1e3, 3), "hbm_frac": round(nbytes / dt / 8e12, 4)}
out["stats"] = idx.stats()
print(json.dumps(out), flush=True)

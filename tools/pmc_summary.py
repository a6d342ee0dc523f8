"""Summarise rocprofv3 PMC passes (tools/pmc.sh) into per-kernel and per-GEMM-shape HBM
traffic and MFMA utilisation per launch.

gfx950 corrections (MI355X_MICROARCH.md §HBM, § Per-instruction cycle constants):
  * FETCH_SIZE reports half the bytes of wide coalesced streaming reads -> doubled; WRITE_SIZE
    is exact for 16-B stores; both in KiB.
  * SQ_VALU_MFMA_BUSY_CYCLES counts SIMD-cycles summed over the chip; GRBM_GUI_ACTIVE is summed
    over the 8 XCDs -> kernel cycles = GRBM_GUI_ACTIVE / 8, and
    mfma_busy_frac = MFMA_BUSY / (kernel cycles * 256 CUs * 4 SIMDs).
  * SQ_INSTS_VALU_MFMA_MOPS_BF16 / _F16 count 512-FLOP units -> MFMA FLOPs = 512 * MOPS (both
    collected: the headline runs fp16 operands).
  * l2_hit_rate = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum) (the XCD L2s; a miss is served by
    the Infinity Cache or HBM).
GEMM launches are labelled by their position in the sequential encode step (tools/pmc.sh runs
bench.py --sequential): vision patch, 12 x (qkv, out, fc1, fc2), then text 12 x (qkv, out, fc1,
fc2); the last layer's out / fc1 / fc2 run on the pooled rows only.
Writes profiles/<tag>_pmc_summary.json (bench.py reads the newest one for roofline.traffic and
roofline.mfma_busy_frac).
"""
import collections
import csv
import glob
import json
import os
import re
import sys

N_CU, SIMD_PER_CU, N_XCD = 256, 4, 8


def short(name):
    m = re.search(r"(gemm2?_kernel)<([^>]*)>", name)
    if m:
        return m.group(1) + "<" + m.group(2) + ">"
    name = name.replace("clm::(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"\(.*", "", name)


def step_labels(layers_v=12, layers_t=12):
    lab = ["vision.patch"]
    for tower, L in (("vision", layers_v), ("text", layers_t)):
        for l in range(L):
            last = ".pooled" if l == L - 1 else ""
            lab += [f"{tower}.qkv", f"{tower}.out{last}", f"{tower}.fc1{last}", f"{tower}.fc2{last}"]
    return lab


def load(path):
    """{dispatch_id: (kernel, {counter: value})} from one pass's counter_collection.csv"""
    out = {}
    for r in csv.DictReader(open(path)):
        did = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or len(out))
        k = short(r["Kernel_Name"])
        ent = out.setdefault(did, (k, {}))
        ent[1][r["Counter_Name"]] = ent[1].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def main(src="gpurun_out/pmc", tag="r02"):
    passes = sorted(d for d in os.listdir(src) if re.fullmatch(r"p\d+", d))
    per_kernel = collections.defaultdict(lambda: collections.defaultdict(list))
    gemm_seq = {}
    for p in passes:
        fs = sorted(glob.glob(os.path.join(src, p, "**", "*counter_collection.csv"), recursive=True))
        if not fs:
            continue
        d = load(fs[0])
        seq = []
        for did in sorted(d):
            k, cv = d[did]
            for c, v in cv.items():
                per_kernel[k][c].append(v)
            if k.startswith("gemm"):
                seq.append(cv)
        gemm_seq[p] = seq
    labels = step_labels()
    shapes = collections.defaultdict(lambda: collections.defaultdict(list))
    for p, seq in gemm_seq.items():
        if len(seq) % len(labels):
            continue
        for i, cv in enumerate(seq):
            for c, v in cv.items():
                shapes[labels[i % len(labels)]][c].append(v)

    def derive(cv):
        m = {c: sum(v) / len(v) for c, v in cv.items()}
        o = {}
        if "FETCH_SIZE" in m:
            o["fetch_bytes"] = 2 * m["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in m:
            o["write_bytes"] = m["WRITE_SIZE"] * 1024
        if "fetch_bytes" in o and "write_bytes" in o:
            o["hbm_bytes_per_launch"] = o["fetch_bytes"] + o["write_bytes"]
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and m.get("GRBM_GUI_ACTIVE"):
            o["mfma_busy_frac"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / N_XCD * N_CU * SIMD_PER_CU)
            o["kernel_cycles"] = m["GRBM_GUI_ACTIVE"] / N_XCD
        if "SQ_INSTS_VALU_MFMA_MOPS_BF16" in m or "SQ_INSTS_VALU_MFMA_MOPS_F16" in m:
            o["mfma_flops"] = 512 * (m.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0) + m.get("SQ_INSTS_VALU_MFMA_MOPS_F16", 0.0))
        if "SQ_LDS_BANK_CONFLICT" in m and m.get("SQ_INSTS_LDS"):
            o["lds_bank_conflicts_per_lds_inst"] = m["SQ_LDS_BANK_CONFLICT"] / m["SQ_INSTS_LDS"]
        if m.get("TCC_HIT_sum") is not None and m.get("TCC_MISS_sum") is not None and m["TCC_HIT_sum"] + m["TCC_MISS_sum"]:
            o["l2_hit_rate"] = m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
        o["launches"] = max(len(v) for v in cv.values())
        return o

    out = {"correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE half-count); "
                         "mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * 256 CU * 4 SIMD)",
           "kernels": {k: derive(cv) for k, cv in sorted(per_kernel.items())},
           "gemm_shapes": {k: derive(cv) for k, cv in shapes.items()}}
    g = [v for k, v in out["kernels"].items() if k.startswith("gemm")]
    n = sum(v["launches"] for v in g)
    if g and all("hbm_bytes_per_launch" in v for v in g):
        out["gemm_mean_hbm_bytes_per_launch"] = sum(v["hbm_bytes_per_launch"] * v["launches"] for v in g) / n
    if g and all("mfma_busy_frac" in v for v in g):
        # launch-cycle-weighted: the chip's MFMA-busy share over all GEMM time
        cyc = sum(v["kernel_cycles"] * v["launches"] for v in g)
        out["gemm_mfma_busy_frac"] = sum(v["mfma_busy_frac"] * v["kernel_cycles"] * v["launches"] for v in g) / cyc
    path = f"profiles/{tag}_pmc_summary.json"
    json.dump(out, open(path, "w"), indent=1)
    print(path, json.dumps({k: out.get(k) for k in ("gemm_mean_hbm_bytes_per_launch", "gemm_mfma_busy_frac")}))


if __name__ == "__main__":
    main(*sys.argv[1:])

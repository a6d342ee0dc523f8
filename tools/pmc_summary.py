"""Summarise rocprofv3 PMC passes (tools/pmc.sh) into per-kernel HBM traffic per launch.

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the bytes of wide
coalesced streaming reads -> doubled; WRITE_SIZE is exact for 16-B stores. Both are in KiB.
Writes profiles/<tag>_pmc_summary.json (bench.py reads the newest one for roofline.traffic).
"""
import collections
import csv
import json
import re
import sys


def short(name):
    m = re.search(r"(gemm2?_kernel)<([^>]*)>", name)
    if m:
        return m.group(1) + "<" + m.group(2) + ">"
    return re.sub(r"\(.*", "", name).replace("clm::(anonymous namespace)::", "").replace("void ", "")


def load(path, counter):
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            per[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return per


def main(src="gpurun_out/pmc", tag="r01"):
    fetch = load(f"{src}/p1/run_counter_collection.csv", "FETCH_SIZE")
    write = load(f"{src}/p2/run_counter_collection.csv", "WRITE_SIZE")
    out = {"correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE half-count)",
           "kernels": {}}
    g_bytes, g_n = 0.0, 0
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [0.0])
        w = write.get(k, [0.0])
        per_launch = (2 * sum(f) / len(f) + sum(w) / len(w)) * 1024
        out["kernels"][k] = {"launches": len(f), "hbm_bytes_per_launch": per_launch,
                             "fetch_bytes": 2 * sum(f) / len(f) * 1024, "write_bytes": sum(w) / len(w) * 1024}
        if k.startswith("gemm"):
            g_bytes += per_launch * len(f)
            g_n += len(f)
    out["gemm_mean_hbm_bytes_per_launch"] = g_bytes / max(g_n, 1)
    path = f"profiles/{tag}_pmc_summary.json"
    json.dump(out, open(path, "w"), indent=1)
    print(path, json.dumps({"gemm_mean_hbm_bytes_per_launch": out["gemm_mean_hbm_bytes_per_launch"]}))


if __name__ == "__main__":
    main(*sys.argv[1:])

"""Summarise tools/attn_pmc.sh's passes for one kernel family (default attn_long_kernel):
  python tools/attn_pmc_summary.py gpurun_out/apmc <tag> [kernel-substring]
Writes profiles/<tag>_attn_pmc_summary.json.
Units (MI355X_MICROARCH.md, rocprofv3 PMC / cycle-constants rows): SQ_WAVE_CYCLES, SQ_WAIT_*,
SQ_ACTIVE_INST_* count quad-cycles summed over waves; WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY
~= WAVE_CYCLES. SQ_VALU_MFMA_BUSY_CYCLES counts SIMD-cycles over the chip; GRBM_GUI_ACTIVE is
summed over the 8 XCDs."""
import collections
import csv
import glob
import json
import os
import re
import sys

N_CU, SIMD_PER_CU, N_XCD = 256, 4, 8


def main(src="gpurun_out/apmc", tag="r05", kern="attn_long_kernel"):
    acc = collections.defaultdict(list)
    names = set()
    for f in sorted(glob.glob(os.path.join(src, "p*", "*counter_collection.csv"))):
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            if kern not in r["Kernel_Name"]:
                continue
            names.add(re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)", "anon")))
            per[r.get("Dispatch_Id") or r.get("Correlation_Id")][r["Counter_Name"]] += float(r["Counter_Value"])
        for cv in per.values():
            for c, v in cv.items():
                acc[c].append(v)
    m = {c: sum(v) / len(v) for c, v in acc.items()}
    o = {"kernel": sorted(names), "launches": max((len(v) for v in acc.values()), default=0),
         "counters_mean_per_launch": m}
    g = m.get("GRBM_GUI_ACTIVE")
    if g:
        cyc = g / N_XCD
        o["kernel_cycles"] = cyc
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            o["mfma_busy_frac"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * N_CU * SIMD_PER_CU)
    wc = m.get("SQ_WAVE_CYCLES")
    if wc:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS",
                  "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
            if c in m:
                o[c.lower().replace("sq_", "") + "_share_of_wave_cycles"] = m[c] / wc
    if m.get("SQ_INSTS_LDS"):
        o["lds_bank_conflicts_per_lds_inst"] = m.get("SQ_LDS_BANK_CONFLICT", 0.0) / m["SQ_INSTS_LDS"]
    if m.get("SQ_INSTS_VALU_MFMA_MOPS_BF16"):
        o["mfma_flops"] = 512 * m["SQ_INSTS_VALU_MFMA_MOPS_BF16"]
    if m.get("SQ_INSTS_VALU") and m.get("SQ_WAVES"):
        o["valu_insts_per_wave"] = m["SQ_INSTS_VALU"] / m["SQ_WAVES"]
    if m.get("SQ_INSTS_LDS") and m.get("SQ_WAVES"):
        o["lds_insts_per_wave"] = m["SQ_INSTS_LDS"] / m["SQ_WAVES"]
    path = f"profiles/{tag}_attn_pmc_summary.json"
    json.dump(o, open(path, "w"), indent=1)
    print(path, json.dumps({k: v for k, v in o.items() if k != "counters_mean_per_launch"}, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])

"""Summarise the rocprofv3 PMC passes written by tools/pmc.sh into per-kernel averages, with
the gfx950 corrections of MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) x 1024 x 2 (it tallies
128-B requests at 64 B), WRITE_SIZE (KB) x 1024 as is.  traffic = fetch + write bytes per
launch (memory-side L2 traffic; Infinity-Cache hits are included).

    python tools/pmc_summary.py gpurun_out/pmc_r1b[,gpurun_out/pmc_r1b_bf16] profiles/r1/pmc_summary.json
"""
import collections
import csv
import json
import os
import sys


def load(path):
    d = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        d[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return d


def main(srcs, dst):
    """srcs: one pass directory, or several separated by commas (e.g. the fp32 and the bf16
    bench runs: their conv kernels have different names, so the summaries merge)."""
    out = collections.defaultdict(dict)
    for src in srcs.split(","):
        for ps in ("fetch", "write", "sq", "lds"):
            p = os.path.join(src, ps, "run_counter_collection.csv")
            if not os.path.exists(p):
                continue
            for k, cs in load(p).items():
                if not k.startswith(("cwt::", "void cwt::")):
                    continue
                for c, v in cs.items():
                    out[k][c] = sum(v) / len(v)
                    out[k]["launches"] = len(v)
    res = {}
    for k, cs in out.items():
        e = dict(cs)
        if "FETCH_SIZE" in cs:
            e["fetch_bytes"] = cs["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in cs:
            e["write_bytes"] = cs["WRITE_SIZE"] * 1024
        if "fetch_bytes" in e and "write_bytes" in e:
            e["traffic_bytes"] = e["fetch_bytes"] + e["write_bytes"]
        if "SQ_VALU_MFMA_BUSY_CYCLES" in cs and "SQ_BUSY_CYCLES" in cs and cs["SQ_BUSY_CYCLES"] > 0:
            # SQ_BUSY_CYCLES is per-SE aggregate; report MFMA busy per SIMD-cycle for 256 CUs x 4 SIMDs
            e["mfma_busy_cycles"] = cs["SQ_VALU_MFMA_BUSY_CYCLES"]
        res[k] = e
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    json.dump(res, open(dst, "w"), indent=1, sort_keys=True)
    for k, e in sorted(res.items(), key=lambda kv: -kv[1].get("traffic_bytes", 0))[:12]:
        print(f"{k[:80]:80s} traffic/launch {e.get('traffic_bytes', 0) / 1e6:9.2f} MB")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])

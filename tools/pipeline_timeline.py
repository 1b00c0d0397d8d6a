"""The pipelined bench's kernel trace, per extractor pass (round 6, DESIGN.md §3 "Round 6"):
how often the extractor streams run kernels concurrently, which kernels of a pass overlap the
previous episode's fused inner loop, and each layer's wall time inside the pipeline.

    python tools/pipeline_timeline.py <rocprofv3 run_kernel_trace.csv> [out.json]

The window is the main (pipelined) leg's steady state: from the 5th to the 23rd fused-loop launch
(the bench's first launches of adapt_persist_tail_kernel<5> are its warm-up and timed steps).
"""
import csv
import json
import sys


def main(path, out=None):
    rows = list(csv.DictReader(open(path)))
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    rows.sort(key=lambda r: r["s"])
    loops = [r for r in rows if "adapt_persist_tail_kernel<5>" in r["Kernel_Name"]]
    t0, t1 = loops[4]["s"], loops[22]["s"]
    ls = loops[4]["Stream_Id"]
    win = [r for r in rows if r["s"] >= t0 and r["e"] <= t1 and r["Stream_Id"] != ls]
    # concurrency of the extractor streams' kernels over the window
    ev = sorted([(r["s"], 1) for r in win] + [(r["e"], -1) for r in win])
    cur, last, acc = 0, t0, {}
    for t, d in ev:
        acc[cur] = acc.get(cur, 0) + t - last
        cur += d
        last = t
    conc = {k: round(v / (t1 - t0), 3) for k, v in sorted(acc.items())}
    # passes: each starts with the stem's first conv
    passes = []
    for sid in sorted(set(r["Stream_Id"] for r in win)):
        p = None
        for r in [x for x in win if x["Stream_Id"] == sid]:
            if "stem_conv1" in r["Kernel_Name"]:
                if p:
                    passes.append(p)
                p = []
            if p is not None:
                p.append(r)
        if p:
            passes.append(p)
    n = max(set(len(p) for p in passes), key=[len(p) for p in passes].count)
    passes = [p for p in passes if len(p) == n]
    L = [(l["s"], l["e"]) for l in loops]

    def overlap(r):
        return sum(max(0, min(e, r["e"]) - max(s, r["s"])) for s, e in L) / max(1, r["e"] - r["s"])

    per = []
    for i in range(n):
        ks = [p[i] for p in passes]
        per.append({"i": i, "kernel": ks[0]["Kernel_Name"].split("(")[0][:70],
                    "us": round(sum(k["e"] - k["s"] for k in ks) / len(ks) / 1e3, 1),
                    "loop_overlap": round(sum(overlap(k) for k in ks) / len(ks), 2)})
    res = {"trace": path, "window_ms": round((t1 - t0) / 1e6, 3), "episodes": 18,
           "ms_per_episode": round((t1 - t0) / 1e6 / 18, 3), "passes": len(passes), "kernels_per_pass": n,
           "pass_wall_ms": round(sum((p[-1]["e"] - p[0]["s"]) for p in passes) / len(passes) / 1e6, 3),
           "loop_ms": round(sum(e - s for s, e in L[4:22]) / 18 / 1e6, 3),
           "extractor_kernels_running_fraction": conc, "per_kernel": per}
    js = json.dumps(res, indent=1)
    if out:
        open(out, "w").write(js + "\n")
    print(js[:1500])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)

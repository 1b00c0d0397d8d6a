"""Per-conv roofline table of one extractor pass from a bench --profile-json file.

    python tools/conv_table.py profiles/r2/per_launch.json > profiles/r2/conv_table.md

Each launch of the per-launch episode (libcwt profile level 2: hipEvent pair around every
launch, so each time carries ~1-3 us of event overhead) is priced at
max(executed FLOPs / MFMA roof, algorithmic bytes / 8 TB/s); roof 838.9 TF for the bf16x3
convs (bf16 MFMA / 3), 2516.6 TF for the plain-bf16 ones.  The footer gives the stack's
roofline_frac (sum of per-launch floors / sum of launch times), the same figure bench.py
reports as conv_stack.roofline_frac.
"""
import json
import sys

HBM = 8.0e12
X3 = 2516.6e12 / 3
B16 = 2516.6e12


def main(path):
    d = json.load(open(path))
    rows = d["per_launch_one_episode"]
    out = ["| # | launch | GFLOP | MB | us | TF/s | floor us | frac |", "|---|---|---|---|---|---|---|---|"]
    tot_t = tot_floor = 0.0
    groups = {}
    for i, r in enumerate(rows):
        name, fl, by, ms = (r if isinstance(r, list) else (r["name"], r["flops"], r["bytes"], r["ms"]))
        if name.startswith(("extract_features", "inner_adapt", "attention", "cwt_", "normalize", "classify", "seg_")):
            continue
        roof = B16 if "b16" in name else X3
        floor = max(fl / roof, by / HBM) * 1e6
        us = ms * 1e3
        tot_t += us
        tot_floor += floor
        key = name.split(" ")[0]
        g = groups.setdefault(key, [0, 0.0, 0.0])
        g[0] += 1
        g[1] += us
        g[2] += floor
        out.append(f"| {i} | `{name}` | {fl / 1e9:.2f} | {by / 1e6:.1f} | {us:.1f} | {fl / ms / 1e9 if ms else 0:.1f} | "
                   f"{floor:.1f} | {floor / us if us else 0:.2f} |")
    out.append("")
    out.append(f"Stack: {tot_t:.0f} us of launches, floor {tot_floor:.0f} us, roofline_frac {tot_floor / tot_t:.3f}")
    out.append("")
    out.append("| kernel | launches | us | floor us | frac |")
    out.append("|---|---|---|---|---|")
    for k, (n, us, fl) in sorted(groups.items(), key=lambda kv: -kv[1][1]):
        out.append(f"| `{k}` | {n} | {us:.1f} | {fl:.1f} | {fl / us:.2f} |")
    print("\n".join(out))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof.json")

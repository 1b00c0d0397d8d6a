"""Per-conv roofline table of one extractor pass from a bench --profile-json file, optionally
joined with the per-kernel PMC summary of the same build (tools/pmc.sh + tools/pmc_summary.py).

    python tools/conv_table.py gpurun_out/prof.json [profiles/r5/pmc_summary.json] > profiles/r5/conv_table_f32.md

Each launch of the per-launch episode (libcwt profile level 2: a hipEvent pair around every
launch, so each time carries ~1-3 us of event overhead) is priced at
max(algorithmic FLOPs / matrix roof, algorithmic bytes / 8 TB/s), the roof of its arithmetic:
x6 / x6w / x6w4 (fp32 width as six bf16 products) 419.4 TF, f32d (v_mfma_f32) 157.3 TF, x3s (bf16x3)
838.9 TF, b16 2516.6 TF.  The Winograd forms (x6w F(2x2,3x3), x6w4 F(4x4,3x3)) are priced on the direct conv's
FLOPs (the algorithm's work; they execute 4/9 and 1/4 of them).  The footer gives the stack's roofline_frac (sum of
per-launch floors / sum of launch times; bench.py's conv_stack.roofline_frac), then one row per
kernel instantiation with its PMC averages: HBM traffic per launch (FETCH_SIZE x 2 + WRITE_SIZE,
gfx950-corrected) against the algorithmic bytes, MFMA busy share, VALU / MFMA / LDS instruction
counts and the wave-wait share.  PMC is per kernel instantiation (one per tile form and stage),
averaged over the launches of every layer that instantiation served, as rocprofv3 reports it.
"""
import json
import re
import sys

HBM = 8.0e12
ROOFS = {"x6w": 2516.6e12 / 6, "x6w4": 2516.6e12 / 6, "x6": 2516.6e12 / 6, "f32d": 157.3e12, "f32": 157.3e12, "x3s": 2516.6e12 / 3,
         "b16": 2516.6e12}


def roof_of(name):
    m = re.match(r"conv_igemm_(\w+?)<", name)
    return ROOFS.get(m.group(1) if m else "", 2516.6e12 / 3)


def pmc_key(name):
    """'conv_igemm_x6w<256,256,6> ...' -> (kind, bm, bn, stage) to match rocprofv3's kernel names
    'void cwt::conv_igemm_x6<256, 256, 4, 2, 2, 7, 0>(cwt::ConvSArgs)' (the Winograd form's GEMMs
    are the stage-7 conv_igemm_x6 instantiations; its transforms are separate kernels)."""
    m = re.match(r"conv_igemm_(\w+?)<(\d+),(\d+),(\d+)>", name)
    if not m:
        return None
    if m.group(1) in ("x6w", "x6w4"):   # F(2x2) / F(4x4): stage 7 / 8 (the bottleneck's F(2x2): its own 6)
        return "x6", m.group(2), m.group(3), ("8" if m.group(1) == "x6w4" else "6" if m.group(4) == "6" else "7")
    return m.group(1), m.group(2), m.group(3), m.group(4)


def pmc_lookup(pmc, key):
    hits = []
    for k, e in pmc.items():
        mk = re.search(r"conv_igemm_(\w+?)<([^>]*)>", k)
        if not mk:
            continue
        targs = [t.strip() for t in mk.group(2).split(",")]
        if mk.group(1) == key[0] and len(targs) >= 6 and targs[0] == key[1] and targs[1] == key[2] and targs[5] == key[3]:
            hits.append(e)
    return hits


def main(path, pmc_path=None):
    d = json.load(open(path))
    pmc = json.load(open(pmc_path)) if pmc_path else {}
    rows = d["per_launch_one_episode"]
    out = ["| # | launch | GFLOP | MB | us | TF/s | roof TF | floor us | frac |",
           "|---|---|---|---|---|---|---|---|---|"]
    tot_t = tot_floor = 0.0
    groups = {}
    for i, r in enumerate(rows):
        name, fl, by, ms = (r if isinstance(r, list) else (r["name"], r["flops"], r["bytes"], r["ms"]))
        if not name.startswith("conv_igemm"):
            continue
        roof = roof_of(name)
        floor = max(fl / roof, by / HBM) * 1e6
        us = ms * 1e3
        tot_t += us
        tot_floor += floor
        key = name.split(" ")[0]
        g = groups.setdefault(key, [0, 0.0, 0.0, 0.0])
        g[0] += 1
        g[1] += us
        g[2] += floor
        g[3] += by
        out.append(f"| {i} | `{name}` | {fl / 1e9:.2f} | {by / 1e6:.1f} | {us:.1f} | {fl / ms / 1e9 if ms else 0:.1f} | "
                   f"{roof / 1e12:.1f} | {floor:.1f} | {floor / us if us else 0:.2f} |")
    out.append("")
    out.append(f"Stack: {tot_t:.0f} us of launches, floor {tot_floor:.0f} us, roofline_frac {tot_floor / tot_t:.3f}")
    # the Winograd forms on the work they execute: each x6w record is followed by
    # its wino_in / wino_gemm / wino_out sub-records (api.hip run_wino_conv)
    wrows = []
    prows = d.get("winograd_parts", rows)   # bench.py's level-3 extraction (the parts' own events)
    for i, r in enumerate(prows):
        name, fl, by, ms = (r if isinstance(r, list) else (r["name"], r["flops"], r["bytes"], r["ms"]))
        if not name.startswith("conv_igemm_x6w"):
            continue
        sub = {}
        for q in prows[i + 1:i + 4]:
            qn = q[0] if isinstance(q, list) else q["name"]
            for k in ("wino_in", "wino_gemm", "wino_out"):
                if qn.startswith(k + " "):
                    sub[k] = q if isinstance(q, list) else (q["name"], q["flops"], q["bytes"], q["ms"])
        if len(sub) < 3:
            continue
        roof = roof_of(name)
        fx, gms = sub["wino_gemm"][1], sub["wino_gemm"][3]
        tms = sub["wino_in"][3] + sub["wino_out"][3]
        tby = sub["wino_in"][2] + sub["wino_out"][2]
        wrows.append(f"| {i} | `{name.split(' ')[0]}` {name.split(' ')[1]} | {fl / 1e9:.2f} | {fx / 1e9:.2f} | "
                     f"{ms * 1e3:.1f} | {fx / ms / 1e9 / (roof / 1e12):.2f} | {gms * 1e3:.1f} | "
                     f"{fx / gms / 1e9:.1f} | {fx / gms / 1e9 / (roof / 1e12):.2f} | {sub['wino_gemm'][2] / 1e6:.1f} | "
                     f"{sub['wino_in'][3] * 1e3:.1f} | {sub['wino_out'][3] * 1e3:.1f} | {tby / 1e6:.1f} | "
                     f"{tby / tms / 1e6:.0f} | {(sub['wino_in'][2] + sub['wino_gemm'][2] + sub['wino_out'][2]) / 1e6:.1f} |")
    if wrows:
        out += ["", "Winograd forms on their executed work (the GEMMs' FLOPs; the transforms' and GEMMs' algorithmic bytes):", "",
                "| # | conv | direct GFLOP | executed GFLOP | bracket us | frac executed (bracket) | GEMM us | GEMM TF/s "
                "| GEMM frac executed | GEMM MB | in-transform us | out-transform us | transforms MB | transforms GB/s "
                "| executed MB total |",
                "|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|"] + wrows
    out.append("")
    hdr = "| record (kernel, tile, stage) | launches | us | floor us | frac |"
    sep = "|---|---|---|---|---|"
    if pmc:
        hdr += " PMC launches | traffic MB / launch | algorithmic MB / launch | MFMA busy | VALU / MFMA insts | LDS insts / MFMA | wave wait |"
        sep += "---|---|---|---|---|---|---|"
    out += [hdr, sep]
    for k, (n, us, fl, by) in sorted(groups.items(), key=lambda kv: -kv[1][1]):
        row = f"| `{k}` | {n} | {us:.1f} | {fl:.1f} | {fl / us:.2f} |"
        if pmc:
            key = pmc_key(k)
            hits = pmc_lookup(pmc, key) if key else []
            if hits:
                # the wave-layout forms of one tile and stage are separate instantiations: their
                # launch-weighted average
                n_l = sum(h.get("launches", 1) for h in hits)
                e = {c: sum(h.get(c, 0) * h.get("launches", 1) for h in hits) / n_l
                     for c in set().union(*hits) if c != "launches"}
                e["launches"] = n_l
                tr = e.get("traffic_bytes")
                mf = e.get("SQ_INSTS_MFMA") or 0
                # MFMA busy share of the SIMD-cycles of the dispatch: GRBM_GUI_ACTIVE sums the 8 XCDs'
                # busy cycles (MI355X_MICROARCH.md DVFS note), 1024 SIMDs
                busy = (e.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (e["GRBM_GUI_ACTIVE"] / 8 * 1024)
                        if e.get("GRBM_GUI_ACTIVE") else None)
                row += (f" {int(e.get('launches', 0))} | {tr / 1e6 if tr else float('nan'):.1f} | {by / n / 1e6:.1f} | "
                        f"{busy if busy is not None else float('nan'):.2f} | "
                        f"{(e.get('SQ_INSTS_VALU', 0) / mf) if mf else float('nan'):.2f} | "
                        f"{(e.get('SQ_INSTS_LDS', 0) / mf) if mf else float('nan'):.2f} | "
                        f"{(e.get('SQ_WAIT_ANY', 0) / e['SQ_WAVE_CYCLES']) if e.get('SQ_WAVE_CYCLES') else float('nan'):.2f} |")
            else:
                row += " - | - | - | - | - | - | - |"
        out.append(row)
    print("\n".join(out))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof.json", sys.argv[2] if len(sys.argv) > 2 else None)

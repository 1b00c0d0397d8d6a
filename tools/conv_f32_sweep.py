"""Time the exact-fp32 conv (conv_igemm_f32 via cwt_debug_conv) over every tile / split-K plan
for each distinct conv shape of the extractor, beside the automatic plan the library picks
today (the measured table conv_plans_f32.inc, else plan_conv's heuristic).  Writes
gpurun_out/<out>; tools/gen_plan_table.py --f32 turns it into conv_plans_f32.inc.

    python tools/conv_f32_sweep.py [--configs 50:473:2] [--only l3c2,bottleneck]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from few_shot_seg_cwt_amd import _lib  # noqa: E402
from conv_s_sweep import shapes, timed  # noqa: E402

TILES = [(128, 128), (128, 64), (64, 64)]


def sweep(layers, size, n_img, reps, only=None):
    print(f"== f32 R{layers} S={size} N={n_img}", flush=True)
    dev = torch.device("cuda", 0)
    lib, ctx, sp = _lib.lib(), _lib.ctx(0), _lib.stream_ptr()
    res_all, tot_auto, tot_best = [], 0.0, 0.0
    for name, cnt, Ci, Co, Hi, k, stride, dil, has_res in shapes(layers, size, n_img):
        if only and name not in only:
            continue
        pad = dil if k == 3 else 0
        Ho = (Hi + 2 * pad - dil * (k - 1) - 1) // stride + 1
        M, K = n_img * Ho * Ho, Ci * k * k
        x = torch.randn(n_img, Hi, Hi, Ci, device=dev)
        w = (torch.randn(Co, k, k, Ci, device=dev) * (2.0 / K) ** 0.5).contiguous()
        sc = torch.ones(Co, device=dev)
        sh = torch.zeros(Co, device=dev)
        r = torch.randn(n_img, Ho, Ho, Co, device=dev) if has_res else None
        y = torch.empty(n_img, Ho, Ho, Co, device=dev)
        flops = 2.0 * M * Co * K

        def new(bm, bn, ns):
            return lambda: _lib.check(lib.cwt_debug_conv(
                ctx, _lib.ptr(x), n_img, Hi, Hi, Ci, Ci, _lib.ptr(w), _lib.ptr(sc), _lib.ptr(sh), Co, k, stride,
                pad, dil, _lib.ptr(r), Co, 1, _lib.ptr(y), Co, 0, bm, bn, ns, 0, sp))

        t_auto = timed(new(0, 0, 0), reps)
        rows = []
        for bm, bn in TILES:
            if Co % bn:
                continue
            tiles = -(-M // bm) * (Co // bn)
            for ns in (1, 2, 3, 4, 6, 8):
                if ns > 1 and ((K // 32) // ns < 4 or tiles * ns > 4096):
                    continue
                us = timed(new(bm, bn, ns), reps)
                rows.append({"bm": bm, "bn": bn, "ns": ns, "var": 0, "us": round(us, 2),
                             "tflops": round(flops / us / 1e6, 1)})
        best = min(rows, key=lambda q: q["us"])
        tot_auto += cnt * t_auto
        tot_best += cnt * best["us"]
        print(f"{name:10s} x{cnt:2d} {Ci:4d}->{Co:4d} k{k} @{Ho:3d} M={M:6d} K={K:6d}: "
              f"auto {t_auto:7.1f} ({flops / t_auto / 1e6:6.1f} TF)  best "
              f"{best['bm']}x{best['bn']}s{best['ns']} {best['us']:7.1f} ({best['tflops']:6.1f} TF)", flush=True)
        res_all.append({"cfg": f"{layers}:{size}:{n_img}", "prec": 0, "name": name, "count": cnt, "Ci": Ci, "Co": Co,
                        "k": k, "Ho": Ho, "M": M, "K": K, "stride": stride, "dil": dil, "res": has_res,
                        "auto_us": round(t_auto, 2), "plans": rows})
        del x, w, r, y
    print(f"sum over the stack: auto {tot_auto:.1f} us, best {tot_best:.1f} us", flush=True)
    torch.cuda.empty_cache()
    return res_all


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="50:473:2")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--out", default="conv_f32_sweep.json")
    ap.add_argument("--only", default="", help="comma list of shape names (default: all)")
    args = ap.parse_args()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    res_all = []
    for cfg in args.configs.split(","):
        L, S, N = (int(v) for v in cfg.split(":"))
        res_all += sweep(L, S, N, args.reps, set(filter(None, args.only.split(","))))
        with open(os.path.join(ROOT, "gpurun_out", args.out), "w") as f:
            json.dump(res_all, f, indent=1)


if __name__ == "__main__":
    main()

"""Time every applicable bf16x3 tile / split-K plan for each distinct conv shape of the
ResNet-50 PSPNet extractor at 473x473, N=2 (support + query), with the weights pre-split
(cwt_debug_conv precision 2), against the automatic plan.  Writes gpurun_out/conv_sweep.json.

    python tools/conv_sweep.py [--layers 50] [--size 473] [--n 2]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from few_shot_seg_cwt_amd import _lib  # noqa: E402

TILES = [(256, 256), (256, 128), (128, 128), (128, 64), (64, 128), (64, 64)]


def shapes(layers, S, N):
    """(name, count, Ci, Co, Hi, k, stride, dil, res) of the implicit-GEMM convs (run_extract)."""
    d2 = lambda x: (x - 1) // 2 + 1  # noqa: E731
    Hs = d2(S)
    H1 = d2(Hs)
    h = d2(H1)
    out = [("stem2", 1, 64, 64, Hs, 3, 1, 1, False), ("stem3", 1, 64, 128, Hs, 3, 1, 1, False)]
    nb = [3, 4, 6, 3] if layers == 50 else [3, 4, 23, 3]
    inpl, H = 128, H1
    for li, planes in enumerate([64, 128, 256, 512]):
        for bi in range(nb[li]):
            s2 = 2 if (li == 1 and bi == 0) else 1
            d = [1, 1, 2, 4][li]
            Ho = d2(H) if s2 == 2 else H
            out.append((f"l{li+1}c1", 1, inpl, planes, H, 1, 1, 1, False))
            out.append((f"l{li+1}c2", 1, planes, planes, H, 3, s2, d, False))
            if bi == 0:
                out.append((f"l{li+1}down", 1, inpl, planes * 4, H, 1, s2, 1, False))
            out.append((f"l{li+1}c3", 1, planes, planes * 4, Ho, 1, 1, 1, True))
            inpl, H = planes * 4, Ho
    out.append(("bottleneck", 1, 2048, 512, h, 3, 1, 1, True))
    merged = {}
    for s in out:
        key = s[2:]
        if key in merged:
            merged[key][1] += 1
        else:
            merged[key] = [s[0], 1]
    return [(v[0], v[1]) + k for k, v in merged.items()]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="50:473:2", help="comma list of layers:size:n")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--out", default="conv_sweep.json")
    args = ap.parse_args()
    res_all = []
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    for cfg in args.configs.split(","):
        L, S, N = (int(v) for v in cfg.split(":"))
        res_all += sweep(L, S, N, args.reps)
        with open(os.path.join(ROOT, "gpurun_out", args.out), "w") as f:  # after every config
            json.dump(res_all, f, indent=1)


def sweep(layers, size, n_img, reps):
    class A:
        pass
    args = A()
    args.layers, args.size, args.n, args.reps = layers, size, n_img, reps
    print(f"== R{layers} S={size} N={n_img}", flush=True)
    dev = torch.device("cuda", 0)
    lib, ctx = _lib.lib(), _lib.ctx(0)
    res_all = []
    total_auto = total_best = 0.0
    for name, cnt, Ci, Co, Hi, k, stride, dil, has_res in shapes(args.layers, args.size, args.n):
        pad = dil if k == 3 else 0
        Ho = (Hi + 2 * pad - dil * (k - 1) - 1) // stride + 1
        M, K = args.n * Ho * Ho, Ci * k * k
        x = torch.randn(args.n, Hi, Hi, Ci, device=dev)
        w = torch.randn(Co, K, device=dev) * (2.0 / K) ** 0.5
        hi = w.to(torch.bfloat16)
        lo = (w - hi.float()).to(torch.bfloat16)
        wsplit = torch.cat([hi.flatten(), lo.flatten()]).contiguous()
        sc = torch.ones(Co, device=dev)
        sh = torch.zeros(Co, device=dev)
        r = torch.randn(args.n, Ho, Ho, Co, device=dev) if has_res else None
        y = torch.empty(args.n, Ho, Ho, Co, device=dev)
        flops = 2.0 * M * Co * K

        def run(bm, bn, ns):
            rc = lib.cwt_debug_conv(ctx, _lib.ptr(x), args.n, Hi, Hi, Ci, Ci, _lib.ptr(wsplit), _lib.ptr(sc),
                                    _lib.ptr(sh), Co, k, stride, pad, dil, _lib.ptr(r), Co, 1, _lib.ptr(y), Co, 0,
                                    bm, bn, ns, 2, _lib.stream_ptr())
            _lib.check(rc, "cwt_debug_conv")

        def timed(bm, bn, ns):
            run(bm, bn, ns)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                run(bm, bn, ns)
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / args.reps * 1e3  # us

        rows = []
        t_auto = timed(0, 0, 0)
        for bm, bn in TILES:
            if Co % bn:
                continue
            tiles = -(-M // bm) * (Co // bn)
            for ns in (1, 2, 4, 8):
                if ns > 1 and (K // 32) // ns < 4:
                    continue
                if ns > 1 and tiles * ns > 4096:
                    continue
                us = timed(bm, bn, ns)
                rows.append({"bm": bm, "bn": bn, "ns": ns, "us": round(us, 2), "tflops": round(flops / us / 1e6, 1)})
        best = min(rows, key=lambda q: q["us"])
        total_auto += cnt * t_auto
        total_best += cnt * best["us"]
        print(f"{name:10s} x{cnt:2d} {Ci:4d}->{Co:4d} k{k} @{Ho:3d} M={M:6d} K={K:6d}: auto {t_auto:8.1f} us "
              f"({flops / t_auto / 1e6:6.1f} TF)  best {best['bm']}x{best['bn']}s{best['ns']} {best['us']:8.1f} us "
              f"({best['tflops']:6.1f} TF)", flush=True)
        res_all.append({"cfg": f"{layers}:{size}:{n_img}", "name": name, "count": cnt, "Ci": Ci, "Co": Co, "k": k, "Ho": Ho, "M": M, "K": K,
                        "stride": stride, "dil": dil, "res": has_res, "auto_us": round(t_auto, 2), "plans": rows})
        del x, w, hi, lo, wsplit, r, y
    print(f"sum over the stack: auto {total_auto:.1f} us, best-per-shape {total_best:.1f} us", flush=True)
    torch.cuda.empty_cache()
    return res_all


if __name__ == "__main__":
    main()

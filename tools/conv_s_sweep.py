"""Time the split-activation conv (conv_x3s, cwt_debug_conv_s) over every tile / split-K plan
for each distinct conv shape of the extractor, beside the current bf16x3 conv's automatic plan
(cwt_debug_conv precision 2).  Writes gpurun_out/<out>.

    python tools/conv_s_sweep.py [--configs 50:473:2] [--quick]
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
from conv_sweep import shapes  # noqa: E402

TILES = [(256, 256), (256, 128), (128, 256), (128, 128), (128, 64), (64, 128), (64, 64)]


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def sweep(layers, size, n_img, reps, quick, prec=3):
    print(f"== R{layers} S={size} N={n_img}", flush=True)
    dev = torch.device("cuda", 0)
    lib, ctx, sp = _lib.lib(), _lib.ctx(0), _lib.stream_ptr()
    res_all, tot_old, tot_auto, tot_best = [], 0.0, 0.0, 0.0
    for name, cnt, Ci, Co, Hi, k, stride, dil, has_res in shapes(layers, size, n_img):
        pad = dil if k == 3 else 0
        Ho = (Hi + 2 * pad - dil * (k - 1) - 1) // stride + 1
        M, K = n_img * Ho * Ho, Ci * k * k
        x = torch.randn(n_img, Hi, Hi, Ci, device=dev)
        w = torch.randn(Co, k, k, Ci, device=dev) * (2.0 / K) ** 0.5
        wp = torch.empty(Co * K, device=dev)
        if prec == 1:   # plain bf16 operands (K order inside a row does not matter for timing)
            xs = x.to(torch.bfloat16).contiguous()
            ws = w.reshape(Co, K).to(torch.bfloat16).contiguous()
        else:
            xs = torch.empty(n_img * Hi * Hi * Ci * 2, dtype=torch.bfloat16, device=dev)
            ws = torch.empty(Co * K * 2, dtype=torch.bfloat16, device=dev)
            _lib.check(lib.cwt_debug_split_act(ctx, _lib.ptr(x), n_img * Hi * Hi, Ci, Ci, _lib.ptr(xs), sp))
            _lib.check(lib.cwt_debug_pack_wsplit(ctx, _lib.ptr(w), Co, k, Ci, _lib.ptr(ws), sp))
        # old path: weights pre-split hi[Co][K] ++ lo[Co][K] (order within K does not matter for timing)
        wf = w.reshape(Co, K)
        hi = wf.to(torch.bfloat16)
        lo = (wf - hi.float()).to(torch.bfloat16)
        wsplit_old = torch.cat([hi.flatten(), lo.flatten()]).contiguous()
        sc = torch.ones(Co, device=dev)
        sh = torch.zeros(Co, device=dev)
        r = torch.randn(n_img, Ho, Ho, Co, device=dev) if has_res else None
        rs = None
        if has_res and prec == 1:
            rs = r.to(torch.bfloat16).contiguous()
        elif has_res:
            rs = torch.empty(M * Co * 2, dtype=torch.bfloat16, device=dev)
            _lib.check(lib.cwt_debug_split_act(ctx, _lib.ptr(r), M, Co, Co, _lib.ptr(rs), sp))
        y = torch.empty(n_img, Ho, Ho, Co, device=dev)
        ys = torch.empty(M * Co * (1 if prec == 1 else 2), dtype=torch.bfloat16, device=dev)
        flops = 2.0 * M * Co * K

        def old():
            _lib.check(lib.cwt_debug_conv(ctx, _lib.ptr(x), n_img, Hi, Hi, Ci, Ci, _lib.ptr(wsplit_old),
                                          _lib.ptr(sc), _lib.ptr(sh), Co, k, stride, pad, dil, _lib.ptr(r), Co, 1,
                                          _lib.ptr(y), Co, 0, 0, 0, 0, 2, sp))

        conv_fn = lib.cwt_debug_conv_b16 if prec == 1 else lib.cwt_debug_conv_s

        def new(bm, bn, ns):
            return lambda: _lib.check(conv_fn(
                ctx, _lib.ptr(xs), n_img, Hi, Hi, Ci, _lib.ptr(ws), _lib.ptr(sc), _lib.ptr(sh), Co, k, stride, pad,
                dil, None, Co, _lib.ptr(rs), 1, None, Co, 0, _lib.ptr(ys), bm, bn, ns, sp))

        t_old = timed(old, reps) if prec == 3 else float("nan")
        t_auto = timed(new(0, 0, 0), reps)
        rows = []
        if not quick:
            for bm, bn in TILES:
                if Co % bn:
                    continue
                tiles = -(-M // bm) * (Co // bn)
                for ns in (1, 2, 4, 8):
                    if ns > 1 and ((K // (64 if prec == 1 else 32)) // ns < 4 or tiles * ns > 4096):
                        continue
                    us = timed(new(bm, bn, ns), reps)
                    rows.append({"bm": bm, "bn": bn, "ns": ns, "us": round(us, 2),
                                 "tflops": round(flops / us / 1e6, 1)})
        best = min(rows, key=lambda q: q["us"]) if rows else {"bm": 0, "bn": 0, "ns": 0, "us": t_auto,
                                                                  "tflops": flops / t_auto / 1e6}
        tot_old += cnt * t_old
        tot_auto += cnt * t_auto
        tot_best += cnt * best["us"]
        print(f"{name:10s} x{cnt:2d} {Ci:4d}->{Co:4d} k{k} @{Ho:3d} M={M:6d} K={K:6d}: old {t_old:7.1f} us "
              f"({flops / t_old / 1e6:6.1f} TF)  new-auto {t_auto:7.1f} ({flops / t_auto / 1e6:6.1f} TF)  best "
              f"{best['bm']}x{best['bn']}s{best['ns']} {best['us']:7.1f} ({best['tflops']:6.1f} TF)", flush=True)
        res_all.append({"cfg": f"{layers}:{size}:{n_img}", "prec": prec, "name": name, "count": cnt, "Ci": Ci, "Co": Co, "k": k,
                        "Ho": Ho, "M": M, "K": K, "stride": stride, "dil": dil, "res": has_res,
                        "old_us": round(t_old, 2), "auto_us": round(t_auto, 2), "plans": rows})
        del x, w, wp, xs, ws, wsplit_old, r, rs, y, ys
    print(f"sum over the stack: old {tot_old:.1f} us, new auto {tot_auto:.1f} us, new best {tot_best:.1f} us",
          flush=True)
    torch.cuda.empty_cache()
    return res_all


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="50:473:2")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--quick", action="store_true", help="old vs new automatic plan only")
    ap.add_argument("--out", default="conv_s_sweep.json")
    ap.add_argument("--prec", type=int, default=3, choices=[1, 3], help="3 = bf16x3 (x3s), 1 = plain bf16 (b16)")
    args = ap.parse_args()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    res_all = []
    for cfg in args.configs.split(","):
        L, S, N = (int(v) for v in cfg.split(":"))
        res_all += sweep(L, S, N, args.reps, args.quick, args.prec)
        with open(os.path.join(ROOT, "gpurun_out", args.out), "w") as f:
            json.dump(res_all, f, indent=1)


if __name__ == "__main__":
    main()

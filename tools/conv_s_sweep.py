"""Time the split-activation conv (conv_x3s, cwt_debug_conv_s) over every tile / split-K /
main-loop-variant plan for each distinct conv shape of the extractor, beside the automatic plan
the library picks today.  Writes gpurun_out/<out>.

    python tools/conv_s_sweep.py [--configs 50:473:2] [--vars 0,1,2] [--only l3c2,l3c1] [--quick]
"""
import argparse
import json
import os
import sys

import torch

# the debug conv entries split / transform the weights per call unless asked to cache them: the
# timed calls are then the conv alone (as the extractor runs it, on weights split at load)
os.environ.setdefault("CWT_DBG_W3_CACHE", "1")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from few_shot_seg_cwt_amd import _lib  # noqa: E402


def shapes(layers, S, N):
    """(name, count, Ci, Co, Hi, k, stride, dil, res) of the implicit-GEMM convs of one
    extractor pass (api.hip run_extract; resnet.py:57-96 blocks with pspnet.py:124-129's
    dilation surgery, the PPM-folded bottleneck conv), identical shapes merged."""
    if layers == 0:   # the variant heads' GEMMs as 1x1 convs over an S x S map (MMN WeightAverage
        # theta|phi|g and conv_back, forward and the backward's row-major products; config 0:60:1)
        return [("wa4_tpg", 1, 2048, 3072, S, 1, 1, 1, False), ("wa4_back", 1, 1024, 2048, S, 1, 1, 1, True),
                ("wa3_tpg", 1, 1024, 1536, S, 1, 1, 1, False), ("wa3_back", 1, 512, 1024, S, 1, 1, 1, True),
                ("wa4_dwavg", 1, 2048, 1024, S, 1, 1, 1, False), ("wa4_dx", 1, 3072, 2048, S, 1, 1, 1, True),
                ("wa3_dwavg", 1, 1024, 512, S, 1, 1, 1, False), ("wa3_dx", 1, 1536, 1024, S, 1, 1, 1, True)]
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

TILES = [(256, 256), (256, 128), (128, 256), (128, 128), (128, 64), (64, 128), (64, 64)]


OCCUPY = 0   # --occupy: CUs held by cwt_debug_occupy on a side stream while each plan is timed
_SIDE = []   # that side stream, created once (a new stream per timing can land on the timed stream's
             # hardware queue, which serialises the blocker before the timed calls)


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if OCCUPY:
        # the pipeline's condition: the resident inner loop holds OCCUPY whole CUs (its 133 KB of LDS
        # leave no room for a conv workgroup); a blocker holds them for longer than the timed calls
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        us = int(min(100000, e0.elapsed_time(e1) * 1e3 * reps * 10 + 3000))
        if not _SIDE:
            _SIDE.append(torch.cuda.Stream())
        side = _SIDE[0]
        eb = torch.cuda.Event(enable_timing=True)
        _lib.check(_lib.lib().cwt_debug_occupy(_lib.ctx(0), OCCUPY, us, side.cuda_stream))
        eb.record(side)
        # ~1 ms on this stream: the blocker's workgroups land, and every timed call is queued before
        # the first one runs (the timing is the GPU's, not the host's submission rate)
        torch.cuda._sleep(2000000)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    if OCCUPY and e0.elapsed_time(eb) <= e0.elapsed_time(e1):
        print(f"  (blocker ended before the timed calls: {e0.elapsed_time(eb):.3f} vs {e0.elapsed_time(e1):.3f} ms; "
              "plan not counted)", flush=True)
        return float("inf")
    return e0.elapsed_time(e1) / reps * 1e3


def sweep(layers, size, n_img, reps, quick, prec=3, variants=(0,), only=None):
    print(f"== R{layers} S={size} N={n_img}", flush=True)
    dev = torch.device("cuda", 0)
    lib, ctx, sp = _lib.lib(), _lib.ctx(0), _lib.stream_ptr()
    res_all, tot_auto, tot_best = [], 0.0, 0.0
    for name, cnt, Ci, Co, Hi, k, stride, dil, has_res in shapes(layers, size, n_img):
        if only and name not in only:
            continue
        if prec in (7, 8) and (k != 3 or stride != 1 or Ci < 128):
            continue   # the Winograd form's candidates: stride-1 3x3 layers with Ci >= 128 (used at >= 256)
        pad = dil if k == 3 else 0
        Ho = (Hi + 2 * pad - dil * (k - 1) - 1) // stride + 1
        M, K = n_img * Ho * Ho, Ci * k * k
        x = torch.randn(n_img, Hi, Hi, Ci, device=dev)
        w = torch.randn(Co, k, k, Ci, device=dev) * (2.0 / K) ** 0.5
        wp = torch.empty(Co * K, device=dev)
        if prec == 1:   # plain bf16 operands (K order inside a row does not matter for timing)
            xs = x.to(torch.bfloat16).contiguous()
            ws = w.reshape(Co, K).to(torch.bfloat16).contiguous()
        elif prec in (0, 6, 7, 8):  # exact fp32 (f32d) / bf16x6 (x6, x6 Winograd): fp32 NHWC and fp32 [Co][K]
            xs = x
            ws = w.reshape(Co, K).contiguous()
        else:
            xs = torch.empty(n_img * Hi * Hi * Ci * 2, dtype=torch.bfloat16, device=dev)
            ws = torch.empty(Co * K * 2, dtype=torch.bfloat16, device=dev)
            _lib.check(lib.cwt_debug_split_act(ctx, _lib.ptr(x), n_img * Hi * Hi, Ci, Ci, _lib.ptr(xs), sp))
            _lib.check(lib.cwt_debug_pack_wsplit(ctx, _lib.ptr(w), Co, k, Ci, _lib.ptr(ws), sp))
        sc = torch.ones(Co, device=dev)
        sh = torch.zeros(Co, device=dev)
        r = torch.randn(n_img, Ho, Ho, Co, device=dev) if has_res else None
        rs = None
        if has_res and prec in (0, 6, 7, 8):
            rs = None
        elif has_res and prec == 1:
            rs = r.to(torch.bfloat16).contiguous()
        elif has_res:
            rs = torch.empty(M * Co * 2, dtype=torch.bfloat16, device=dev)
            _lib.check(lib.cwt_debug_split_act(ctx, _lib.ptr(r), M, Co, Co, _lib.ptr(rs), sp))
        y = torch.empty(n_img, Ho, Ho, Co, device=dev)
        ys = torch.empty(M * Co * (1 if prec == 1 else 2), dtype=torch.bfloat16, device=dev)
        flops = 2.0 * M * Co * K

        conv_fn = lib.cwt_debug_conv_b16 if prec == 1 else lib.cwt_debug_conv_s

        def new(bm, bn, ns):
            if prec in (0, 6, 7, 8):
                fn = {0: lib.cwt_debug_conv_f32d, 6: lib.cwt_debug_conv_x6, 7: lib.cwt_debug_conv_x6w,
                      8: lib.cwt_debug_conv_x6w}[prec]
                if prec in (7, 8):   # the Winograd entry's nsplit argument is its output tile
                    ns = 4 if prec == 8 else 2
                return lambda: _lib.check(fn(
                    ctx, _lib.ptr(xs), n_img, Hi, Hi, Ci, _lib.ptr(ws), _lib.ptr(sc), _lib.ptr(sh), Co, k, stride,
                    pad, dil, _lib.ptr(r), Co, 1, _lib.ptr(y), Co, 0, bm, bn, ns, sp))
            return lambda: _lib.check(conv_fn(
                ctx, _lib.ptr(xs), n_img, Hi, Hi, Ci, _lib.ptr(ws), _lib.ptr(sc), _lib.ptr(sh), Co, k, stride, pad,
                dil, None, Co, _lib.ptr(rs), 1, None, Co, 0, _lib.ptr(ys), bm, bn, ns, sp))

        t_auto = timed(new(0, 0, 0), reps)
        rows = []
        if not quick:
            for bm, bn in TILES:
                if Co % bn:
                    continue
                tiles = -(-M // bm) * (Co // bn)
                for var in variants:
                    x6v = prec in (6, 7, 8)
                    if var == 3 and not (x6v and ((bm >= 128 and bn >= 128) or (bm, bn) in ((64, 128), (128, 64), (64, 64)))):
                        continue   # x6 only: the 4x1 / WN = 128 wave layouts
                    if var == 5 and not (x6v and (bm, bn) in ((128, 128), (64, 128), (128, 64))):
                        continue   # x6 only: 4x1 waves on a 2-stage ring
                    if var in (1, 2) and bm == 256 and bn == 256:
                        continue   # no prefetch form of 256x256
                    if var == 4 and (bm, bn) != (128, 128):
                        continue   # two-workgroups-per-CU 128x128 form
                    if 8 <= var < 18 and (bm, bn) != ((64, 64) if var < 10 else (128, 128)):
                        continue   # timing-study kernels: fixed tiles
                    if var == 2 and (bm == 256 or bn == 256):
                        continue   # 8-wave form only for the 128/64 tiles
                    for ns in (1, 2, 4, 8):
                        if ns > 1 and (prec in (7, 8) or (K // (64 if prec == 1 else 32)) // ns < 4 or tiles * ns > 4096):
                            continue
                        us = timed(new(1000 * var + bm, bn, ns), reps)
                        rows.append({"bm": bm, "bn": bn, "ns": ns, "var": var, "us": round(us, 2),
                                     "tflops": round(flops / us / 1e6, 1)})
        best = min(rows, key=lambda q: q["us"]) if rows else {"bm": 0, "bn": 0, "ns": 0, "var": 0, "us": t_auto,
                                                                  "tflops": flops / t_auto / 1e6}
        tot_auto += cnt * t_auto
        tot_best += cnt * best["us"]
        print(f"{name:10s} x{cnt:2d} {Ci:4d}->{Co:4d} k{k} @{Ho:3d} M={M:6d} K={K:6d}: "
              f"auto {t_auto:7.1f} ({flops / t_auto / 1e6:6.1f} TF)  best "
              f"{best['bm']}x{best['bn']}s{best['ns']}v{best['var']} {best['us']:7.1f} ({best['tflops']:6.1f} TF)",
              flush=True)
        batch = 0
        if prec in (7, 8):   # the plan table keys the batched GEMMs by (tiles, Co, Ci, batch)
            d_, m_ = dil, (2 if prec == 7 else 4)
            TY = (-(-Ho // d_) + m_ - 1) // m_
            M, K, batch = n_img * d_ * d_ * TY * TY, Ci, (m_ + 2) ** 2
        res_all.append({"cfg": f"{layers}:{size}:{n_img}", "prec": prec, "name": name, "count": cnt, "Ci": Ci, "Co": Co, "k": k,
                        "Ho": Ho, "M": M, "K": K, "batch": batch, "stride": stride, "dil": dil, "res": has_res,
                        "auto_us": round(t_auto, 2), "plans": rows})
        del x, w, wp, xs, ws, r, rs, y, ys
    print(f"sum over the stack: auto {tot_auto:.1f} us, best {tot_best:.1f} us", flush=True)
    torch.cuda.empty_cache()
    return res_all


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="50:473:2")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--quick", action="store_true", help="old vs new automatic plan only")
    ap.add_argument("--out", default="conv_s_sweep.json")
    ap.add_argument("--prec", type=int, default=3, choices=[0, 1, 3, 6, 7, 8],
                    help="3 = bf16x3 (x3s), 1 = plain bf16 (b16), 0 = exact fp32 on the LDS-DMA body (f32d), "
                         "6 = fp32 width on bf16 MFMA (x6), 7 = x6 in the Winograd F(2x2,3x3) form (x6w), "
                         "8 = x6 in the Winograd F(4x4,3x3) form (x6w4)")
    ap.add_argument("--vars", default="0,1,2,4", help="main-loop variants (0 base, 1 prefetch, 2 prefetch 8 waves, 4 128x128 two per CU; 8-15 timing "
                         "studies; x6: 3 / 5 WN = 128 layouts)")
    ap.add_argument("--only", default="", help="comma list of shape names (default: all)")
    ap.add_argument("--occupy", type=int, default=0,
                    help="time every plan while this many CUs are held (the pipeline's resident inner loop: 59)")
    args = ap.parse_args()
    global OCCUPY
    OCCUPY = args.occupy
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    res_all = []
    for cfg in args.configs.split(","):
        L, S, N = (int(v) for v in cfg.split(":"))
        res_all += sweep(L, S, N, args.reps, args.quick, args.prec,
                         tuple(int(v) for v in args.vars.split(",")), set(filter(None, args.only.split(","))))
        with open(os.path.join(ROOT, "gpurun_out", args.out), "w") as f:
            json.dump(res_all, f, indent=1)


if __name__ == "__main__":
    main()

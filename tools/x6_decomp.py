"""Timing decomposition of the x6 direct conv (conv_igemm_x6, 128x128 tile, 4x1 waves, two-stage
ring: var 5) on the extractor's 1x1 shapes: the full kernel against the timing-study forms that
compile the same kernel without operand DMA (var 14), without MFMAs (15), without both (16) and
without both and the epilogue (17: the launch, prologue and per-K-tile barriers alone), and the
launch alone (18: every workgroup returns at once).  Weights
split once (CWT_DBG_W3_CACHE).  Writes gpurun_out/<out>.

    python tools/x6_decomp.py [--reps 50] [--only l3c3,l2c3] [--out x6_decomp.json]
"""
import argparse
import json
import os
import sys

os.environ.setdefault("CWT_DBG_W3_CACHE", "1")
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from conv_s_sweep import shapes, timed  # noqa: E402
from few_shot_seg_cwt_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--only", default="l1c1,l1c3,l2c1,l2c3,l3c1,l3c3,l3down,l4c1,l4c3")
    ap.add_argument("--vars", default="5,14,15,16,17,18")
    ap.add_argument("--out", default="x6_decomp.json")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    lib, ctx, sp = _lib.lib(), _lib.ctx(0), _lib.stream_ptr()
    only = set(args.only.split(","))
    res = []
    for name, cnt, Ci, Co, Hi, k, stride, dil, has_res in shapes(50, 473, 2):
        if name not in only or k != 1:
            continue
        Ho = (Hi - 1) // stride + 1
        M, K = 2 * Ho * Ho, Ci
        x = torch.randn(2, Hi, Hi, Ci, device=dev)
        w = (torch.randn(Co, Ci, device=dev) * (2.0 / K) ** 0.5).contiguous()
        sc, sh = torch.ones(Co, device=dev), torch.zeros(Co, device=dev)
        r = torch.randn(2, Ho, Ho, Co, device=dev) if has_res else None
        y = torch.empty(2, Ho, Ho, Co, device=dev)

        def fn(bm, bn):
            return lambda: _lib.check(lib.cwt_debug_conv_x6(
                ctx, _lib.ptr(x), 2, Hi, Hi, Ci, _lib.ptr(w), _lib.ptr(sc), _lib.ptr(sh), Co, 1, stride, 0, 1,
                _lib.ptr(r), Co, 1, _lib.ptr(y), Co, 0, bm, bn, 1 if bm else 0, sp))
        row = {"name": name, "count": cnt, "Ci": Ci, "Co": Co, "M": M, "K": K, "res": has_res,
               "gflop": 2.0 * M * Co * K / 1e9,
               "mb": 4.0 * (2 * Hi * Hi * Ci + Co * K + M * Co * (2 if has_res else 1)) / 1e6,
               "auto_us": round(timed(fn(0, 0), args.reps), 2)}
        for v in (int(s) for s in args.vars.split(",")):
            if Co % 128 == 0:
                row[f"v{v}_us"] = round(timed(fn(1000 * v + 128, 128), args.reps), 2)
        print(json.dumps(row), flush=True)
        res.append(row)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", args.out), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()

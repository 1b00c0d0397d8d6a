"""Timing study: how much of the x6 Winograd GEMMs' time is the in-register A split?  Times the
bottleneck / l4c2 / l3c2 Winograd convs (cwt_debug_conv_x6w) with the production WN = 128 forms
(var 5: 128x128 4x1 waves, var 3: 256x256 4x2) against the same kernels built without the split
(var 12 / 13: the raw fp32 bits stand in for the three terms -- wrong numbers, identical DMA,
LDS reads and MFMAs).  Writes gpurun_out/x6_split_study.json.

    python tools/x6_split_study.py
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from few_shot_seg_cwt_amd import _lib  # noqa: E402


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    dev = torch.device("cuda", 0)
    lib, ctx, sp = _lib.lib(), _lib.ctx(0), _lib.stream_ptr()
    out = []
    for name, Ci, Co, d in (("bottleneck", 2048, 512, 1), ("l4c2", 512, 512, 4), ("l3c2", 256, 256, 2)):
        N, H = 2, 60
        x = torch.randn(N, H, H, Ci, device=dev)
        w = torch.randn(Co, 9 * Ci, device=dev) * (2.0 / (9 * Ci)) ** 0.5
        sc, sh = torch.ones(Co, device=dev), torch.zeros(Co, device=dev)
        y = torch.empty(N, H, H, Co, device=dev)
        row = {"conv": name, "Ci": Ci, "Co": Co, "dil": d}
        for tag, bm, bn in (("128x128 var5", 5128, 128), ("128x128 var5 no split", 12128, 128),
                            ("256x256 var3", 3256, 256), ("256x256 var3 no split", 13256, 256)):
            fn = lambda bm=bm, bn=bn: _lib.check(lib.cwt_debug_conv_x6w(  # noqa: E731
                ctx, _lib.ptr(x), N, H, H, Ci, _lib.ptr(w), _lib.ptr(sc), _lib.ptr(sh), Co, 3, 1, d, d, None, Co, 0,
                _lib.ptr(y), Co, 0, bm, bn, 0, sp))
            row[tag] = round(timed(fn), 2)
        print(row, flush=True)
        out.append(row)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", "x6_split_study.json"), "w"), indent=1)


if __name__ == "__main__":
    main()

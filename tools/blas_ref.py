"""Reference point for the conv GEMMs: hipBLASLt (torch.matmul) bf16 GEMM time for each
distinct conv GEMM shape (M x Co x K) of the extractor, and the bf16x3-equivalent rate
(three such products per fp32 product).  Not used by the product; a ceiling check for the
hand-written conv kernels.  Writes gpurun_out/blas_ref.json."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from conv_sweep import shapes  # noqa: E402


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


dev = torch.device("cuda", 0)
out = []
for cfg in (sys.argv[1] if len(sys.argv) > 1 else "50:473:2").split(","):
    L, S, N = (int(v) for v in cfg.split(":"))
    for name, cnt, Ci, Co, Hi, k, stride, dil, has_res in shapes(L, S, N):
        pad = dil if k == 3 else 0
        Ho = (Hi + 2 * pad - dil * (k - 1) - 1) // stride + 1
        M, K = N * Ho * Ho, Ci * k * k
        a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        b = torch.randn(K, Co, device=dev, dtype=torch.bfloat16)
        us = timed(lambda: torch.matmul(a, b))
        tf = 2.0 * M * Co * K / us / 1e6
        print(f"{name:10s} M={M:6d} N={Co:5d} K={K:6d}: bf16 {us:7.1f} us {tf:7.1f} TF -> bf16x3-equiv "
              f"{3 * us:7.1f} us {tf / 3:6.1f} TF", flush=True)
        out.append({"cfg": cfg, "name": name, "M": M, "N": Co, "K": K, "bf16_us": round(us, 2), "bf16_tf": round(tf, 1)})
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(out, open(os.path.join(ROOT, "gpurun_out", "blas_ref.json"), "w"), indent=1)

"""Wall time of the inner loop alone (inner_adapt, 200 steps) for A/B runs of two library builds
in one session: CWT_LIB_PATH=tools/ab/libX.so python tools/time_adapt.py [shots] [S] [reps]."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from few_shot_seg_cwt_amd import synthetic as syn  # noqa: E402
from few_shot_seg_cwt_amd.episode import inner_adapt  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1
S = int(sys.argv[2]) if len(sys.argv) > 2 else 473
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 50
h = (S - 1) // 8 + 1
dev = torch.device("cuda", 0)
ep = syn.make_episode(2021, 0, S, n)
f = torch.from_numpy(syn.normal(2021, "f", (n, 512, h, h), 0.1)).abs().to(dev).contiguous(
    memory_format=torch.channels_last)
lbl = torch.from_numpy(ep["s_label"][0]).to(dev)   # [shots, S, S]
W = torch.zeros(2, 512, device=dev)
for _ in range(5):
    inner_adapt(f, lbl, W, 0.1, 200)
torch.cuda.synchronize()
ts = []
for _ in range(reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    Wa = inner_adapt(f, lbl, W, 0.1, 200)
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
ts.sort()
print(json.dumps({"lib": os.environ.get("CWT_LIB_PATH", "default"), "shots": n, "S": S,
                  "median_ms": round(ts[len(ts) // 2], 4), "min_ms": round(ts[0], 4),
                  "W_sum": float(Wa.double().sum())}))

"""The post-loop tail alone at the 473^2 geometry (h = 60, B = 1): the one-launch
cwt_episode_tail against the module path (cwt_attention_infer + cwt_classify_scaled +
cwt_seg_metrics_pair), event-timed, then the one-launch kernel's per-phase times from its
timing-study instantiation (CWT_TAIL_STAMPS=1, cwt_debug_tail_stamps).
    python tools/tail_stamps.py [h] [reps]"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from few_shot_seg_cwt_amd import MultiHeadAttentionOne, _lib  # noqa: E402
from few_shot_seg_cwt_amd import synthetic as syn  # noqa: E402
from few_shot_seg_cwt_amd.episode import cwt_tail, episode_tail  # noqa: E402
from few_shot_seg_cwt_amd.util import seg_metrics_pair  # noqa: E402

h = int(sys.argv[1]) if len(sys.argv) > 1 else 60
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
dev = torch.device("cuda", 0)
S = 8 * (h - 1) + 1
t = MultiHeadAttentionOne(4, 512, 512, 512, dropout=0.5)
t.load_state_dict(syn.make_transformer_state(4, 512, 2021))
t.eval()
f = torch.from_numpy(syn.normal(3, "ts", (1, 512, h, h), 1.0)).abs().to(dev).contiguous(memory_format=torch.channels_last)
W = torch.from_numpy(syn.normal(4, "tw", (1, 2, 512), 0.05)).to(dev)
ql = torch.from_numpy((syn.uniform01(9, "tl", S * S) < 0.3).astype(np.int64).reshape(1, S, S)).to(dev)


def timed(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return round(float(np.median(ts)), 1)


def modules():
    W2, pq, pq0 = cwt_tail(t, W, f)
    seg_metrics_pair(pq, pq0, ql)


out = {"h": h, "one_launch_us": timed(lambda: episode_tail(t, W, f, ql)), "modules_us": timed(modules)}
os.environ["CWT_TAIL_STAMPS"] = "1"
episode_tail(t, W, f, ql)
torch.cuda.synchronize()
n = C.c_int64()
_lib.check(_lib.lib().cwt_debug_tail_stamps(_lib.ctx(0), None, 0, C.byref(n)), "stamps")
buf = (C.c_uint64 * n.value)()
_lib.check(_lib.lib().cwt_debug_tail_stamps(_lib.ctx(0), buf, n.value, C.byref(n)), "stamps")
st = np.array(buf, dtype=np.float64).reshape(-1, 16)
clk = (st[:, 11] - st[:, 0]) / ((st[:, 15] - st[:, 14]) / 100.0)   # memtime ticks per us (realtime 100 MHz)
mhz = float(np.median(clk))
names = ["P0 r=M.q", "barrier1", "P1 tokens", "barrier2", "P2 combine", "barrier3", "P3 y=P.g", "barrier4",
         "P4 LN+classifier", "barrier5", "P5 metrics partials"]
t0 = st[:, 0].min()
phase = {}
for i, nm in enumerate(names):
    d = (st[:, i + 1] - st[:, i]) / mhz
    phase[nm] = {"median_us": round(float(np.median(d)), 2), "max_us": round(float(d.max()), 2)}
out["clock_MHz"] = round(mhz, 1)
out["phases"] = phase
out["edge_spread_us"] = {"entry": round(float((st[:, 0].max() - t0) / mhz), 2),
                         "partials_done_last": round(float((st[:, 11].max() - t0) / mhz), 2)}
print(json.dumps(out, indent=1))

"""Timing study of the persistent inner loop (adapt_persist_kernel, CWT_ADAPT_DBG=32 stamps).

Per (step, workgroup) thread 0 records s_memtime at: step start, z ready, gradient ready,
dW atomics issued, atomics performed (+ workgroup barrier), poll matched, post-poll barrier,
W updated; and realtime at its arrival and when its poll matched.  Prints mean phase durations (us) over steps 1.., the spread of barrier arrival
over workgroups, and the whole-loop time per step.

    CWT_ADAPT_DBG=32 python tools/persist_stamps.py [shots] [S]
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from few_shot_seg_cwt_amd import _lib, synthetic as syn  # noqa: E402
from few_shot_seg_cwt_amd.episode import inner_adapt  # noqa: E402

assert int(os.environ.get("CWT_ADAPT_DBG", "0")) & 32, "run with CWT_ADAPT_DBG=32"
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1
S = int(sys.argv[2]) if len(sys.argv) > 2 else 473
h = (S - 1) // 8 + 1
iters = 200
dev = torch.device("cuda", 0)
ep = syn.make_episode(2021, 0, S, n)
f = torch.from_numpy(syn.normal(2021, "f", (n, 512, h, h), 0.1)).abs().to(dev).contiguous(
    memory_format=torch.channels_last)
lbl = torch.from_numpy(ep["s_label"][0]).to(dev)
# CWT_STAMP_UNITS=2: the episode pipeline's adapt geometry (cwt_ctx_set_adapt_units; <5> at 1-shot 473^2)
if os.environ.get("CWT_STAMP_UNITS"):
    _lib.check(_lib.lib().cwt_ctx_set_adapt_units(_lib.ctx(0), int(os.environ["CWT_STAMP_UNITS"])), "units")
W = torch.zeros(2, 512, device=dev)
for _ in range(3):
    inner_adapt(f, lbl, W, 0.1, iters)
torch.cuda.synchronize()
inner_adapt(f, lbl, W, 0.1, iters)
torch.cuda.synchronize()
cnt = ctypes.c_int64()
_lib.check(_lib.lib().cwt_debug_adapt_stamps(_lib.ctx(0), None, 0, ctypes.byref(cnt)), "stamps")
buf = (ctypes.c_uint64 * cnt.value)()
_lib.check(_lib.lib().cwt_debug_adapt_stamps(_lib.ctx(0), buf, cnt.value, ctypes.byref(cnt)), "stamps")
raw = np.frombuffer(buf, dtype=np.uint64).astype(np.int64)
G = cnt.value // ((iters + 1) * 10)
st = raw[: (iters + 1) * G * 10].reshape(iters + 1, G, 10)
ends = st[iters]
rt = (ends[:, 2] - ends[:, 0]).astype(np.float64)      # 100 MHz ticks
mt = (ends[:, 3] - ends[:, 1]).astype(np.float64)
clk = float(np.median(mt / rt))                          # shader cycles per 10 ns
us = lambda c: c / clk / 100.0  # noqa: E731
body = st[1:iters]
names = ["z (d.f + partial sums)", "hi-res + gradient sum", "dW pass + atomics issued (+ other units)",
         "atomics performed", "poll until all arrived", "post-poll barrier", "replica read + W update"]
ph = {nm: round(float(us(np.mean(body[:, :, i + 1] - body[:, :, i]))), 3) for i, nm in enumerate(names)}
arr, seen = body[:, :, 8].astype(np.float64), body[:, :, 9].astype(np.float64)   # realtime, 100 MHz
ph["arrival spread over workgroups (max-min, realtime)"] = round(float(np.mean(arr.max(1) - arr.min(1))) / 100.0, 3)
ph["last arrival -> first poll match"] = round(float(np.mean(seen.min(1) - arr.max(1))) / 100.0, 3)
ph["last arrival -> last poll match"] = round(float(np.mean(seen.max(1) - arr.max(1))) / 100.0, 3)
ph["most frequent last arriver (workgroup)"] = int(np.argmax(np.bincount(np.argmax(arr, axis=1), minlength=G)))
work = us(np.mean(body[:, :, 4] - body[:, :, 0], axis=0))   # step start -> atomics performed, per workgroup
ph["step work per workgroup min/median/max"] = [round(float(x), 3) for x in (work.min(), np.median(work), work.max())]
ph["slowest workgroups"] = [int(i) for i in np.argsort(work)[-4:]]
per_wg = np.stack([us(np.mean(body[:, :, i + 1] - body[:, :, i], axis=0)) for i in range(4)], 1)   # [G, 4]
med = np.median(per_wg, axis=0)
ph["phases z/hires/dW/atomics: median workgroup"] = [round(float(x), 3) for x in med]
ph["phases z/hires/dW/atomics: slowest workgroups"] = {
    int(g): [round(float(x), 3) for x in per_wg[g]] for g in np.argsort(work)[-8:]}
ph["mean arrival rank (0 first) of the slowest workgroups"] = {
    int(g): round(float(np.mean(np.argsort(np.argsort(arr, axis=1), axis=1)[:, g])), 1) for g in np.argsort(work)[-8:]}
ph["step period"] = round(float(us(np.mean(np.diff(st[:iters, :, 0], axis=0)))), 3)
ph["loop per step (realtime)"] = round(float(np.median(rt)) / 100.0 / iters, 3)
ph["workgroups"] = G
ph["clock GHz"] = round(clk / 10.0, 3)
print(json.dumps(ph, indent=1))
out = os.path.join(ROOT, "gpurun_out")
if os.path.isdir(out):
    json.dump(ph, open(os.path.join(out, f"persist_stamps_{n}shot_{S}_u{os.environ.get('CWT_STAMP_UNITS', 0)}.json"),
                       "w"), indent=1)

"""Timing study of the inner-loop step kernel (CWT_ADAPT_DBG=32 clock stamps).

Per (step, workgroup), wave 0 records: realtime at entry, memtime at entry, before the W
barrier (its W publish done), after it, after the z barrier, after the hi-res barrier, after
the reduce barrier, after its atomic has been performed, realtime at exit.  Prints the mean
phase durations and the step-to-step timeline (launch gaps).

    CWT_ADAPT_DBG=32 python tools/adapt_stamps.py [shots]
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
dev = torch.device("cuda", 0)
ep = syn.make_episode(2021, 0, 473, n)
f = torch.from_numpy(syn.normal(2021, "f", (n, 512, 60, 60), 0.1)).abs().to(dev).contiguous(
    memory_format=torch.channels_last)
lbl = torch.from_numpy(ep["s_label"][0]).to(dev)
W = torch.zeros(2, 512, device=dev)
for _ in range(3):
    inner_adapt(f, lbl, W, 0.1, 200)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
inner_adapt(f, lbl, W, 0.1, 200)
e1.record()
torch.cuda.synchronize()
cnt = ctypes.c_int64()
_lib.check(_lib.lib().cwt_debug_adapt_stamps(_lib.ctx(0), None, 0, ctypes.byref(cnt)), "stamps")
buf = (ctypes.c_uint64 * cnt.value)()
_lib.check(_lib.lib().cwt_debug_adapt_stamps(_lib.ctx(0), buf, cnt.value, ctypes.byref(cnt)), "stamps")
st = np.frombuffer(buf, dtype=np.uint64).astype(np.int64).reshape(200, -1, 10)
rt0, mt = st[:, :, 0], st[:, :, 1:8]
rt1 = st[:, :, 8]
# cycles per realtime tick (100 MHz) from each workgroup's own entry/exit
dur_rt = (rt1 - rt0).astype(np.float64)
dur_mt = (mt[:, :, 6] - mt[:, :, 0]).astype(np.float64)
ok = dur_rt > 0
clk = float(np.median(dur_mt[ok] / dur_rt[ok]))  # shader cycles per 10 ns
us = lambda cyc: cyc / clk / 100.0  # noqa: E731
names = ["W publish (wave 0)", "W barrier", "z pass + barrier", "hi-res + barrier", "dW reduce + barrier",
         "atomic performed"]
ph = {nm: float(us(np.mean(mt[1:, :, i + 1] - mt[1:, :, i]))) for i, nm in enumerate(names)}
ph["tile-0 f/labels landed after the W barrier"] = float(us(np.mean(st[1:, :, 9] - st[1:, :, 3])))
ph["z pass after f landed (+ barrier)"] = float(us(np.mean(st[1:, :, 4] - st[1:, :, 9])))
steps = []
for s in range(1, 200):
    steps.append(dict(first_in=rt0[s].min(), last_in=rt0[s].max(), first_out=rt1[s].min(), last_out=rt1[s].max()))
gap = np.mean([(steps[i + 1]["first_in"] - steps[i]["last_out"]) / 100.0 for i in range(len(steps) - 1)])
skew = np.mean([(x["last_in"] - x["first_in"]) / 100.0 for x in steps])
span = np.mean([(x["last_out"] - x["first_in"]) / 100.0 for x in steps])
wg = np.mean(dur_rt[1:]) / 100.0
out = dict(shots=n, ms_per_loop=e0.elapsed_time(e1), us_per_step=e0.elapsed_time(e1) * 1e3 / 200,
           clock_ghz=clk / 10.0, phases_us=ph, wg_lifetime_us=wg, dispatch_skew_us=skew, step_span_us=span,
           gap_last_exit_to_next_entry_us=gap)
print(json.dumps(out, indent=1))
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(out, open(os.path.join(ROOT, "gpurun_out", f"adapt_stamps_n{n}.json"), "w"), indent=1)

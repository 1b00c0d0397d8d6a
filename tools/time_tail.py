"""Timing study of the episode tail's launches (seg_metrics forms, token pass) on synthetic
inputs: python tools/time_tail.py  (prints us per call)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from few_shot_seg_cwt_amd import MultiHeadAttentionOne  # noqa: E402
from few_shot_seg_cwt_amd import synthetic as syn  # noqa: E402
from few_shot_seg_cwt_amd.episode import cwt_tail  # noqa: E402
from few_shot_seg_cwt_amd.util import seg_metrics_pair  # noqa: E402


def timed(fn, reps=50):
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
    S, h = 473, 60
    ep = syn.make_episode(2021, 3, S, 1)
    ql = torch.from_numpy(ep["q_label"]).to(dev)
    lg = torch.randn(1, 2, h, h, device=dev)
    lg0 = torch.randn(1, 2, h, h, device=dev)
    print(f"seg_metrics_pair: {timed(lambda: seg_metrics_pair(lg, lg0, ql)):.2f} us")
    t = MultiHeadAttentionOne(4, 512, 512, 512, dropout=0.5)
    t.load_state_dict(syn.make_transformer_state(4, 512, 2021))
    f = torch.randn(1, 512, h, h, device=dev).abs().contiguous(memory_format=torch.channels_last)
    W = torch.randn(1, 2, 512, device=dev) * 0.05
    print(f"cwt_tail (infer_raw + classify_scaled): {timed(lambda: cwt_tail(t, W, f)):.2f} us")


if __name__ == "__main__":
    main()

"""Does a CU mask confine our kernels (including graph replays), and how do a masked inner
loop and a masked conv stack overlap?  Prints ms for each arm; writes gpurun_out/cu_probe.json."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from few_shot_seg_cwt_amd import _lib, get_model  # noqa: E402
from few_shot_seg_cwt_amd import synthetic as syn  # noqa: E402
from few_shot_seg_cwt_amd.episode import inner_adapt  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
S = 473
cfg = syn.cfg_defaults(image_size=S)
m = get_model(cfg)
m.load_state_dict(syn.make_pspnet_state(50, 2021))
ep = syn.make_episode(2021, 0, S, 1)
imgs = torch.from_numpy(np.concatenate([ep["spprt_imgs"][0], ep["qry_img"]])).to(dev)
lbl = torch.from_numpy(ep["s_label"][0]).to(dev)
ncu = _lib.cu_count()
print("CUs", ncu, flush=True)
f, _ = m.extract_features(imgs)
f_s = f[:1].clone(memory_format=torch.channels_last)
W = torch.zeros(2, 512, device=dev)
torch.cuda.synchronize()


def t_adapt(stream):
    with torch.cuda.stream(stream):
        inner_adapt(f_s, lbl, W, 0.1, 200)
        inner_adapt(f_s, lbl, W, 0.1, 200)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            inner_adapt(f_s, lbl, W, 0.1, 200)
        e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 5


def t_extract(stream):
    with torch.cuda.stream(stream):
        m.extract_features(imgs)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            m.extract_features(imgs)
        e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 5


out = {}
default = torch.cuda.current_stream()
out["adapt_default"] = t_adapt(default)
out["extract_default"] = t_extract(default)
per_xcd = ncu // 8
for name, cus in [("all", range(ncu)),
                  ("first32", range(32)),
                  ("strided32", [x * per_xcd + i for x in range(8) for i in range(4)]),
                  ("strided64", [x * per_xcd + i for x in range(8) for i in range(8)])]:
    ms = _lib.MaskedStream(list(cus))
    out[f"adapt_{name}"] = t_adapt(ms.torch)
    print(name, "adapt ms", round(out[f"adapt_{name}"], 3), flush=True)
    if name.startswith("strided"):
        comp = [c for c in range(ncu) if c not in set(cus)]
        cs = _lib.MaskedStream(comp)
        out[f"extract_complement_{name}"] = t_extract(cs.torch)
        # concurrent: adapt on the partition, extract on the complement
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            with torch.cuda.stream(ms.torch):
                inner_adapt(f_s, lbl, W, 0.1, 200)
            with torch.cuda.stream(cs.torch):
                m.extract_features(imgs)
        torch.cuda.synchronize()
        out[f"concurrent_{name}"] = (time.perf_counter() - t0) * 1e3 / 5
        print(name, "extract on complement", round(out[f"extract_complement_{name}"], 3),
              "concurrent pair", round(out[f"concurrent_{name}"], 3), flush=True)
print(json.dumps(out, indent=1), flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(out, open(os.path.join(ROOT, "gpurun_out", "cu_probe.json"), "w"), indent=1)

"""Which physical CU does CU-mask bit i select?  For each bit, a census grid on a stream masked
to that single bit records HW_REG_HW_ID / HW_REG_XCC_ID; prints the bit -> (xcc, se, sh, cu)
map and writes gpurun_out/cu_census.json.  Then times an extract + inner-loop pair on two
unmasked streams against the sequential order (can the latency-bound inner loop share the chip
with a conv stack without a partition?)."""
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


def decode(hw, xcc):
    return {"xcc": xcc & 0xF, "se": (hw >> 13) & 0x7, "sh": (hw >> 12) & 1, "cu": (hw >> 8) & 0xF,
            "simd": (hw >> 4) & 3}


torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
ncu = _lib.cu_count()
out = torch.zeros(2 * 64, dtype=torch.int32, device=dev)
mapping = {}
for bit in range(ncu):
    ms = _lib.MaskedStream([bit])
    _lib.check(_lib.lib().cwt_debug_census(_lib.ctx(0), 64, _lib.ptr(out), ms.ptr), "census")
    torch.cuda.synchronize()
    o = out.cpu().numpy().astype(np.uint32)
    cus = sorted({tuple(decode(int(o[2 * b]), int(o[2 * b + 1])).values())[:4] for b in range(64)})
    mapping[bit] = cus
    del ms
print("bit -> [(xcc, se, sh, cu)]")
for bit in range(0, ncu, 1):
    print(bit, mapping[bit])
json.dump({str(k): v for k, v in mapping.items()}, open(os.path.join(ROOT, "gpurun_out", "cu_census.json"), "w"))

# two unmasked streams: extract (N=2) on one, inner loop on the other
S = 473
cfg = syn.cfg_defaults(image_size=S)
m = get_model(cfg)
m.load_state_dict(syn.make_pspnet_state(50, 2021))
ep = syn.make_episode(2021, 0, S, 1)
imgs = torch.from_numpy(np.concatenate([ep["spprt_imgs"][0], ep["qry_img"]])).to(dev)
lbl = torch.from_numpy(ep["s_label"][0]).to(dev)
f, _ = m.extract_features(imgs)
f_s = f[:1].clone(memory_format=torch.channels_last)
W = torch.zeros(2, 512, device=dev)
sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
for _ in range(2):
    inner_adapt(f_s, lbl, W, 0.1, 200)
    m.extract_features(imgs)
torch.cuda.synchronize()
res = {}
for name in ("sequential", "two_streams"):
    t0 = time.perf_counter()
    for _ in range(5):
        if name == "sequential":
            m.extract_features(imgs)
            inner_adapt(f_s, lbl, W, 0.1, 200)
        else:
            with torch.cuda.stream(sa):
                m.extract_features(imgs)
            with torch.cuda.stream(sb):
                inner_adapt(f_s, lbl, W, 0.1, 200)
    torch.cuda.synchronize()
    res[name] = (time.perf_counter() - t0) * 1e3 / 5
    print(name, "ms per pair", round(res[name], 3), flush=True)
json.dump({"mapping": {str(k): v for k, v in mapping.items()}, "pair_ms": res},
          open(os.path.join(ROOT, "gpurun_out", "cu_census.json"), "w"))

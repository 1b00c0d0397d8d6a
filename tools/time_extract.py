"""Per-launch timing of one extractor pass (libcwt profile level 2, hipEvent pair per launch) on
synthetic weights / images: python tools/time_extract.py [--layers 50] [--size 473] [--n 2]
[--reps 5] [--match stem,maxpool,ppm]  -- prints the median us per named launch (all launches
whose name contains one of the --match substrings), the conv sum, and the whole pass.
Environment A/B switches (e.g. CWT_STEM_VALU=1) are read by the library at the first launch."""
import argparse
import collections
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from few_shot_seg_cwt_amd import _lib, get_model  # noqa: E402
from few_shot_seg_cwt_amd import synthetic as syn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=50)
    ap.add_argument("--size", type=int, default=473)
    ap.add_argument("--n", type=int, default=2)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--match", default="stem,maxpool,ppm")
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = syn.cfg_defaults(image_size=a.size, layers=a.layers)
    model = get_model(cfg)
    model.load_state_dict(syn.make_pspnet_state(a.layers, 2021))
    x = torch.from_numpy(syn.normal(2021, "te_img", (a.n, 3, a.size, a.size), 1.0)).to(dev)
    with torch.no_grad():
        for _ in range(3):
            model.extract_features(x)
        torch.cuda.synchronize()
        per = collections.defaultdict(list)
        conv, whole = [], []
        for _ in range(a.reps):
            _lib.profile_enable(2)
            model.extract_features(x)
            torch.cuda.synchronize()
            recs = _lib.profile_records()
            _lib.profile_enable(0)
            cs = 0.0
            for name, fl, by, ms in recs:
                if name.startswith("extract_features"):
                    whole.append(ms * 1e3)
                elif name.startswith("conv_igemm"):
                    cs += ms * 1e3
                if any(m and m in name for m in a.match.split(",")):
                    per[name].append(ms * 1e3)
            conv.append(cs)
    out = {"tag": a.tag, "layers": a.layers, "size": a.size, "n": a.n,
           "launches_us": {k: round(float(np.median(v)), 2) for k, v in per.items()},
           "conv_sum_us": round(float(np.median(conv)), 1), "extract_us": round(float(np.median(whole)), 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()

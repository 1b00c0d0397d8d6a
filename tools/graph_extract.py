"""Does a hipGraph of the extractor pass cut its per-launch overhead?  One R50 473^2 two-image pass
(~80 launches): timed directly (back-to-back passes on one stream, the host enqueueing each) and as
a captured graph replayed (torch.cuda.CUDAGraph over extract_features: libcwt launches on torch's
current stream, its workspaces allocated by the warm-up).  Also the result equality of the two.

    python tools/graph_extract.py [--reps 30]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from few_shot_seg_cwt_amd import get_model  # noqa: E402
from few_shot_seg_cwt_amd import synthetic as syn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--n", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = syn.cfg_defaults()
    model = get_model(cfg)
    model.load_state_dict(syn.make_pspnet_state(50, 2021))
    x = torch.from_numpy(syn.normal(2021, "ge_img", (a.n, 3, 473, 473), 1.0)).to(dev)
    s = torch.cuda.Stream()
    out = {}
    with torch.no_grad(), torch.cuda.stream(s):
        for _ in range(3):
            f_ref = model.extract_features(x)[0].clone()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(s)
        for _ in range(a.reps):
            model.extract_features(x)
        e1.record(s)
        t_host = (time.perf_counter() - t0) / a.reps
        torch.cuda.synchronize()
        out["direct_ms"] = round(e0.elapsed_time(e1) / a.reps, 4)
        out["direct_host_submit_ms"] = round(t_host * 1e3, 4)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            f_g = model.extract_features(x)[0]
        g.replay()
        torch.cuda.synchronize()
        out["graph_equal"] = bool(torch.equal(f_g, f_ref))
        e0.record(s)
        for _ in range(a.reps):
            g.replay()
        e1.record(s)
        torch.cuda.synchronize()
        out["graph_ms"] = round(e0.elapsed_time(e1) / a.reps, 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

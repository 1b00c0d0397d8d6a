"""Time the 200-step inner loop under CWT_ADAPT_DBG ablation flags (one process per setting:
the flags are read when the step graph is captured)."""
import os, sys, json, subprocess
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r'''
import sys, torch, numpy as np
sys.path.insert(0, "%s")
from few_shot_seg_cwt_amd import synthetic as syn, _lib
from few_shot_seg_cwt_amd.episode import inner_adapt
dev = torch.device("cuda", 0)
n = int(sys.argv[1])
ep = syn.make_episode(2021, 0, 473, n)
f = torch.from_numpy(syn.normal(2021, "f", (n, 512, 60, 60), 0.1)).to(dev).contiguous(memory_format=torch.channels_last)
lbl = torch.from_numpy(ep["s_label"][0]).to(dev)
W = torch.zeros(2, 512, device=dev)
for _ in range(3): inner_adapt(f, lbl, W, 0.1, 200)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10): inner_adapt(f, lbl, W, 0.1, 200)
e1.record(); torch.cuda.synchronize()
print(e0.elapsed_time(e1) / 10 / 200 * 1e3)
''' % ROOT
out = {}
for n in [int(x) for x in os.environ.get("SHOTS", "1,5").split(",")]:
    for flags in [int(x) for x in os.environ.get("FLAGS", "0,1,2,4,8,15,16").split(",")]:
        env = dict(os.environ, CWT_ADAPT_DBG=str(flags))
        r = subprocess.run([sys.executable, "-c", CODE, str(n)], env=env, capture_output=True, text=True, timeout=300)
        us = r.stdout.strip().splitlines()[-1] if r.returncode == 0 else "ERR " + r.stderr[-300:]
        out[f"n{n}_dbg{flags}"] = us
        print(f"shots={n} dbg={flags:2d}: {us} us/step", flush=True)
json.dump(out, open(os.path.join(ROOT, "gpurun_out", "adapt_ablate.json"), "w"), indent=1)

"""MMN.forward at the 473^2 geometry (h = w = 60, one shot), `reps` times, for a rocprofv3 kernel
summary of the head (python tools/prof_mmn.py [reps])."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from few_shot_seg_cwt_amd.match import MMN, init_match_params  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda", 0)
h = 60
args = dict(rmid="l34", layers=50, all_lr="l", temp=20.0, att_wt=0.2, conv4d="red")
net = MMN(args, agg="cat", wa=True, device=dev)
init_match_params(net, 1)
g = torch.Generator().manual_seed(3)
mk = lambda n, c: torch.rand(n, c, h, h, generator=g).to(dev).contiguous(memory_format=torch.channels_last)  # noqa
fq_lst = {3: [mk(1, 1024)], 4: [mk(1, 2048)]}
fs_lst = {3: [mk(1, 1024)], 4: [mk(1, 2048)]}
f_q, f_s = mk(1, 512), mk(1, 512)
with torch.no_grad():
    for _ in range(reps):
        net(fq_lst, fs_lst, f_q, f_s)
torch.cuda.synchronize()
print("done")

"""Wall time of the MMN head at the 473^2 geometry (h = w = 60): MMN.forward (rmid l34, wa,
agg cat; one query, `shots` supports) and MatchNet.corr_forward alone (in_channel 2, v 512
channels).  python tools/time_match.py [shots] [reps]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from few_shot_seg_cwt_amd.match import MMN, init_match_params  # noqa: E402

shots = int(sys.argv[1]) if len(sys.argv) > 1 else 1
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
dev = torch.device("cuda", 0)
h = 60
args = dict(rmid="l34", layers=50, all_lr="l", temp=20.0, att_wt=0.2, conv4d="red")
net = MMN(args, agg="cat", wa=True, device=dev)
init_match_params(net, 1)
g = torch.Generator().manual_seed(3)
mk = lambda n, c: torch.rand(n, c, h, h, generator=g).to(dev).contiguous(memory_format=torch.channels_last)  # noqa
fq_lst = {3: [mk(1, 1024)], 4: [mk(1, 2048)]}
fs_lst = {3: [mk(shots, 1024)], 4: [mk(shots, 2048)]}
f_q, f_s = mk(1, 512), mk(shots, 512)
corr = torch.rand(shots, 2, h * h, h * h, generator=g).to(dev)


def timed(fn):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return round(ts[len(ts) // 2], 3)


G = torch.rand(1, 512, h, h, generator=g).to(dev)


def train_step():
    """the head's forward + backward as the MMN trainers run it (train_cca.py:158-196)"""
    net.zero_grad(set_to_none=True)
    fq, att_fq = net(fq_lst, fs_lst, f_q, f_s)
    (att_fq * G).sum().backward()


with torch.no_grad():
    out = {"h": h, "shots": shots,
           "mmn_forward_ms": timed(lambda: net(fq_lst, fs_lst, f_q, f_s)),
           "corr_forward_ms": timed(lambda: net.corr_net._run(corr, h, h, f_s)),
           "weight_average_l4_ms": timed(lambda: net.wa_4(fq_lst[4][0]))}
out["mmn_forward_backward_ms"] = timed(train_step)
print(json.dumps(out))

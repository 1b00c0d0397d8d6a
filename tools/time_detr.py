"""Wall time of the DeTr head at the 473^2 geometry (h = w = 60): DeTr.forward (rmid l34, cross and
self attention), its deformable self attention alone, and one adjust_feature product.
python tools/time_detr.py [reps]"""
import json
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from few_shot_seg_cwt_amd.detr import DeTr  # noqa: E402
from few_shot_seg_cwt_amd.match import init_match_params  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda", 0)
h = 60
torch.manual_seed(0)
net = DeTr(dict(rmid="l34", temp=20.0, att_wt=0.2), sf_att=True, cs_att=True, reduce_dim=512, device=dev)
init_match_params(net.cross_trans, 1)
with torch.no_grad():
    net.adjust_feature[0].weight.mul_(1.0)
g = torch.Generator().manual_seed(3)
mk = lambda n, c: torch.rand(n, c, h, h, generator=g).to(dev).contiguous(memory_format=torch.channels_last)  # noqa
fq_lst = {3: [mk(1, 1024)], 4: [mk(1, 2048)]}
fs_lst = {3: [mk(1, 1024)], 4: [mk(1, 2048)]}
f_q, f_s = mk(1, 512), mk(1, 512)
fq_fea = mk(1, 512)


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


out = {"h": h,
       "detr_forward_ms": timed(lambda: net(fq_lst, fs_lst, f_q, f_s)),
       "deform_att_ms": timed(lambda: net.self_trans(fq_fea, f_q)),
       "compute_feat_ms": timed(lambda: net.compute_feat(fq_lst, fs_lst))}
print(json.dumps(out))

"""Time one CenterPivotConv4d layer at the MMN geometry (60^2 x 60^2) per kernel variant
(cwt_debug_cp4d_layer: 1 the tile kernels, 2 the rolling-window kernel).  CWT_CP4D_WC sets the
rolling kernel's a columns per workgroup.  python tools/time_cp4d.py [reps]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from few_shot_seg_cwt_amd import _lib  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda", 0)
h = 60
out = {"wc": os.environ.get("CWT_CP4D_WC", "30")}
for cin, cout in ((2, 10), (10, 10), (10, 1)):
    x = torch.rand(1, h * h, h * h, cin, device=dev)
    y = torch.empty(1, h * h, h * h, cout, device=dev)
    Wa, Wb = torch.rand(cout, cin, 3, 3, device=dev) * 0.1, torch.rand(cout, cin, 3, 3, device=dev) * 0.1
    ba, bb = torch.zeros(cout, device=dev), torch.zeros(cout, device=dev)
    for v in (1, 2):
        fn = lambda: _lib.check(_lib.lib().cwt_debug_cp4d_layer(  # noqa: E731
            _lib.ctx(0), _lib.ptr(x), 1, h, h, h, h, cin, cout, _lib.ptr(Wa), _lib.ptr(ba), _lib.ptr(Wb), _lib.ptr(bb),
            _lib.ptr(y), v, _lib.stream_ptr(dev)), "cwt_debug_cp4d_layer")
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        flop = 2 * 2 * 9 * cin * cout * (h ** 4)
        out[f"{cin}to{cout}_v{v}_us"] = round(ms * 1e3, 1)
        out[f"{cin}to{cout}_v{v}_tf"] = round(flop / ms / 1e9, 1)
print(json.dumps(out))

import sys, os, torch
sys.path.insert(0, os.getcwd())
from few_shot_seg_cwt_amd import _lib
lib, ctx = _lib.lib(), _lib.ctx(0)
side = torch.cuda.Stream()
for us in (200, 2000):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(side)
    rc = lib.cwt_debug_occupy(ctx, 59, us, side.cuda_stream)
    b.record(side)
    torch.cuda.synchronize()
    print("us", us, "rc", rc, "blocker ms", a.elapsed_time(b), flush=True)
# a kernel on the main stream while the blocker holds 255 CUs: it must wait or share
a, b, c = (torch.cuda.Event(enable_timing=True) for _ in range(3))
a.record(side)
lib.cwt_debug_occupy(ctx, 59, 3000, side.cuda_stream)
b.record(side)
torch.cuda._sleep(200000)
x = torch.randn(4096, 4096, device="cuda")
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(); y = x @ x; e1.record()
torch.cuda.synchronize()
print("blocker", a.elapsed_time(b), "a->e0", a.elapsed_time(e0), "a->e1", a.elapsed_time(e1), flush=True)

"""RCCL on the box: the collectives the multi-GPU path issues (few_shot_seg_cwt_amd/dist.py),
run through the "nccl" (= RCCL) backend in a one-rank process group on cuda:0 -- the 8.39 MB
fp32 CWT-gradient SUM all-reduce, the fp64 MAX of the timing, the fp64 SUM of the IoU table and
the device barrier.  One rank only: the box has one GPU (RCCL refuses two ranks on one device);
the N > 1 arithmetic is covered by the gloo tests (tests/test_dist_gloo.py)."""
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import os, sys, torch, torch.distributed as dist
sys.path.insert(0, os.environ["CWT_ROOT"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", init_method="tcp://127.0.0.1:" + os.environ["CWT_PORT"], rank=0, world_size=1,
                        device_id=torch.device("cuda", 0))
g = torch.arange(2098688, dtype=torch.float32, device="cuda")
dist.all_reduce(g, op=dist.ReduceOp.SUM)
assert torch.equal(g, torch.arange(2098688, dtype=torch.float32, device="cuda"))
t = torch.tensor([3.5], dtype=torch.float64, device="cuda")
dist.all_reduce(t, op=dist.ReduceOp.MAX)
assert float(t.item()) == 3.5
tab = torch.ones((20, 4), dtype=torch.float64, device="cuda")
dist.all_reduce(tab, op=dist.ReduceOp.SUM)
dist.barrier(device_ids=[0])
torch.cuda.synchronize()
dist.destroy_process_group()
print("rccl ok")
"""


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_collectives_one_rank():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    env = dict(os.environ, CWT_ROOT=ROOT, CWT_PORT=str(_free_port()))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run([sys.executable, "-c", SCRIPT], env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0 and "rccl ok" in r.stdout, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])

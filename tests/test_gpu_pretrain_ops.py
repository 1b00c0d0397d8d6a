"""Single kernels of the pretraining iteration (cwt_debug_pretrain_op) against float64 torch
autograd on random data -- well conditioned, unlike the whole-network step (test_gpu_pretrain.py),
so the bars are tight: conv weight / input gradients over every conv geometry of the ResNet
(1x1, 3x3 dilated, stride 2, the 4096-channel bottleneck shape reduced), training BN + ReLU
backward, max-pool adjoint, label-smoothed CE of the upsampled logits and its gradient, the
folded PPM field of the bottleneck conv and its adjoint."""
import ctypes as C

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


def op(opcode, bufs, ia, fa=()):
    from few_shot_seg_cwt_amd import _lib
    b = (C.c_void_p * len(bufs))(*[t.data_ptr() for t in bufs])
    i = (C.c_int64 * len(ia))(*ia)
    f = (C.c_float * max(1, len(fa)))(*fa) if fa else None
    _lib.check(_lib.lib().cwt_debug_pretrain_op(_lib.ctx(0), opcode, b, i, f, _lib.stream_ptr()), "pretrain_op")
    torch.cuda.synchronize()


def pack(w):
    """[Co][Ci][k][k] -> conv.hip packed [Co][K], K = (32-channel block, tap, channel)."""
    Co, Ci, k, _ = w.shape
    t = w.reshape(Co, Ci // 32, 32, k * k).permute(0, 1, 3, 2)  # co, cb, tap, c
    return t.reshape(Co, -1).contiguous()


GEOMS = [  # N Hi Ci Co k stride pad dil
    (2, 15, 64, 64, 3, 1, 1, 1), (2, 17, 128, 64, 1, 1, 0, 1), (2, 15, 128, 128, 3, 2, 1, 1),
    (2, 15, 256, 512, 1, 2, 0, 1), (2, 9, 256, 256, 3, 1, 2, 2), (2, 9, 512, 128, 3, 1, 4, 4),
    (1, 7, 1024, 128, 3, 1, 1, 1), (3, 33, 64, 128, 3, 1, 1, 1)]


@pytest.mark.parametrize("g", GEOMS)
def test_conv_grads(dev, g):
    N, Hi, Ci, Co, k, s, pad, dil = g
    gen = torch.Generator().manual_seed(hash(g) & 0xFFFF)
    x = torch.randn(N, Ci, Hi, Hi, generator=gen, dtype=torch.float64, requires_grad=True)
    w = (torch.randn(Co, Ci, k, k, generator=gen, dtype=torch.float64) / (Ci * k * k) ** 0.5).requires_grad_(True)
    y = F.conv2d(x, w, None, s, pad, dil)
    dy = torch.randn(y.shape, generator=gen, dtype=torch.float64)
    gx, gw = torch.autograd.grad(y, [x, w], dy)
    nhwc = lambda t: t.permute(0, 2, 3, 1).contiguous().float().to(dev)
    gw_d = torch.empty(Co, Ci * k * k, device=dev)
    op(0, [nhwc(dy), nhwc(x.detach()), gw_d], [N, Hi, Ci, Co, k, s, pad, dil])
    assert rel(gw_d.cpu(), pack(gw).float()) < 1e-5
    gx_d = torch.empty(N, Hi, Hi, Ci, device=dev)
    op(1, [nhwc(dy), pack(w.detach()).float().to(dev), gx_d], [N, Hi, Ci, Co, k, s, pad, dil])
    assert rel(gx_d.cpu(), gx.permute(0, 2, 3, 1)) < 1e-5


@pytest.mark.parametrize("M,Cc", [(2 * 81, 64), (8, 512), (3 * 225, 128)])
def test_bn_relu_fwd_bwd(dev, M, Cc):
    gen = torch.Generator().manual_seed(M * 7 + Cc)
    y = torch.randn(M, Cc, generator=gen, dtype=torch.float64) * 2 + 0.5
    gamma = (torch.rand(Cc, generator=gen, dtype=torch.float64) + 0.5).requires_grad_(True)
    beta = (torch.randn(Cc, generator=gen, dtype=torch.float64) * 0.1).requires_grad_(True)
    yv = y.clone().requires_grad_(True)
    out = F.relu(F.batch_norm(yv, None, None, gamma, beta, training=True, eps=1e-5))
    dout = torch.randn(M, Cc, generator=gen, dtype=torch.float64)
    gy, gg, gb = torch.autograd.grad(out, [yv, gamma, beta], dout)
    d = lambda t: t.detach().float().contiguous().to(dev)
    o, dy_, dg, db = (torch.empty(M, Cc, device=dev), torch.empty(M, Cc, device=dev), torch.empty(Cc, device=dev),
                      torch.empty(Cc, device=dev))
    op(3, [d(y), d(gamma), d(beta), o, d(dout), dy_, dg, db], [M, Cc], [1e-5])
    assert rel(o.cpu(), out) < 1e-5
    assert rel(dy_.cpu(), gy) < 1e-4
    assert rel(dg.cpu(), gg) < 1e-5 and rel(db.cpu(), gb) < 1e-5


def test_maxpool_adjoint(dev):
    gen = torch.Generator().manual_seed(5)
    x = F.relu(torch.randn(2, 64, 17, 17, generator=gen, dtype=torch.float64)).requires_grad_(True)
    y = F.max_pool2d(x, 3, 2, 1)
    dy = torch.randn(y.shape, generator=gen, dtype=torch.float64)
    gx, = torch.autograd.grad(y, [x], dy)
    nhwc = lambda t: t.detach().permute(0, 2, 3, 1).contiguous().float().to(dev)
    out, din = torch.empty(2, 9, 9, 64, device=dev), torch.empty(2, 17, 17, 64, device=dev)
    op(4, [nhwc(x), out, nhwc(dy), din], [2, 17, 64])
    assert rel(out.cpu(), y.float().permute(0, 2, 3, 1)) == 0.0
    assert rel(din.cpu(), gx.permute(0, 2, 3, 1)) < 1e-6


@pytest.mark.parametrize("nc,S", [(16, 33), (61, 65), (16, 473)])
def test_smoothed_ce(dev, nc, S):
    from oracle.pretrain_oracle import smoothed_ce
    N, h = 2, (S - 1) // 8 + 1
    gen = torch.Generator().manual_seed(nc + S)
    lg = torch.randn(N, nc, h, h, generator=gen, dtype=torch.float64, requires_grad=True)
    t = torch.randint(0, nc, (N, S, S), generator=gen)
    t[torch.rand(N, S, S, generator=gen) < 0.1] = 255
    up = F.interpolate(lg, size=(S, S), mode="bilinear", align_corners=True)
    loss = smoothed_ce(up, t, nc, True)
    g, = torch.autograd.grad(loss, [lg])
    dl, lo = torch.empty(N, h, h, nc, device=dev), torch.empty(1, device=dev)
    op(2, [lg.detach().permute(0, 2, 3, 1).contiguous().float().to(dev), t.to(dev), dl, lo], [N, S, h, nc],
       [0.9, 0.1 / (nc - 1)])
    assert abs(float(lo) - loss.item()) / loss.item() < 1e-5
    assert rel(dl.cpu(), g.permute(0, 2, 3, 1)) < 1e-4


def test_smoothed_ce_all_ignored(dev):
    """Every target pixel 255: the reference's masked_select(...).mean() is NaN and its gradient
    zero (pretrain.py:163-219), so the SGD step that follows sees a zero gradient."""
    from oracle.pretrain_oracle import smoothed_ce
    nc, S, N = 16, 33, 2
    h = (S - 1) // 8 + 1
    gen = torch.Generator().manual_seed(9)
    lg = torch.randn(N, nc, h, h, generator=gen, dtype=torch.float64, requires_grad=True)
    t = torch.full((N, S, S), 255, dtype=torch.int64)
    loss = smoothed_ce(F.interpolate(lg, size=(S, S), mode="bilinear", align_corners=True), t, nc, True)
    g, = torch.autograd.grad(loss, [lg])
    dl, lo = torch.empty(N, h, h, nc, device=dev), torch.empty(1, device=dev)
    op(2, [lg.detach().permute(0, 2, 3, 1).contiguous().float().to(dev), t.to(dev), dl, lo], [N, S, h, nc],
       [0.9, 0.1 / (nc - 1)])
    assert np.isnan(loss.item()) and np.isnan(float(lo))
    assert float(g.abs().max()) == 0.0 and float(dl.abs().max()) == 0.0


@pytest.mark.parametrize("N,h", [(2, 17), (1, 60)])
def test_ppm_field_fold_and_adjoint(dev, N, h):
    """The pretraining bottleneck's folded PPM branch (pretrain.hip pt_forward / pt_backward):
    F = conv3x3(W_ppm, cat_b upsample_b(P_b)) without the upsampled maps, and its adjoint dP, dW
    (the field's transpose), against the unfolded float64 form of pspnet.py:19-38,124-128."""
    gen = torch.Generator().manual_seed(h)
    bins = (1, 2, 3, 6)
    Ps = [torch.randn(N, 512, b, b, generator=gen, dtype=torch.float64, requires_grad=True) for b in bins]
    Wfull = torch.randn(512, 4096, 3, 3, generator=gen, dtype=torch.float64) * 0.02
    Wp = Wfull[:, 2048:].clone().requires_grad_(True)
    up = torch.cat([F.interpolate(p, size=(h, h), mode="bilinear", align_corners=True) for p in Ps], 1)
    Fr = F.conv2d(up, Wp, padding=1)
    dF = torch.randn(Fr.shape, generator=gen, dtype=torch.float64)
    gps = torch.autograd.grad(Fr, Ps + [Wp], dF)
    cells = lambda ts: torch.cat([t.detach().permute(0, 2, 3, 1).reshape(-1, 512) for t in ts], 0)
    nhwc = lambda t: t.detach().permute(0, 2, 3, 1).contiguous().float().to(dev)
    Pd = cells(Ps).float().contiguous().to(dev)
    Fo, dP = torch.empty(N, h, h, 512, device=dev), torch.empty_like(Pd)
    W = pack(Wfull).float().contiguous().to(dev)
    dW = torch.zeros_like(W)
    op(5, [Pd, nhwc(dF), Fo, dP, W, dW], [N, h])
    assert rel(Fo.cpu(), Fr.permute(0, 2, 3, 1)) < 1e-5
    assert rel(dP.cpu(), cells(gps[:4])) < 1e-5
    gW = torch.zeros_like(Wfull)
    gW[:, 2048:] = gps[4]
    assert rel(dW.cpu(), pack(gW)) < 1e-5

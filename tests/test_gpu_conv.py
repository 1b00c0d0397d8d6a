"""Every tile / split-K plan of the implicit-GEMM conv (cwt_debug_conv) against a torch fp32
conv + folded BN (+ residual) (+ ReLU), including channel-strided input/output (the PPM
concat buffer)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from few_shot_seg_cwt_amd import synthetic as syn  # noqa: E402


def run_conv(x_nchw, w, scale, shift, stride, pad, dil, res=None, relu=True, bm=0, bn=0, nsplit=0, x_pad=0,
             y_pad=0, y_off=0, precision=0):
    from few_shot_seg_cwt_amd import _lib
    dev = torch.device("cuda", 0)
    N, Ci, Hi, Wi = x_nchw.shape
    Co, _, k, _ = w.shape
    x_ld = Ci + x_pad
    xb = torch.zeros(N, Hi, Wi, x_ld)
    xb[..., :Ci] = x_nchw.permute(0, 2, 3, 1)
    xd = xb.to(dev).contiguous()
    wp = w.permute(0, 2, 3, 1).contiguous().to(dev)
    Ho = (Hi + 2 * pad - dil * (k - 1) - 1) // stride + 1
    y_ld = Co + y_pad
    y = torch.full((N, Ho, Ho, y_ld), float("nan"), device=dev)
    rd = res.permute(0, 2, 3, 1).contiguous().to(dev) if res is not None else None
    sc, sh = scale.to(dev), shift.to(dev)   # named: a temporary would be freed before the launch
    rc = _lib.lib().cwt_debug_conv(_lib.ctx(0), _lib.ptr(xd), N, Hi, Wi, Ci, x_ld, _lib.ptr(wp),
                                   _lib.ptr(sc), _lib.ptr(sh), Co, k, stride, pad, dil,
                                   _lib.ptr(rd), Co, int(relu), _lib.ptr(y), y_ld, y_off, bm, bn, nsplit,
                                   precision, _lib.stream_ptr())
    _lib.check(rc, "cwt_debug_conv")
    torch.cuda.synchronize()
    yc = y.cpu()
    if y_pad:
        untouched = torch.cat([yc[..., :y_off], yc[..., y_off + Co:]], -1)
        assert torch.isnan(untouched).all(), "wrote outside its channel slice"
    return yc[..., y_off:y_off + Co].permute(0, 3, 1, 2)


def ref_conv(x, w, scale, shift, stride, pad, dil, res=None, relu=True):
    y = F.conv2d(x.double(), w.double(), None, stride, pad, dil)
    y = y * scale.double()[None, :, None, None] + shift.double()[None, :, None, None]
    if res is not None:
        y = y + res.double()
    return F.relu(y) if relu else y


CASES = [  # N, Ci, Co, Hi, k, stride, dil, residual
    (2, 64, 64, 37, 3, 1, 1, False),
    (2, 64, 128, 37, 3, 1, 1, False),
    (1, 128, 256, 23, 1, 1, 1, True),
    (2, 256, 128, 21, 1, 2, 1, False),
    (1, 128, 128, 21, 3, 2, 1, False),
    (2, 256, 256, 15, 3, 1, 2, True),
    (1, 512, 128, 13, 3, 1, 4, False),
    (3, 96, 64, 9, 1, 1, 1, True),
    (1, 64, 512, 19, 3, 1, 1, True),
]
PLANS = [(0, 0, 0), (128, 128, 1), (128, 64, 1), (64, 64, 1), (64, 64, 3), (128, 128, 2)]
# the exact-fp32 MFMA conv (CWT_CONV=f32, the training-mode-BN pass); the bf16x3 S-layout plans
# are covered by test_gpu_conv_s.py
TOLS = {0: 1e-5}


@pytest.mark.parametrize("precision", [0], ids=["f32"])
@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c)))
@pytest.mark.parametrize("plan", PLANS, ids=lambda p: f"{p[0]}x{p[1]}s{p[2]}")
def test_conv_plans(case, plan, precision):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    N, Ci, Co, Hi, k, stride, dil, has_res = case
    bm, bn, ns = plan
    if bn and Co % bn:
        pytest.skip("Co not a multiple of the tile")
    tag = f"{N}_{Ci}_{Co}_{Hi}_{k}"
    x = torch.from_numpy(syn.normal(1, "x" + tag, (N, Ci, Hi, Hi), 1.0))
    w = torch.from_numpy(syn.normal(1, "w" + tag, (Co, Ci, k, k), (2.0 / (Ci * k * k)) ** 0.5))
    scale = torch.from_numpy(syn.uniform(1, "s" + tag, (Co,), 0.5, 1.5))
    shift = torch.from_numpy(syn.normal(1, "b" + tag, (Co,), 0.1))
    pad = dil if k == 3 else 0
    Ho = (Hi + 2 * pad - dil * (k - 1) - 1) // stride + 1
    res = torch.from_numpy(syn.normal(1, "r" + tag, (N, Co, Ho, Ho), 1.0)) if has_res else None
    out = run_conv(x, w, scale, shift, stride, pad, dil, res, True, bm, bn, ns, precision=precision)
    ref = ref_conv(x, w, scale, shift, stride, pad, dil, res, True)
    err = float((out.double() - ref).abs().max() / ref.abs().max())
    assert err < TOLS[precision], err


@pytest.mark.parametrize("precision", [0], ids=["f32"])
def test_conv_channel_strided_io(precision):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    x = torch.from_numpy(syn.normal(2, "x", (2, 64, 11, 11), 1.0))
    w = torch.from_numpy(syn.normal(2, "w", (128, 64, 3, 3), 0.06))
    scale = torch.ones(128)
    shift = torch.zeros(128)
    out = run_conv(x, w, scale, shift, 1, 1, 1, None, False, x_pad=32, y_pad=256, y_off=128, precision=precision)
    ref = ref_conv(x, w, scale, shift, 1, 1, 1, None, False)
    assert float((out.double() - ref).abs().max() / ref.abs().max()) < TOLS[precision]

"""One CenterPivotConv4d layer + ReLU (src/model/conv4d.py:40-62) through cwt_debug_cp4d_layer:
the rolling-window kernel (cp4d_roll_kernel, variant 2) and the tile kernels (variant 1) against
a float64 restatement by 2-D convolutions (torch conv2d over the a plane for every b and over the
b plane for every a, both summed).  Exact fp32 arithmetic in both kernels (f32 MFMA = an fmaf
chain); they differ only in summation order.  Bar: max|y - ref| / max|ref| < 1e-5 (float64
reference), and at the MMN geometry (60^2, float32 reference on the device) < 1e-4."""
import pytest
import torch

from few_shot_seg_cwt_amd import _lib

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


def ref_layer(x, B, hA, wA, hB, wB, Wa, ba, Wb, bb):
    C = x.shape[-1]
    NA, NB = hA * wA, hB * wB
    F = torch.nn.functional
    xa = x.view(B, hA, wA, NB, C).permute(0, 3, 4, 1, 2).reshape(B * NB, C, hA, wA)
    ya = F.conv2d(xa, Wa, ba, padding=1)
    ya = ya.view(B, NB, -1, hA, wA).permute(0, 3, 4, 1, 2).reshape(B, NA, NB, -1)
    xb = x.view(B * NA, hB, wB, C).permute(0, 3, 1, 2)
    yb = F.conv2d(xb, Wb, bb, padding=1).permute(0, 2, 3, 1).reshape(B, NA, NB, -1)
    return (ya + yb).relu()


def run(x, B, hA, wA, hB, wB, cin, cout, Wa, ba, Wb, bb, variant):
    y = torch.empty((B, hA * wA, hB * wB, cout), device=x.device, dtype=torch.float32)
    _lib.check(_lib.lib().cwt_debug_cp4d_layer(_lib.ctx(0), _lib.ptr(x), B, hA, wA, hB, wB, cin, cout, _lib.ptr(Wa),
                                               _lib.ptr(ba), _lib.ptr(Wb), _lib.ptr(bb), _lib.ptr(y), variant,
                                               _lib.stream_ptr(x.device)), "cwt_debug_cp4d_layer")
    torch.cuda.synchronize()
    return y


def params(cin, cout, seed, dev):
    g = torch.Generator().manual_seed(seed)
    s = (9 * cin) ** -0.5
    mk = lambda *sh: (torch.rand(*sh, generator=g, dtype=torch.float64) * 2 - 1)  # noqa: E731
    return [t.to(dev) for t in (mk(cout, cin, 3, 3) * s, mk(cout) * 0.1, mk(cout, cin, 3, 3) * s, mk(cout) * 0.1)]


@pytest.mark.parametrize("B,hA,wA,hB,wB,cin,cout", [(1, 12, 12, 12, 12, 1, 10), (2, 9, 13, 11, 7, 2, 10),
                                                    (1, 5, 5, 17, 26, 10, 10), (1, 7, 4, 4, 25, 10, 10),
                                                    (2, 13, 6, 9, 12, 10, 10), (1, 3, 2, 5, 3, 10, 10),
                                                    (1, 5, 5, 17, 26, 10, 1), (2, 13, 6, 9, 12, 10, 1),
                                                    (1, 3, 2, 5, 3, 10, 1)])
def test_roll_layer_small(dev, B, hA, wA, hB, wB, cin, cout):
    g = torch.Generator().manual_seed(hA * 100 + wB)
    x64 = torch.rand(B, hA * wA, hB * wB, cin, generator=g, dtype=torch.float64).to(dev) - 0.3
    p64 = params(cin, cout, cin + cout, dev)
    ref = ref_layer(x64, B, hA, wA, hB, wB, *p64)
    x, p = x64.float().contiguous(), [t.float().contiguous() for t in p64]
    for v in (1, 2):
        y = run(x, B, hA, wA, hB, wB, cin, cout, *p, v)
        err = float((y.double() - ref).abs().max() / ref.abs().max())
        print(f"cp4d layer {cin}->{cout} B={B} a={hA}x{wA} b={hB}x{wB} variant {v}: {err:.2e}")
        assert err < 1e-5, (v, err)


@pytest.mark.parametrize("cin,cout", [(2, 10), (10, 10), (10, 1)])
def test_roll_layer_mmn_geometry(dev, cin, cout):
    """The MMN head's 60 x 60 by 60 x 60 correlation (473^2 images)."""
    h = 60
    g = torch.Generator().manual_seed(7 + cin)
    x = (torch.rand(1, h * h, h * h, cin, generator=g) - 0.3).to(dev)
    p = [t.float().contiguous() for t in params(cin, cout, 11 + cin + cout, dev)]
    ref = ref_layer(x, 1, h, h, h, h, *p)
    y2 = run(x, 1, h, h, h, h, cin, cout, *p, 2)
    e2 = float((y2 - ref).abs().max() / ref.abs().max())
    del y2
    y1 = run(x, 1, h, h, h, h, cin, cout, *p, 1)
    e1 = float((y1 - ref).abs().max() / ref.abs().max())
    print(f"cp4d layer {cin}->{cout} at 60^2: roll {e2:.2e}, tile {e1:.2e}")
    assert e2 < 1e-4 and e1 < 1e-4, (e2, e1)

"""Every tile / split-K plan of the split-activation conv (cwt_debug_conv_s, conv_x3s.hip)
against a float64 torch conv + folded BN (+ fp32 or S-layout residual) (+ ReLU), with both
output forms (fp32 NHWC at a channel offset/stride, and S-layout), plus the S-layout
split/unsplit round trip."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from few_shot_seg_cwt_amd import synthetic as syn  # noqa: E402

# bf16x3 drops the lo*lo term (~2^-16 relative per product); the S-layout input is hi+lo
# (16 significant bits), which is exactly what the bf16x3 MFMAs see anyway
TOL = 1e-4


def _lib():
    from few_shot_seg_cwt_amd import _lib as L
    return L


def split(t_nhwc):
    """fp32 [..., C] (device) -> S-layout bf16 [..., C/32, 64]"""
    L = _lib()
    C = t_nhwc.shape[-1]
    P = t_nhwc.numel() // C
    out = torch.empty(P * C * 2, dtype=torch.bfloat16, device=t_nhwc.device)
    L.check(L.lib().cwt_debug_split_act(L.ctx(0), L.ptr(t_nhwc), P, C, C, L.ptr(out), L.stream_ptr()), "split")
    return out


def unsplit(s, P, C):
    L = _lib()
    out = torch.empty(P, C, device=s.device)
    L.check(L.lib().cwt_debug_unsplit_act(L.ctx(0), L.ptr(s), P, C, L.ptr(out), C, L.stream_ptr()), "unsplit")
    return out


def run_conv_s(x, w, scale, shift, stride, pad, dil, res=None, res_split=False, relu=True, bm=0, bn=0, nsplit=0,
               y_pad=0, y_off=0):
    L = _lib()
    dev = torch.device("cuda", 0)
    N, Ci, Hi, Wi = x.shape
    Co, _, k, _ = w.shape
    xs = split(x.permute(0, 2, 3, 1).contiguous().to(dev))
    wd = w.permute(0, 2, 3, 1).contiguous().to(dev)
    ws = torch.empty(Co * k * k * Ci * 2, dtype=torch.bfloat16, device=dev)
    L.check(L.lib().cwt_debug_pack_wsplit(L.ctx(0), L.ptr(wd), Co, k, Ci, L.ptr(ws), L.stream_ptr()), "pack")
    Ho = (Hi + 2 * pad - dil * (k - 1) - 1) // stride + 1
    y_ld = Co + y_pad
    y = torch.full((N, Ho, Ho, y_ld), float("nan"), device=dev)
    ys = torch.zeros(N * Ho * Ho * Co * 2, dtype=torch.bfloat16, device=dev)
    rd = res.permute(0, 2, 3, 1).contiguous().to(dev) if res is not None else None
    rs = split(rd) if (rd is not None and res_split) else None
    sc, sh = scale.to(dev), shift.to(dev)
    rc = L.lib().cwt_debug_conv_s(L.ctx(0), L.ptr(xs), N, Hi, Wi, Ci, L.ptr(ws), L.ptr(sc), L.ptr(sh), Co, k,
                                  stride, pad, dil, None if res_split else L.ptr(rd), Co, L.ptr(rs), int(relu),
                                  L.ptr(y), y_ld, y_off, L.ptr(ys), bm, bn, nsplit, L.stream_ptr())
    L.check(rc, "cwt_debug_conv_s")
    torch.cuda.synchronize()
    yc = y.cpu()
    if y_pad:
        untouched = torch.cat([yc[..., :y_off], yc[..., y_off + Co:]], -1)
        assert torch.isnan(untouched).all(), "wrote outside its channel slice"
    yf = yc[..., y_off:y_off + Co]
    yu = unsplit(ys, N * Ho * Ho, Co).cpu().reshape(N, Ho, Ho, Co)
    return yf.permute(0, 3, 1, 2), yu.permute(0, 3, 1, 2)


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
PLANS = [(0, 0, 0), (256, 256, 1), (256, 128, 1), (128, 256, 1), (128, 256, 2), (128, 128, 1), (128, 64, 1), (64, 128, 1), (64, 64, 1),
         (64, 64, 3), (128, 128, 2), (256, 256, 4),
         # main-loop variants (bm = 1000 * variant + rows): 1 fragment prefetch, 2 prefetch with 8 waves,
         # 4 = 128x128 with a 2-stage ring
         (1064, 64, 1), (1064, 64, 3), (1128, 128, 1), (1128, 64, 2), (1064, 128, 1), (1128, 256, 1), (1256, 128, 2),
         (2064, 64, 1), (2064, 64, 2), (2128, 128, 1), (2128, 128, 3), (2128, 64, 1), (2064, 128, 1),
         (4128, 128, 1), (4128, 128, 3)]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c)))
@pytest.mark.parametrize("plan", PLANS, ids=lambda p: f"{p[0]}x{p[1]}s{p[2]}")
def test_conv_s_plans(case, plan):
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
    yf, yu = run_conv_s(x, w, scale, shift, stride, pad, dil, res, res_split=(ns % 2 == 1), bm=bm, bn=bn,
                        nsplit=ns)
    ref = ref_conv(x, w, scale, shift, stride, pad, dil, res, True)
    err = float((yf.double() - ref).abs().max() / ref.abs().max())
    assert err < TOL, err
    # the S-layout output is the split of the fp32 output (hi + lo = 16 significant bits)
    assert float((yu.double() - yf.double()).abs().max() / ref.abs().max()) < 2.0 ** -15


def test_conv_s_channel_strided_out():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    x = torch.from_numpy(syn.normal(2, "x", (2, 64, 11, 11), 1.0))
    w = torch.from_numpy(syn.normal(2, "w", (128, 64, 3, 3), 0.06))
    scale, shift = torch.ones(128), torch.zeros(128)
    yf, _ = run_conv_s(x, w, scale, shift, 1, 1, 1, None, relu=False, y_pad=256, y_off=128)
    ref = ref_conv(x, w, scale, shift, 1, 1, 1, None, False)
    assert float((yf.double() - ref).abs().max() / ref.abs().max()) < TOL


def test_split_roundtrip():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    x = torch.from_numpy(syn.normal(3, "rt", (1000, 96), 10.0)).cuda()
    s = split(x)
    hi = s.view(1000, 3, 2, 32)[:, :, 0].reshape(1000, 96)
    assert torch.equal(hi, x.to(torch.bfloat16))          # hi = bf16_rne(x)
    back = unsplit(s, 1000, 96)
    assert float(((back - x).abs() / x.abs().clamp_min(1e-30)).max()) < 2.0 ** -16


# ---------------------------------------------------------------- plain bf16 (CWT_CONV_BF16)
# fp32 accumulation of exact bf16 x bf16 products: against a float64 conv of the SAME
# bf16-rounded operands only the summation order differs (~K * 2^-24 relative).
TOL_B16 = 2e-5


def bf16_nhwc(t_nchw):
    return t_nchw.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)


def pack_w_b16(w):
    """[Co,Ci,k,k] fp32 -> bf16 [Co][K], K ordered (64-channel block, tap, channel)."""
    Co, Ci, k, _ = w.shape
    return w.reshape(Co, Ci // 64, 64, k * k).permute(0, 1, 3, 2).contiguous().to(torch.bfloat16)


def run_conv_b16(x, w, scale, shift, stride, pad, dil, res=None, res_bf16=False, relu=True, bm=0, bn=0, nsplit=0):
    L = _lib()
    dev = torch.device("cuda", 0)
    N, Ci, Hi, Wi = x.shape
    Co, _, k, _ = w.shape
    xs = bf16_nhwc(x).to(dev)
    ws = pack_w_b16(w).to(dev)
    Ho = (Hi + 2 * pad - dil * (k - 1) - 1) // stride + 1
    y = torch.full((N, Ho, Ho, Co), float("nan"), device=dev)
    ys = torch.zeros((N, Ho, Ho, Co), dtype=torch.bfloat16, device=dev)
    rd = res.permute(0, 2, 3, 1).contiguous().to(dev) if res is not None else None
    rs = rd.to(torch.bfloat16) if (rd is not None and res_bf16) else None
    sc, sh = scale.to(dev), shift.to(dev)
    rc = L.lib().cwt_debug_conv_b16(L.ctx(0), L.ptr(xs), N, Hi, Wi, Ci, L.ptr(ws), L.ptr(sc), L.ptr(sh), Co, k,
                                    stride, pad, dil, None if res_bf16 else L.ptr(rd), Co, L.ptr(rs), int(relu),
                                    L.ptr(y), Co, 0, L.ptr(ys), bm, bn, nsplit, L.stream_ptr())
    L.check(rc, "cwt_debug_conv_b16")
    torch.cuda.synchronize()
    return y.cpu().permute(0, 3, 1, 2), ys.cpu().float().permute(0, 3, 1, 2)


CASES_B16 = [c for c in CASES if c[1] % 64 == 0]


@pytest.mark.parametrize("case", CASES_B16, ids=lambda c: "x".join(map(str, c)))
@pytest.mark.parametrize("plan", PLANS, ids=lambda p: f"{p[0]}x{p[1]}s{p[2]}")
def test_conv_b16_plans(case, plan):
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
    res_bf16 = ns % 2 == 1
    yf, yb = run_conv_b16(x, w, scale, shift, stride, pad, dil, res, res_bf16=res_bf16, bm=bm, bn=bn, nsplit=ns)
    xr = x.to(torch.bfloat16).float()
    wr = w.to(torch.bfloat16).float()
    rr = res.to(torch.bfloat16).float() if (res is not None and res_bf16) else res
    ref = ref_conv(xr, wr, scale, shift, stride, pad, dil, rr, True)
    err = float((yf.double() - ref).abs().max() / ref.abs().max())
    assert err < TOL_B16, err
    # the bf16 output is the round-to-nearest bf16 of the fp32 output
    assert torch.equal(yb, yf.to(torch.bfloat16).float())


# ---------------------------------------------------------------- exact fp32 (conv_igemm_f32d)
# the LDS-DMA body over fp32 NHWC operands with v_mfma_f32_16x16x4_f32 (fmaf chains): against a
# float64 conv only the fp32 summation order differs
TOL_F32D = 1e-5


def pack_w_f32(w):
    """[Co,Ci,k,k] fp32 -> fp32 [Co][K], K in packed_k order (32-channel block, tap, channel)."""
    Co, Ci, k, _ = w.shape
    return w.reshape(Co, Ci // 32, 32, k * k).permute(0, 1, 3, 2).contiguous()


def run_conv_f32d(x, w, scale, shift, stride, pad, dil, res=None, relu=True, bm=0, bn=0, nsplit=0, y_pad=0, y_off=0,
                  entry="cwt_debug_conv_f32d"):
    L = _lib()
    dev = torch.device("cuda", 0)
    N, Ci, Hi, Wi = x.shape
    Co, _, k, _ = w.shape
    xd = x.permute(0, 2, 3, 1).contiguous().to(dev)
    wd = pack_w_f32(w).to(dev)
    Ho = (Hi + 2 * pad - dil * (k - 1) - 1) // stride + 1
    y_ld = Co + y_pad
    y = torch.full((N, Ho, Ho, y_ld), float("nan"), device=dev)
    rd = res.permute(0, 2, 3, 1).contiguous().to(dev) if res is not None else None
    sc, sh = scale.to(dev), shift.to(dev)
    rc = getattr(L.lib(), entry)(L.ctx(0), L.ptr(xd), N, Hi, Wi, Ci, L.ptr(wd), L.ptr(sc), L.ptr(sh), Co, k,
                                 stride, pad, dil, L.ptr(rd), Co, int(relu), L.ptr(y), y_ld, y_off, bm, bn,
                                 nsplit, L.stream_ptr())
    L.check(rc, entry)
    torch.cuda.synchronize()
    yc = y.cpu()
    if y_pad:
        untouched = torch.cat([yc[..., :y_off], yc[..., y_off + Co:]], -1)
        assert torch.isnan(untouched).all(), "wrote outside its channel slice"
    return yc[..., y_off:y_off + Co].permute(0, 3, 1, 2)


@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c)))
@pytest.mark.parametrize("plan", PLANS, ids=lambda p: f"{p[0]}x{p[1]}s{p[2]}")
def test_conv_f32d_plans(case, plan):
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
    y = run_conv_f32d(x, w, scale, shift, stride, pad, dil, res, bm=bm, bn=bn, nsplit=ns)
    ref = ref_conv(x, w, scale, shift, stride, pad, dil, res, True)
    err = float((y.double() - ref).abs().max() / ref.abs().max())
    assert err < TOL_F32D, err


def test_conv_f32d_channel_strided_out():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    x = torch.from_numpy(syn.normal(2, "x", (2, 64, 11, 11), 1.0))
    w = torch.from_numpy(syn.normal(2, "w", (128, 64, 3, 3), 0.06))
    scale, shift = torch.ones(128), torch.zeros(128)
    y = run_conv_f32d(x, w, scale, shift, 1, 1, 1, None, relu=False, y_pad=256, y_off=128)
    ref = ref_conv(x, w, scale, shift, 1, 1, 1, None, False)
    assert float((y.double() - ref).abs().max() / ref.abs().max()) < TOL_F32D


# ---------------------------------------------------------------- fp32 width on bf16 MFMA (conv_igemm_x6)
# f32d's operands split exactly into bf16 hi + mid + lo in registers; the three dropped products
# total < 2^-23 |a||b| per product (one fp32 rounding): the same bar as the exact-fp32 kernel
TOL_X6 = 1e-5
# the x6-only forms (bm = 1000 * variant + rows): 3 the WN = 128 wave layouts, 5 128x128 4x1 on a
# 2-stage ring (two workgroups per CU); round 6: the WN = 64 4x1 forms of the Co = 64 layers (128x64
# var 3 / 5, 64x64 var 3)
X6_FORMS = [(3256, 256, 1), (3256, 128, 1), (3128, 256, 1), (3128, 128, 1), (3128, 128, 2), (5128, 128, 1),
            (5128, 128, 4), (3064, 128, 1), (5064, 128, 1), (5064, 128, 2),
            (3128, 64, 1), (5128, 64, 1), (5128, 64, 2), (3064, 64, 1), (3064, 64, 2)]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c)))
@pytest.mark.parametrize("plan", PLANS + X6_FORMS, ids=lambda p: f"{p[0]}x{p[1]}s{p[2]}")
def test_conv_x6_plans(case, plan):
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
    y = run_conv_f32d(x, w, scale, shift, stride, pad, dil, res, bm=bm, bn=bn, nsplit=ns, entry="cwt_debug_conv_x6")
    ref = ref_conv(x, w, scale, shift, stride, pad, dil, res, True)
    err = float((y.double() - ref).abs().max() / ref.abs().max())
    assert err < TOL_X6, err


def test_conv_x6_wide_range_operands():
    """Operands spanning 2^-30 .. 2^30 (every split level populated, tiny lo terms): the x6 conv
    against float64 relative to the reference's own fp32 conv error, element by element."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    g = torch.Generator().manual_seed(5)
    N, Ci, Co, Hi = 1, 64, 64, 9
    mant = torch.rand((N, Ci, Hi, Hi), generator=g) + 0.5
    expo = torch.randint(-30, 31, (N, Ci, Hi, Hi), generator=g).float()
    x = (mant * torch.pow(2.0, expo) * torch.sign(torch.randn((N, Ci, Hi, Hi), generator=g))).float()
    w = torch.randn((Co, Ci, 3, 3), generator=g) * 0.05
    one, zero = torch.ones(Co), torch.zeros(Co)
    y = run_conv_f32d(x, w, one, zero, 1, 1, 1, None, relu=False, entry="cwt_debug_conv_x6")
    ref = ref_conv(x, w, one, zero, 1, 1, 1, None, False)
    # bound per output: the dropped split terms (< 2^-23 |x||w| per product) plus the worst-case
    # fp32 accumulation of K = 576 terms (gamma_K ~ K * 2^-24), both relative to sum |x||w|
    absref = F.conv2d(x.double().abs(), w.double().abs(), None, 1, 1, 1)
    bound = (2.0 * 2.0 ** -24 + 576 * 2.0 ** -24) * absref
    assert bool(((y.double() - ref).abs() <= bound).all()), float(((y.double() - ref).abs() / absref).max())
    y32 = F.conv2d(x, w, None, 1, 1, 1).double()
    print("x6 max err / sum|x||w|:", float(((y.double() - ref).abs() / absref).max()),
          " torch fp32:", float(((y32 - ref).abs() / absref).max()))


def test_conv_x6_channel_strided_out():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    x = torch.from_numpy(syn.normal(2, "x", (2, 64, 11, 11), 1.0))
    w = torch.from_numpy(syn.normal(2, "w", (128, 64, 3, 3), 0.06))
    scale, shift = torch.ones(128), torch.zeros(128)
    y = run_conv_f32d(x, w, scale, shift, 1, 1, 1, None, relu=False, y_pad=256, y_off=128, entry="cwt_debug_conv_x6")
    ref = ref_conv(x, w, scale, shift, 1, 1, 1, None, False)
    assert float((y.double() - ref).abs().max() / ref.abs().max()) < TOL_X6


# ------------------------------------------------ x6 Winograd F(2x2, 3x3) and F(4x4, 3x3) (wino.hip)
# the x6 stack's forms for stride-1 3x3 convs: transforms in fp32 (small integer coefficients;
# G g G^T in double, rounded once), 16 / 36 batched x6 GEMMs; against float64 at the same bar as
# the direct x6 (wtile = the entry's nsplit argument: the output tile edge m)
WINO_CASES = [  # N, Ci, Co, Hi, dil, residual
    (2, 64, 64, 37, 1, False),
    (2, 128, 128, 15, 1, True),
    (1, 128, 64, 13, 2, False),     # H not a multiple of 2d: ragged sub-grids (7 and 6 rows)
    (2, 256, 256, 15, 2, True),
    (1, 512, 128, 13, 4, False),
    (1, 256, 64, 9, 4, True),       # sub-grids of 3 and 2 rows: half-empty edge tiles
    (1, 64, 512, 19, 1, True),
    (1, 256, 128, 23, 1, True),     # 23 rows: the last 4x4 tile row three quarters empty
    (2, 128, 64, 30, 2, False),     # sub-grids of 15 rows: F(4x4) tiles ragged, F(2x2) exact-ish
]
# F(4x4,3x3), the opt-in form (CWT_WINO=4): the fp32 GEMM's accumulation error amplified by its
# transforms, 4e-6 .. 1.2e-5 of max |y| on these cases (F(2x2): 2-6e-7, a plain fp32 conv 2-3e-7)
TOL_X6W4 = 3e-5
WINO_TILES = [(0, 0), (256, 256), (256, 128), (128, 256), (128, 128), (128, 64), (64, 128), (64, 64), (4128, 128),
              (1064, 64), (2128, 128), (3256, 256), (3128, 128), (5128, 128)]


@pytest.mark.parametrize("case", WINO_CASES, ids=lambda c: "x".join(map(str, c)))
@pytest.mark.parametrize("tile", WINO_TILES, ids=lambda p: f"{p[0]}x{p[1]}")
@pytest.mark.parametrize("wtile", [2, 4], ids=lambda m: f"F{m}")
def test_conv_x6_winograd(case, tile, wtile):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    N, Ci, Co, Hi, dil, has_res = case
    bm, bn = tile
    if bn and Co % bn:
        pytest.skip("Co not a multiple of the tile")
    tag = f"w{N}_{Ci}_{Co}_{Hi}_{dil}"
    x = torch.from_numpy(syn.normal(1, "x" + tag, (N, Ci, Hi, Hi), 1.0))
    w = torch.from_numpy(syn.normal(1, "w" + tag, (Co, Ci, 3, 3), (2.0 / (Ci * 9)) ** 0.5))
    scale = torch.from_numpy(syn.uniform(1, "s" + tag, (Co,), 0.5, 1.5))
    shift = torch.from_numpy(syn.normal(1, "b" + tag, (Co,), 0.1))
    res = torch.from_numpy(syn.normal(1, "r" + tag, (N, Co, Hi, Hi), 1.0)) if has_res else None
    y = run_conv_f32d(x, w, scale, shift, 1, dil, dil, res, bm=bm, bn=bn, nsplit=wtile, entry="cwt_debug_conv_x6w")
    ref = ref_conv(x, w, scale, shift, 1, dil, dil, res, True)
    err = float((y.double() - ref).abs().max() / ref.abs().max())
    assert err < (TOL_X6 if wtile == 2 else TOL_X6W4), err


@pytest.mark.parametrize("wtile", [2, 4], ids=lambda m: f"F{m}")
def test_conv_x6_winograd_channel_strided_out(wtile):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    x = torch.from_numpy(syn.normal(2, "xw", (2, 128, 11, 11), 1.0))
    w = torch.from_numpy(syn.normal(2, "ww", (128, 128, 3, 3), 0.04))
    scale, shift = torch.ones(128), torch.zeros(128)
    y = run_conv_f32d(x, w, scale, shift, 1, 2, 2, None, relu=False, y_pad=256, y_off=128, nsplit=wtile,
                      entry="cwt_debug_conv_x6w")
    ref = ref_conv(x, w, scale, shift, 1, 2, 2, None, False)
    assert float((y.double() - ref).abs().max() / ref.abs().max()) < (TOL_X6 if wtile == 2 else TOL_X6W4)


@pytest.mark.parametrize("wtile", [2, 4], ids=lambda m: f"F{m}")
def test_conv_x6_winograd_error_vs_fp32_conv(wtile):
    """Each Winograd form's error against float64 beside a plain fp32 conv's (torch on the CPU),
    on a bottleneck-like conv (post-ReLU input, Ci = 512): F(2x2,3x3), the product form, stays
    within a small multiple of the fp32 conv's own error; F(4x4,3x3) (opt-in) within its bar."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    g = torch.Generator().manual_seed(11)
    x = torch.relu(torch.randn((1, 512, 24, 24), generator=g))
    w = torch.randn((128, 512, 3, 3), generator=g) * (2.0 / (512 * 9)) ** 0.5
    one, zero = torch.ones(128), torch.zeros(128)
    y = run_conv_f32d(x, w, one, zero, 1, 1, 1, None, relu=False, nsplit=wtile, entry="cwt_debug_conv_x6w")
    ref = ref_conv(x, w, one, zero, 1, 1, 1, None, False)
    y32 = F.conv2d(x, w, None, 1, 1, 1).double()
    mx = float(ref.abs().max())
    e_w = float((y.double() - ref).abs().max()) / mx
    e_32 = float((y32 - ref).abs().max()) / mx
    print(f"F({wtile}x{wtile},3x3) max err / max|y|: {e_w:.3g}   torch fp32 conv: {e_32:.3g}")
    if wtile == 2:
        assert e_w < max(4 * e_32, 1e-6), (e_w, e_32)
    else:
        assert e_w < TOL_X6W4, (e_w, e_32)

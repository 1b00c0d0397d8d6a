"""The DeTr head on the device (few_shot_seg_cwt_amd.detr: csrc/detr.hip, the f32-MFMA GEMM,
MatchNet) against oracle/detr_oracle.py in float64.  Parity unpinned (no reference fixture exists
for this head and the reference cannot be run here): the oracle restates
detr.py:13-151, ms_deform_attn.py:84-117 and ms_deform_attn_func.py:41-61 and is itself checked by
tests/test_detr_oracle.py.  Bars (max|HIP - oracle| / max|oracle|): 1e-5 for the linear layers,
the position embedding and the deformable attention, 2e-5 through MatchNet's temp-20 softmax."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


def _rand(shape, seed, lo=-1.0, hi=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(shape, generator=g) * (hi - lo) + lo


@pytest.mark.parametrize("P,K,N,relu,bias", [(3600, 512, 144, False, True), (777, 1024, 512, True, False),
                                             (100, 512, 72, False, True)])
def test_linear(dev, P, K, N, relu, bias):
    from few_shot_seg_cwt_amd.detr import linear
    x, w = _rand((P, K), 1), _rand((N, K), 2) / math.sqrt(K)
    b = _rand((N,), 3) if bias else None
    y = linear(x.to(dev), w.to(dev), b.to(dev) if bias else None, relu=relu)
    ref = torch.nn.functional.linear(x.double(), w.double(), b.double() if bias else None)
    if relu:
        ref = ref.relu()
    e = rel(y, ref)
    print(f"linear P={P} K={K} N={N}: {e:.2e}")
    assert e < 1e-5


def test_linear_accumulate(dev):
    from few_shot_seg_cwt_amd.detr import linear
    x1, x2 = _rand((500, 1024), 4), _rand((500, 2048), 5)
    w = _rand((512, 3072), 6) / math.sqrt(3072)
    out = linear(x1.to(dev), w[:, :1024].contiguous().to(dev))
    linear(x2.to(dev), w[:, 1024:].contiguous().to(dev), relu=True, out=out, accumulate=True)
    ref = torch.relu(torch.cat([x1, x2], 1).double() @ w.double().T)
    e = rel(out, ref)
    print(f"linear over a channel concat (accumulated): {e:.2e}")
    assert e < 1e-5


def test_sine_pos_add(dev):
    from few_shot_seg_cwt_amd.detr import SinePositionalEncoding
    from oracle import detr_oracle as D
    B, C, h, w = 2, 512, 60, 60
    x = _rand((B, C, h, w), 7)
    y = SinePositionalEncoding(C // 2, normalize=True).add_to(x.to(dev))
    ref = x.double() + D.sine_pos_embed(torch.zeros((B, h, w)).long(), C // 2, normalize=True)
    e = rel(y, ref)
    print(f"sine position embedding {h}x{w}: {e:.2e}")
    assert e < 1e-5


def _deform_params(mod, seed):
    """Non-trivial parameters (the reference init zeroes the attention logits' weights)."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for name, p in mod.named_parameters():
            if name.endswith("sampling_offsets.weight"):
                p.copy_((torch.rand(p.shape, generator=g) * 2 - 1) * 0.02)   # offsets of a few pixels
            elif name.endswith("attention_weights.weight"):
                p.copy_((torch.rand(p.shape, generator=g) * 2 - 1) * 0.1)
            elif name.endswith("bias") and "sampling_offsets" not in name:
                p.copy_((torch.rand(p.shape, generator=g) * 2 - 1) * 0.1)


@pytest.mark.parametrize("h,w", [(13, 17), (60, 60)])
def test_deform_att(dev, h, w):
    from few_shot_seg_cwt_amd.detr import DeformAtt
    from oracle import detr_oracle as D
    mod = DeformAtt(embed_dims=512, n_heads=8, n_points=9, device=dev)
    _deform_params(mod, 11)
    fq_fea = _rand((1, 512, h, w), 12, 0.0, 1.0)
    f_q = _rand((1, 512, h, w), 13)
    out = mod(fq_fea.to(dev), f_q.to(dev))
    p = {k[len("self_trans."):]: v.detach().double().cpu() for k, v in mod.state_dict().items()
         if k.startswith("self_trans.")}
    ref = D.deform_att(fq_fea.double(), f_q.double(), p)
    e = rel(out, ref)
    print(f"DeformAtt {h}x{w}: {e:.2e}")
    assert e < 1e-5


def test_ms_deform_attn_reference_init(dev):
    """The reference initialisation (offsets = the head's direction x (point + 1) pixels, uniform
    attention): samples reach past the border, where grid_sample reads zeros."""
    from few_shot_seg_cwt_amd.detr import MSDeformAttn
    from oracle import detr_oracle as D
    torch.manual_seed(0)
    mod = MSDeformAttn(d_model=512, n_levels=1, n_heads=8, n_points=9, device=dev)
    h, w = 9, 11
    q, v = _rand((2, h * w, 512), 14), _rand((2, h * w, 512), 15)
    out = mod(q.to(dev), None, v.to(dev), [[h, w]])
    p = {k: t.detach().double().cpu() for k, t in mod.state_dict().items()}
    ref = D.ms_deform_attn(q.double(), v.double(), h, w, p, 8, 9)
    e = rel(out, ref)
    print(f"MSDeformAttn (reference init) {h}x{w}: {e:.2e}")
    assert e < 1e-5


@pytest.mark.parametrize("cs,sf,h", [(True, False, 20), (False, True, 20), (True, True, 20), (True, True, 60)])
def test_detr_forward(dev, cs, sf, h):
    from few_shot_seg_cwt_amd.detr import DeTr
    from few_shot_seg_cwt_amd.match import init_match_params
    from oracle import detr_oracle as D
    from oracle import match_oracle as MO
    w = h
    args = dict(rmid="l34", temp=20.0, att_wt=0.2)
    torch.manual_seed(1)
    net = DeTr(args, sf_att=sf, cs_att=cs, reduce_dim=512, device=dev)
    with torch.no_grad():
        net.adjust_feature[0].weight.copy_(_rand(tuple(net.adjust_feature[0].weight.shape), 21) / math.sqrt(3072))
    if cs:
        init_match_params(net.cross_trans, 22)
    if sf:
        _deform_params(net.self_trans, 23)
    fq3, fq4 = _rand((1, 1024, h, w), 24, 0.0, 1.0), _rand((1, 2048, h, w), 25, 0.0, 1.0)
    fs3, fs4 = _rand((1, 1024, h, w), 26, 0.0, 1.0), _rand((1, 2048, h, w), 27, 0.0, 1.0)
    f_q, f_s = _rand((1, 512, h, w), 28, 0.0, 1.0), _rand((1, 512, h, w), 29, 0.0, 1.0)
    fq_lst = {2: [None], 3: [fq3.to(dev)], 4: [fq4.to(dev)]}
    fs_lst = {2: [None], 3: [fs3.to(dev)], 4: [fs4.to(dev)]}
    fq, sa, ca = net(fq_lst, fs_lst, f_q.to(dev), f_s.to(dev))
    sd = {k: v.detach().double().cpu() for k, v in net.state_dict().items()}
    layers = MO.layers_from_state(sd, prefix="cross_trans.NeighConsensus.conv.") if cs else None
    dp = {k[len("self_trans.self_trans."):]: v for k, v in sd.items() if k.startswith("self_trans.self_trans.")}
    rq, rsa, rca = D.detr_forward([fq3.double(), fq4.double()], [fs3.double(), fs4.double()], f_q.double(),
                                  f_s.double(), sd["adjust_feature.0.weight"], layers, dp, 20.0, 0.2, cs, sf)
    errs = {"fq": rel(fq, rq)}
    if cs:
        errs["ca"] = rel(ca, rca)
    if sf:
        errs["sa"] = rel(sa, rsa)
    print(f"DeTr cs={cs} sf={sf} {h}x{w}: {errs}")
    assert all(v < 2e-5 for v in errs.values()), errs

"""Backward of the DeTr head on the device (cwt_linear_backward, cwt_deform_attn_backward,
cwt_norm_blend_backward, MatchNet's cwt_match_corr_backward / cwt_corr_backward) against float64
autograd through oracle/detr_oracle.py (detr.py:13-151, ms_deform_attn.py:84-117,
ms_deform_attn_func.py:41-61 with torch's own grid_sample).  Parity unpinned (no reference
fixture for this head).

Bar: every gradient within 1e-4 of float64 autograd, per tensor
max|HIP - oracle| / max|oracle|, printed per case; the loss is a fixed random linear functional
of the outputs."""
import math

import pytest
import torch

from test_gpu_detr import _deform_params, _rand, rel  # noqa: E402

pytestmark = pytest.mark.gpu

TOL = 1e-4


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


@pytest.mark.parametrize("P,K,N,relu,bias", [(900, 512, 144, False, True), (333, 1024, 512, True, False),
                                             (100, 512, 72, False, True), (50, 64, 30, True, True)])
def test_linear_backward(dev, P, K, N, relu, bias):
    from few_shot_seg_cwt_amd.detr import linear_t
    x0, w0 = _rand((P, K), 1).double(), (_rand((N, K), 2) / math.sqrt(K)).double()
    b0 = _rand((N,), 3).double() if bias else None
    G = _rand((P, N), 4).double()
    x = x0.float().to(dev).requires_grad_(True)
    w = w0.float().to(dev).requires_grad_(True)
    b = b0.float().to(dev).requires_grad_(True) if bias else None
    y = linear_t(x, w, b, relu=relu)
    (y * G.float().to(dev)).sum().backward()
    xo, wo = x0.clone().requires_grad_(True), w0.clone().requires_grad_(True)
    bo = b0.clone().requires_grad_(True) if bias else None
    yo = torch.nn.functional.linear(xo, wo, bo)
    if relu:
        yo = yo.relu()
    (yo * G).sum().backward()
    errs = dict(y=rel(y, yo), dx=rel(x.grad, xo.grad), dw=rel(w.grad, wo.grad))
    if bias:
        errs["db"] = rel(b.grad, bo.grad)
    print(f"linear backward P={P} K={K} N={N} relu={relu}: {errs}")
    assert max(errs.values()) < TOL, errs


def test_norm_blend_backward(dev):
    from few_shot_seg_cwt_amd.detr import norm_blend
    a0, b0, G = _rand((2, 512, 7, 9), 5).double(), _rand((2, 512, 7, 9), 6).double(), _rand((2, 512, 7, 9), 7).double()
    a = a0.float().to(dev).requires_grad_(True)
    b = b0.float().to(dev).requires_grad_(True)
    (norm_blend(a, b, 0.3) * G.float().to(dev)).sum().backward()
    ao, bo = a0.clone().requires_grad_(True), b0.clone().requires_grad_(True)
    F = torch.nn.functional
    ((F.normalize(ao, dim=1) + F.normalize(bo, dim=1) * 0.3) * G).sum().backward()
    errs = dict(da=rel(a.grad, ao.grad), db=rel(b.grad, bo.grad))
    print(f"norm_blend backward: {errs}")
    assert max(errs.values()) < TOL, errs


@pytest.mark.parametrize("h,w", [(9, 11), (20, 20)])
def test_deform_att_backward(dev, h, w):
    """DeformAtt (detr.py:78-151, one level): gradients with respect to the query features, the
    sampled values and every MSDeformAttn projection."""
    from few_shot_seg_cwt_amd.detr import DeformAtt
    from oracle import detr_oracle as D
    mod = DeformAtt(embed_dims=512, n_heads=8, n_points=9, device=dev)
    _deform_params(mod, 11)
    fq0, v0 = _rand((1, 512, h, w), 12, 0.0, 1.0).double(), _rand((1, 512, h, w), 13).double()
    G = _rand((1, 512, h, w), 14).double()
    fq = fq0.float().to(dev).requires_grad_(True)
    v = v0.float().to(dev).requires_grad_(True)
    out = mod(fq, v)
    (out * G.float().to(dev)).sum().backward()
    p = {k[len("self_trans."):]: t.detach().double().cpu().requires_grad_(True) for k, t in mod.state_dict().items()
         if k.startswith("self_trans.")}
    fqo, vo = fq0.clone().requires_grad_(True), v0.clone().requires_grad_(True)
    ref = D.deform_att(fqo, vo, p)
    (ref * G).sum().backward()
    errs = dict(out=rel(out, ref), d_fq=rel(fq.grad, fqo.grad), d_v=rel(v.grad, vo.grad))
    for n, t in mod.named_parameters():
        if n.startswith("self_trans."):
            errs[n[len("self_trans."):]] = rel(t.grad, p[n[len("self_trans."):]].grad)
    print(f"DeformAtt backward {h}x{w}: " + ", ".join(f"{k} {e:.1e}" for k, e in errs.items()))
    assert max(errs.values()) < TOL, errs


def test_deform_att_backward_nonfinite(dev):
    """A NaN / Inf in the upstream gradient reaches d_value as it does through the reference's float
    atomics (the fixed-point scatter used to turn it into large finite garbage): every
    position whose oracle gradient is non-finite is non-finite here, and the finite rest still
    matches float64 autograd."""
    from few_shot_seg_cwt_amd.detr import DeformAtt
    from oracle import detr_oracle as D
    h, w = 9, 11
    mod = DeformAtt(embed_dims=512, n_heads=8, n_points=9, device=dev)
    _deform_params(mod, 11)
    fq0, v0 = _rand((1, 512, h, w), 12, 0.0, 1.0).double(), _rand((1, 512, h, w), 13).double()
    G = _rand((1, 512, h, w), 14).double()
    G[0, 5, 4, 6] = float("nan")
    G[0, 7, 2, 3] = float("inf")
    fq = fq0.float().to(dev).requires_grad_(True)
    v = v0.float().to(dev).requires_grad_(True)
    (mod(fq, v) * G.float().to(dev)).sum().backward()
    p = {k[len("self_trans."):]: t.detach().double().cpu().requires_grad_(True) for k, t in mod.state_dict().items()
         if k.startswith("self_trans.")}
    vo = v0.clone().requires_grad_(True)
    (D.deform_att(fq0.clone(), vo, p) * G).sum().backward()
    hip, ref = v.grad.detach().cpu().double(), vo.grad
    bad_ref = ~torch.isfinite(ref)
    print(f"non-finite d_v entries: oracle {int(bad_ref.sum())}, HIP {int((~torch.isfinite(hip)).sum())}")
    assert bad_ref.any()
    assert not torch.isfinite(hip[bad_ref]).any()
    ok = torch.isfinite(hip) & ~bad_ref
    assert float((hip[ok] - ref[ok]).abs().max()) <= TOL * float(ref[ok].abs().max())


@pytest.mark.parametrize("cs,sf", [(True, False), (True, True)])
def test_detr_backward(dev, cs, sf):
    """DeTr.forward (detr.py:36-47) as train_trans.py trains it: gradients of a linear functional of
    the blended query map with respect to adjust_feature, the MatchNet layers, the deformable
    attention and the layer features."""
    from few_shot_seg_cwt_amd.detr import DeTr
    from few_shot_seg_cwt_amd.match import init_match_params
    from oracle import detr_oracle as D
    from oracle import match_oracle as MO
    h = w = 8
    args = dict(rmid="l34", temp=20.0, att_wt=0.2)
    torch.manual_seed(1)
    net = DeTr(args, sf_att=sf, cs_att=cs, reduce_dim=512, device=dev)
    with torch.no_grad():
        net.adjust_feature[0].weight.copy_(_rand(tuple(net.adjust_feature[0].weight.shape), 21) / math.sqrt(3072))
        if cs:
            init_match_params(net.cross_trans, 22)
            net.cross_trans.NeighConsensus.conv[4].conv1.bias.add_(0.2)
    if sf:
        _deform_params(net.self_trans, 23)
    feats0 = [_rand((1, c, h, w), s, 0.0, 1.0).double() for c, s in ((1024, 24), (2048, 25), (1024, 26), (2048, 27))]
    fq0, fs0 = _rand((1, 512, h, w), 28, 0.0, 1.0).double(), _rand((1, 512, h, w), 29, 0.0, 1.0).double()
    G = _rand((1, 512, h, w), 30).double()
    feats = [f.float().to(dev).requires_grad_(True) for f in feats0]
    f_q = fq0.float().to(dev).requires_grad_(True)
    f_s = fs0.float().to(dev).requires_grad_(True)
    fq_lst = {3: [feats[0]], 4: [feats[1]]}
    fs_lst = {3: [feats[2]], 4: [feats[3]]}
    out, _, _ = net(fq_lst, fs_lst, f_q, f_s)
    (out * G.float().to(dev)).sum().backward()
    # deterministic: a second forward + backward in the same process gives bitwise the same
    # gradients (the deformable attention's d_value in fixed point, the bias sums in fixed order)
    first = {n: t.grad.clone() for n, t in net.named_parameters() if t.grad is not None}
    first.update({f"feat{i}": f.grad.clone() for i, f in enumerate(feats)})
    first.update(f_q=f_q.grad.clone(), f_s=f_s.grad.clone())
    for t in list(net.parameters()) + feats + [f_q, f_s]:
        t.grad = None
    out2, _, _ = net(fq_lst, fs_lst, f_q, f_s)
    (out2 * G.float().to(dev)).sum().backward()
    assert torch.equal(out2, out)
    second = {n: t.grad for n, t in net.named_parameters() if t.grad is not None}
    second.update({f"feat{i}": f.grad for i, f in enumerate(feats)})
    second.update(f_q=f_q.grad, f_s=f_s.grad)
    assert first.keys() == second.keys()
    assert all(torch.equal(first[k], second[k]) for k in first), [k for k in first if not torch.equal(first[k], second[k])]
    sd = {k: t.detach().double().cpu().requires_grad_(True) for k, t in net.state_dict().items()}
    layers = MO.layers_from_state(sd, prefix="cross_trans.NeighConsensus.conv.") if cs else None
    dp = {k[len("self_trans.self_trans."):]: t for k, t in sd.items() if k.startswith("self_trans.self_trans.")}
    fo = [f.clone().requires_grad_(True) for f in feats0]
    fqo, fso = fq0.clone().requires_grad_(True), fs0.clone().requires_grad_(True)
    ro, _, _ = D.detr_forward(fo[:2], fo[2:], fqo, fso, sd["adjust_feature.0.weight"], layers, dp, 20.0, 0.2, cs, sf)
    (ro * G).sum().backward()
    errs = dict(out=rel(out, ro), d_fq=rel(f_q.grad, fqo.grad), d_fs=rel(f_s.grad, fso.grad))
    for i in range(4):
        errs[f"d_feat{i}"] = rel(feats[i].grad, fo[i].grad)
    for n, t in net.named_parameters():
        if t.grad is not None or sd[n].grad is not None:
            errs[n] = rel(t.grad, sd[n].grad)
    print(f"DeTr backward cs={cs} sf={sf}: " + ", ".join(f"{k} {e:.1e}" for k, e in errs.items()))
    assert max(errs.values()) < TOL, errs

"""Backward of the MatchNet / MMN head on the device (csrc/match_bwd.hip: cwt_match_corr_backward,
cwt_corr_backward, cwt_weight_average_backward, cwt_mmn_blend_backward) against float64
autograd through oracle/match_oracle.py, the restatement of match.py:21-163, conv4d.py:40-62,
msm_func.py:50-104, model_util.py:101-109 and mmn.py:42-71.  Parity unpinned (the reference holds
no fixture for this head): these check the device gradients against autograd of
the same float64 restatement the forward tests use.

Bar: every gradient within 1e-4 of float64 autograd, measured per tensor as
max|HIP - oracle| / max|oracle|, printed per case.  The loss is a fixed random linear functional
of the outputs, so every output element carries gradient."""
import pytest
import torch

pytestmark = pytest.mark.gpu

TOL = 1e-4


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


def _rand(shape, seed, lo=0.0, hi=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(*shape, generator=g, dtype=torch.float64) * (hi - lo) + lo


@pytest.mark.parametrize("B,Pq,Pk,C", [(2, 36, 36, 64), (1, 25, 49, 512), (1, 64, 64, 1024)])
def test_corr_backward(dev, B, Pq, Pk, C):
    """get_corr (model_util.py:101-109): dq, dk of <G, normalize(q) normalize(k)^T>."""
    from few_shot_seg_cwt_amd.heads import get_corr
    q0, k0 = _rand((B, C, Pq, 1), 1) - 0.3, _rand((B, C, Pk, 1), 2) - 0.3
    G = _rand((B, Pq, Pk), 3, -1, 1)
    q = q0.float().to(dev).requires_grad_(True)
    k = k0.float().to(dev).requires_grad_(True)
    sim = get_corr(q, k)
    (sim * G.float().to(dev)).sum().backward()
    qo, ko = q0.clone().requires_grad_(True), k0.clone().requires_grad_(True)
    so = torch.bmm(torch.nn.functional.normalize(qo.reshape(B, C, Pq), dim=1).transpose(1, 2),
                   torch.nn.functional.normalize(ko.reshape(B, C, Pk), dim=1))
    (so * G).sum().backward()
    errs = dict(sim=rel(sim, so), dq=rel(q.grad, qo.grad), dk=rel(k.grad, ko.grad))
    print(f"corr backward B={B} {Pq}x{Pk} C={C}: {errs}")
    assert max(errs.values()) < TOL, errs


@pytest.mark.parametrize("N,C,h,w", [(2, 512, 6, 7), (1, 1024, 5, 5), (1, 2048, 4, 6)])
def test_weight_average_backward(dev, N, C, h, w):
    """msm_func.py:50-104: d x and every parameter gradient of WeightAverage."""
    from few_shot_seg_cwt_amd.match import WeightAverage, init_match_params
    from oracle import match_oracle as M
    m = WeightAverage(C, {}, device=dev)
    init_match_params(m, seed=C + h)
    x0 = _rand((N, C, h, w), C)
    G = _rand((N, C, h, w), C + 1, -1, 1)
    x = x0.float().to(dev).requires_grad_(True)
    y = m(x)
    (y * G.float().to(dev)).sum().backward()
    names = ["conv_theta.weight", "conv_theta.bias", "conv_phi.weight", "conv_phi.bias", "conv_g.weight",
             "conv_g.bias", "conv_back.weight", "conv_back.bias"]
    sd = {k: t.detach().cpu().double().requires_grad_(True) for k, t in m.state_dict().items()}
    xo = x0.clone().requires_grad_(True)
    yo = M.weight_average(xo, tuple(sd[n] for n in names))
    (yo * G).sum().backward()
    params = dict(m.named_parameters())
    errs = dict(y=rel(y, yo), dx=rel(x.grad, xo.grad))
    for n in names:
        errs[n] = rel(params[n].grad, sd[n].grad)
    print(f"WeightAverage backward N={N} C={C} {h}x{w}: " + ", ".join(f"{k} {v:.1e}" for k, v in errs.items()))
    assert max(errs.values()) < TOL, errs


def _net(dev, L, sym, temp, seed):
    from few_shot_seg_cwt_amd.match import MatchNet, init_match_params
    net = MatchNet(temp=temp, in_channel=L, sym_mode=sym, device=dev)
    init_match_params(net, seed)
    with torch.no_grad():   # keep the one-channel last layer's ReLU open somewhere (a live gradient)
        net.NeighConsensus.conv[4].conv1.bias.add_(0.2)
    return net


@pytest.mark.parametrize("B,L,h,w,sym", [(1, 1, 6, 6, True), (2, 2, 5, 7, True), (1, 1, 7, 5, False),
                                         (1, 2, 12, 12, True)])
def test_corr_forward_backward(dev, B, L, h, w, sym):
    """match.py:142-163: gradients of <G1, corr2d> + <G2, weighted_v> with respect to the input
    correlation, the NeighConsensus parameters and v."""
    from oracle import match_oracle as M
    temp = 20.0
    net = _net(dev, L, sym, temp, seed=11 + L + h)
    c0 = _rand((B, L, h, w, h, w), 5 * h + w, -0.2, 1.0)
    v0 = _rand((B, 64, h, w), 13)
    G1 = _rand((B, h * w, h * w), 17, -1, 1)
    G2 = _rand((B, 64, h, w), 19, -1, 1)
    corr = c0.float().to(dev).requires_grad_(True)
    v = v0.float().to(dev).requires_grad_(True)
    corr2d, wv = net.corr_forward(corr, v, ret_attn=True)
    ((corr2d * G1.float().to(dev)).sum() + (wv * G2.float().to(dev)).sum()).backward()
    names = [f"NeighConsensus.conv.{i}.{c}.{p}" for i in (0, 2, 4) for c in ("conv1", "conv2") for p in ("weight", "bias")]
    sd = {k: t.detach().cpu().double().requires_grad_(True) for k, t in net.state_dict().items()}
    layers = M.layers_from_state(sd)
    co, vo = c0.clone().requires_grad_(True), v0.clone().requires_grad_(True)
    c2o, wvo = M.corr_forward(co, vo, layers, temp, sym)
    ((c2o * G1).sum() + (wvo * G2).sum()).backward()
    params = dict(net.named_parameters())
    assert float(co.grad.abs().max()) > 0 and float(sd[names[-1]].grad.abs().max()) > 0   # not a dead stack
    errs = dict(corr2d=rel(corr2d, c2o), wv=rel(wv, wvo), d_corr=rel(corr.grad, co.grad), d_v=rel(v.grad, vo.grad))
    for n in names:
        errs[n.replace("NeighConsensus.conv.", "")] = rel(params[n].grad, sd[n].grad)
    print(f"corr_forward backward B={B} L={L} {h}x{w} sym={sym}: " + ", ".join(f"{k} {e:.1e}" for k, e in errs.items()))
    assert max(errs.values()) < TOL, errs


def test_corr_backward_deterministic(dev):
    """Fixed-order reductions: two backward passes give bit-identical gradients."""
    net = _net(dev, 2, True, 20.0, seed=3)
    c = _rand((1, 2, 8, 8, 8, 8), 4, -0.2, 1.0).float().to(dev)
    v = _rand((1, 64, 8, 8), 5).float().to(dev)
    G = _rand((1, 64, 8, 8), 6, -1, 1).float().to(dev)
    grads = []
    for _ in range(2):
        net.zero_grad()
        x = c.clone().requires_grad_(True)
        _, wv = net.corr_forward(x, v, ret_attn=True)
        (wv * G).sum().backward()
        grads.append([x.grad.clone()] + [p.grad.clone() for p in net.parameters()])
    for a, b in zip(*grads):
        assert torch.equal(a, b)


def test_mmn_backward(dev):
    """mmn.py:42-71 (rmid l34, all_lr l, agg cat, wa True, two shots): gradients of a linear
    functional of (fq, att_fq) with respect to every MMN parameter (WeightAverage of both layers,
    the NeighConsensus layers) and the layer features."""
    from few_shot_seg_cwt_amd.match import MMN, init_match_params
    from oracle import match_oracle as M
    args = dict(rmid="l34", layers=50, all_lr="l", temp=20.0, att_wt=0.3, conv4d="red")
    net = MMN(args, agg="cat", wa=True, red_dim=False, device=dev)
    init_match_params(net, seed=9)
    h, B = 6, 2
    fq0 = {3: _rand((1, 1024, h, h), 31), 4: _rand((1, 2048, h, h), 32)}
    fs0 = {3: _rand((B, 1024, h, h), 33), 4: _rand((B, 2048, h, h), 34)}
    fq_in, fs_in = _rand((1, 512, h, h), 35), _rand((B, 512, h, h), 36)
    G1, G2 = _rand((1, 512, h, h), 37, -1, 1), _rand((1, 512, h, h), 38, -1, 1)
    fq_d = {k: [t.float().to(dev).requires_grad_(True)] for k, t in fq0.items()}
    fs_d = {k: [t.float().to(dev).requires_grad_(True)] for k, t in fs0.items()}
    fq, att_fq = net(fq_d, fs_d, fq_in.float().to(dev), fs_in.float().to(dev))
    ((fq * G1.float().to(dev)).sum() + (att_fq * G2.float().to(dev)).sum()).backward()
    sd = {k: t.detach().cpu().double().requires_grad_(True) for k, t in net.state_dict().items()}
    wa = {b: M.wa_params_from_state(sd, f"wa_{b}.") for b in (3, 4)}
    layers = M.layers_from_state(sd, prefix="corr_net.NeighConsensus.conv.")
    fq_o = {k: t.clone().requires_grad_(True) for k, t in fq0.items()}
    fs_o = {k: t.clone().requires_grad_(True) for k, t in fs0.items()}
    fqo, atto = M.mmn_forward(fq_o, fs_o, fq_in, fs_in, [3, 4], wa, layers, 20.0, 0.3)
    ((fqo * G1).sum() + (atto * G2).sum()).backward()
    errs = dict(fq=rel(fq, fqo), att_fq=rel(att_fq, atto))
    for k in (3, 4):
        errs[f"d_fq{k}"] = rel(fq_d[k][0].grad, fq_o[k].grad)
        errs[f"d_fs{k}"] = rel(fs_d[k][0].grad, fs_o[k].grad)
    for n, p in net.named_parameters():
        errs[n] = rel(p.grad, sd[n].grad)
    print("MMN backward: " + ", ".join(f"{k} {e:.1e}" for k, e in errs.items()))
    assert max(errs.values()) < TOL, errs


def test_mmn_no_grad_matches_train_path(dev):
    """The inference path (no_grad) and the autograd path give the same forward values."""
    from few_shot_seg_cwt_amd.match import MMN, init_match_params
    args = dict(rmid="l34", layers=50, all_lr="l", temp=20.0, att_wt=0.3, conv4d="red")
    net = MMN(args, agg="cat", wa=True, red_dim=False, device=dev)
    init_match_params(net, seed=2)
    h = 8
    fq = {3: [_rand((1, 1024, h, h), 1).float().to(dev)], 4: [_rand((1, 2048, h, h), 2).float().to(dev)]}
    fs = {3: [_rand((1, 1024, h, h), 3).float().to(dev)], 4: [_rand((1, 2048, h, h), 4).float().to(dev)]}
    f_q, f_s = _rand((1, 512, h, h), 5).float().to(dev), _rand((1, 512, h, h), 6).float().to(dev)
    with torch.no_grad():
        a = net(fq, fs, f_q, f_s)
    b = net(fq, fs, f_q, f_s)
    for x, y in zip(a, b):
        assert torch.equal(x, y.detach())


@pytest.mark.parametrize("agg,red_dim", [("sum", False), ("cat", 512)])
def test_mmn_backward_agg_red_dim(dev, agg, red_dim):
    """MMN with agg 'sum' (mmn.py:62-63) and with red_dim (rd_<layer> 1x1 conv + ReLU, mmn.py:28-31,
    49-51): parameter and feature gradients against the oracle chain."""
    from few_shot_seg_cwt_amd.match import MMN, init_match_params
    from oracle import match_oracle as M
    args = dict(rmid="l34", layers=50, all_lr="l", temp=20.0, att_wt=0.3, conv4d="red")
    net = MMN(args, agg=agg, wa=True, red_dim=red_dim, device=dev)
    init_match_params(net, seed=12)
    h, B = 6, 2
    fq0 = {3: _rand((1, 1024, h, h), 41), 4: _rand((1, 2048, h, h), 42)}
    fs0 = {3: _rand((B, 1024, h, h), 43), 4: _rand((B, 2048, h, h), 44)}
    fq_in, fs_in = _rand((1, 512, h, h), 45), _rand((B, 512, h, h), 46)
    G = _rand((1, 512, h, h), 47, -1, 1)
    fq_d = {k: [t.float().to(dev).requires_grad_(True)] for k, t in fq0.items()}
    fs_d = {k: [t.float().to(dev).requires_grad_(True)] for k, t in fs0.items()}
    _, att_fq = net(fq_d, fs_d, fq_in.float().to(dev), fs_in.float().to(dev))
    (att_fq * G.float().to(dev)).sum().backward()
    sd = {k: t.detach().cpu().double().requires_grad_(True) for k, t in net.state_dict().items()}
    wa = {b: M.wa_params_from_state(sd, f"wa_{b}.") for b in (3, 4)}
    rdw = {b: sd[f"rd_{b}.0.weight"] for b in (3, 4)} if red_dim else None
    layers = M.layers_from_state(sd, prefix="corr_net.NeighConsensus.conv.")
    fq_o = {k: t.clone().requires_grad_(True) for k, t in fq0.items()}
    fs_o = {k: t.clone().requires_grad_(True) for k, t in fs0.items()}
    _, atto = M.mmn_forward(fq_o, fs_o, fq_in, fs_in, [3, 4], wa, layers, 20.0, 0.3, agg=agg, rd_weights=rdw)
    (atto * G).sum().backward()
    errs = dict(att_fq=rel(att_fq, atto))
    for k in (3, 4):
        errs[f"d_fq{k}"] = rel(fq_d[k][0].grad, fq_o[k].grad)
        errs[f"d_fs{k}"] = rel(fs_d[k][0].grad, fs_o[k].grad)
    for n, p in net.named_parameters():
        errs[n] = rel(p.grad, sd[n].grad)
    print(f"MMN backward agg={agg} red_dim={red_dim}: " + ", ".join(f"{k} {e:.1e}" for k, e in errs.items()))
    assert max(errs.values()) < TOL, errs


def _get_corr64(fq, fs):
    """heads.get_corr in float64: cosine similarity of every query / support pixel pair."""
    B, C, h, w = fq.shape
    nq = torch.nn.functional.normalize(fq, dim=1).reshape(B, C, h * w)
    ns = torch.nn.functional.normalize(fs, dim=1).reshape(B, C, h * w)
    return torch.bmm(nq.transpose(1, 2), ns).reshape(B, 1, h, w, h, w)


@pytest.mark.parametrize("use_ig,use_cyc,train", [(True, False, False), (False, True, False), (True, True, True)])
def test_forward_masks_backward(dev, use_ig, use_cyc, train):
    """MatchNet.forward with ig_mask and / or the cycle mask under autograd (match.py:103-130,
    165-182; train_tp_match.py:188, train_match.py:164): gradients of <G1, weighted_v> +
    <G2, masked corr2d> with respect to v and every NeighConsensus parameter, against float64
    autograd through the oracle chain.  The cycle mask (argmax decisions, and in training mode its
    Dropout draw) is the device's own, a constant under autograd in both."""
    from oracle import match_oracle as M
    B, C, h, w, Cv, temp = 2, 64, 7, 8, 48, 20.0
    net = _net(dev, 1, True, temp, seed=41)
    net.cyc = use_cyc
    net.train(train)
    g = torch.Generator().manual_seed(42)
    fq0, fs0 = torch.rand(B, C, h, w, generator=g).double(), torch.rand(B, C, h, w, generator=g).double()
    v0 = torch.randn(B, Cv, h, w, generator=g).double()
    ig = (torch.rand(B, h * w, generator=g) < 0.25) if use_ig else None
    sm = (torch.rand(B, h, w, generator=g) < 0.4).long() if use_cyc else None
    G1, G2 = _rand((B, Cv, h, w), 43, -1, 1), _rand((B, h * w, h * w), 44, -1, 1)
    v = v0.float().to(dev).requires_grad_(True)
    host_rng = torch.get_rng_state()
    out = net(fq0.float().to(dev), fs0.float().to(dev), v, s_mask=sm.to(dev) if use_cyc else None,
              ig_mask=ig.to(dev) if use_ig else None, ret_corr=True, use_cyc=use_cyc, ret_cyc=use_cyc)
    # the train-mode Dropout draw leaves the host RNG stream (the W0 draws) untouched, as the
    # reference's nn.Dropout on a CUDA tensor does
    assert torch.equal(torch.get_rng_state(), host_rng)
    wv, corr = out[0], out[1]
    ((wv * G1.float().to(dev)).sum() + (corr.reshape(B, h * w, h * w) * G2.float().to(dev)).sum()).backward()
    names = [f"NeighConsensus.conv.{i}.{c}.{p}" for i in (0, 2, 4) for c in ("conv1", "conv2") for p in ("weight", "bias")]
    sd = {k: t.detach().cpu().double().requires_grad_(True) for k, t in net.state_dict().items()}
    vo = v0.clone().requires_grad_(True)
    c2 = M.run_match_model(_get_corr64(fq0, fs0), M.layers_from_state(sd), True).reshape(B, h * w, h * w)
    if use_ig:
        c2 = c2.masked_fill(ig.reshape(B, 1, h * w).expand(c2.shape), 0.0001)
    if use_cyc:
        inc = out[2][:, 0].detach().cpu().double()
        c2 = c2 + inc.unsqueeze(1) * (-1000.0)
        if train:
            assert set(torch.unique(inc).tolist()) <= {0.0, float(torch.tensor(1 / 0.9, dtype=torch.float32))}
    attn = torch.softmax(c2 * temp, dim=-1)
    wvo = torch.bmm(vo.reshape(B, Cv, h * w), attn.transpose(1, 2)).reshape(B, Cv, h, w)
    ((wvo * G1).sum() + (c2 * G2).sum()).backward()
    params = dict(net.named_parameters())
    errs = dict(wv=rel(wv, wvo), corr2d=rel(corr.reshape(B, h * w, h * w), c2), d_v=rel(v.grad, vo.grad))
    for n in names:
        errs[n.replace("NeighConsensus.conv.", "")] = rel(params[n].grad, sd[n].grad)
    print(f"MatchNet masks backward ig={use_ig} cyc={use_cyc} train={train}: "
          + ", ".join(f"{k} {e:.1e}" for k, e in errs.items()))
    assert float(sd[names[0]].grad.abs().max()) > 0
    assert max(errs.values()) < TOL, errs


def test_sce_backward(dev):
    """MatchNet(sce=True) training (train_match.py:104 sce=args.sce): the spatial context encoder's
    1x1 conv weight and bias (spatial_context.py:84-87), the NeighConsensus parameters and v get
    their gradients; the frozen features carry none (the reference cannot differentiate its
    descriptor).  Against float64 autograd through the oracle chain."""
    from few_shot_seg_cwt_amd.match import MatchNet, init_match_params
    from oracle import match_oracle as M
    B, C, h, w, Cv, temp = 1, 2048, 6, 7, 32, 20.0
    net = MatchNet(temp=temp, sce=True, device=dev)
    init_match_params(net, 51)
    with torch.no_grad():
        net.NeighConsensus.conv[4].conv1.bias.add_(0.2)
    g = torch.Generator().manual_seed(52)
    # zero-mean features: with all-positive ones the encoder's outputs are nearly parallel (cosines
    # near 1), and the last consensus layer's two scalar bias gradients -- sums over every pair with
    # heavy cancellation -- inherit the fp32 rounding of corr2d amplified (8e-4 measured); the
    # gradient code is the same either way
    fq0, fs0 = torch.randn(B, C, h, w, generator=g).double(), torch.randn(B, C, h, w, generator=g).double()
    v0 = torch.randn(B, Cv, h, w, generator=g).double()
    G = _rand((B, Cv, h, w), 53, -1, 1)
    v = v0.float().to(dev).requires_grad_(True)
    wv = net(fq0.float().to(dev), fs0.float().to(dev), v)
    (wv * G.float().to(dev)).sum().backward()
    sd = {k: t.detach().cpu().double().requires_grad_(True) for k, t in net.state_dict().items()}
    W, b = sd["SpatialContextEncoder.embeddingFea.0.weight"], sd["SpatialContextEncoder.embeddingFea.0.bias"]
    eq = M.spatial_context_encoder(torch.nn.functional.normalize(fq0, dim=1), 25, W, b)
    es = M.spatial_context_encoder(torch.nn.functional.normalize(fs0, dim=1), 25, W, b)
    vo = v0.clone().requires_grad_(True)
    _, wvo = M.corr_forward(_get_corr64(eq, es), vo, M.layers_from_state(sd), temp, True)
    (wvo * G).sum().backward()
    params = dict(net.named_parameters())
    errs = dict(wv=rel(wv, wvo), d_v=rel(v.grad, vo.grad))
    for n in ["SpatialContextEncoder.embeddingFea.0.weight", "SpatialContextEncoder.embeddingFea.0.bias"] + \
            [f"NeighConsensus.conv.{i}.{c}.{p}" for i in (0, 2, 4) for c in ("conv1", "conv2") for p in ("weight", "bias")]:
        errs[n.split(".", 1)[1] if n.startswith("NeighConsensus") else n.split(".")[-1]] = rel(params[n].grad, sd[n].grad)
    print("MatchNet sce backward: " + ", ".join(f"{k} {e:.1e}" for k, e in errs.items()))
    assert float(W.grad.abs().max()) > 0
    assert max(errs.values()) < TOL, errs

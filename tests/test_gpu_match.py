"""MatchNet's 4-D matching head on the device (few_shot_seg_cwt_amd.match, csrc/match.hip)
against oracle/match_oracle.py in float64.  Parity unpinned (no reference fixture exists for
this head): the oracle restates match.py:21-163 / conv4d.py:11-62 and is itself
checked by tests/test_match_oracle.py.  Bar: 2e-5 relative (max|HIP - oracle| / max|oracle|),
printed per case; the softmax at temp 20 multiplies the score error by the temperature."""
import pytest
import torch

pytestmark = pytest.mark.gpu

TOL = 2e-5


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


def _net(dev, L, sym, temp, seed):
    from few_shot_seg_cwt_amd.match import MatchNet, init_match_params
    net = MatchNet(temp=temp, in_channel=L, sym_mode=sym, device=dev)
    init_match_params(net, seed)
    return net


def _corr(dev, B, L, h, w, seed):
    g = torch.Generator().manual_seed(seed)
    # cosine-like scores in [-1, 1], most of them positive (normalised ReLU features)
    c = torch.rand(B, L, h, w, h, w, generator=g) * 1.2 - 0.2
    return c.to(dev)


@pytest.mark.parametrize("C", [1, 2, 3])  # 1 / 2: the vector kernels; 3: the scalar forms
def test_mutual_matching(dev, C):
    from few_shot_seg_cwt_amd.match import MutualMatching
    from oracle import match_oracle as M
    g = torch.Generator().manual_seed(7)
    x = (torch.rand(2, C, 5, 7, 6, 4, generator=g) * 2 - 1).to(dev)
    y = MutualMatching(x)
    e = rel(y, M.mutual_matching(x.double().cpu()))
    print(f"MutualMatching C={C}: {e:.2e}")
    assert e < 1e-6


@pytest.mark.parametrize("B,L,h,w,sym", [(1, 1, 12, 12, True), (2, 2, 9, 13, True), (1, 1, 11, 7, False),
                                         (1, 2, 30, 30, True)])
def test_corr_forward(dev, B, L, h, w, sym):
    from oracle import match_oracle as M
    temp = 20.0
    net = _net(dev, L, sym, temp, seed=11 + L)
    corr = _corr(dev, B, L, h, w, seed=5 * h + w)
    g = torch.Generator().manual_seed(13)
    v = torch.rand(B, 64, h, w, generator=g).to(dev)
    corr2d, wv = net.corr_forward(corr, v, ret_attn=True)
    torch.cuda.synchronize()
    layers = M.layers_from_state({k: t.cpu() for k, t in net.state_dict().items()})
    c2o, wvo = M.corr_forward(corr.double().cpu(), v.double().cpu(), layers, temp, sym)
    errs = dict(corr2d=rel(corr2d, c2o), weighted_v=rel(wv, wvo))
    print(f"corr_forward B={B} L={L} {h}x{w} sym={sym}: {errs}")
    assert max(errs.values()) < TOL, errs


def test_forward_from_features_and_state_dict_keys(dev):
    """MatchNet.forward (match.py:103-140): get_corr of the features -> run_match_model ->
    softmax -> bmm; the module's state_dict carries the reference's key names."""
    from oracle import match_oracle as M
    from oracle.cwt_oracle import get_corr as corr_o
    net = _net(dev, 1, True, 20.0, seed=3)
    keys = list(net.state_dict().keys())
    assert keys == [f"NeighConsensus.conv.{i}.{c}.{p}" for i in (0, 2, 4) for c in ("conv1", "conv2")
                    for p in ("weight", "bias")]
    g = torch.Generator().manual_seed(17)
    fq = torch.rand(1, 64, 10, 10, generator=g).to(dev)
    fs = torch.rand(1, 64, 10, 10, generator=g).to(dev)
    v = torch.rand(1, 32, 10, 10, generator=g).to(dev)
    wv = net(fq, fs, v)
    layers = M.layers_from_state({k: t.cpu() for k, t in net.state_dict().items()})
    c = corr_o(fq.double().cpu(), fs.double().cpu()).reshape(1, 1, 10, 10, 10, 10)
    _, wvo = M.corr_forward(c, v.double().cpu(), layers, 20.0, True)
    e = rel(wv, wvo)
    print(f"MatchNet.forward: {e:.2e}")
    assert e < TOL


@pytest.mark.parametrize("N,C,h,w", [(2, 512, 9, 11), (1, 2048, 7, 7), (1, 1024, 6, 5)])
def test_weight_average(dev, N, C, h, w):
    """msm_func.py:50-104 (R 3) against the float64 restatement."""
    from few_shot_seg_cwt_amd.match import WeightAverage, init_match_params
    from oracle import match_oracle as M
    m = WeightAverage(C, {}, device=dev)
    init_match_params(m, seed=C + h)
    g = torch.Generator().manual_seed(C)
    x = torch.rand(N, C, h, w, generator=g).to(dev)
    y = m(x)
    sd = {k: t.cpu() for k, t in m.state_dict().items()}
    yo = M.weight_average(x.double().cpu(), M.wa_params_from_state(sd, ""))
    e = rel(y, yo)
    print(f"WeightAverage N={N} C={C} {h}x{w}: {e:.2e}")
    assert e < TOL


def test_mmn_forward(dev):
    """mmn.py:42-71 (rmid l34, all_lr l, agg cat, wa True) on random layer features, 2 shots."""
    from few_shot_seg_cwt_amd.match import MMN, init_match_params
    from oracle import match_oracle as M
    args = dict(rmid="l34", layers=50, all_lr="l", temp=20.0, att_wt=0.2, conv4d="red")
    net = MMN(args, agg="cat", wa=True, red_dim=False, device=dev)
    init_match_params(net, seed=5)
    g = torch.Generator().manual_seed(23)
    h = 8
    fq_lst = {3: [torch.rand(1, 1024, h, h, generator=g).to(dev)], 4: [torch.rand(1, 2048, h, h, generator=g).to(dev)]}
    fs_lst = {3: [torch.rand(2, 1024, h, h, generator=g).to(dev)], 4: [torch.rand(2, 2048, h, h, generator=g).to(dev)]}
    f_q = torch.rand(1, 512, h, h, generator=g).to(dev)
    f_s = torch.rand(2, 512, h, h, generator=g).to(dev)
    fq, att_fq = net(fq_lst, fs_lst, f_q, f_s)
    sd = {k: t.cpu() for k, t in net.state_dict().items()}
    wa = {b: M.wa_params_from_state(sd, f"wa_{b}.") for b in (3, 4)}
    layers = M.layers_from_state(sd, prefix="corr_net.NeighConsensus.conv.")
    d = lambda t: t.double().cpu()  # noqa: E731
    fqo, atto = M.mmn_forward({k: d(v[0]) for k, v in fq_lst.items()}, {k: d(v[0]) for k, v in fs_lst.items()},
                              d(f_q), d(f_s), [3, 4], wa, layers, 20.0, 0.2)
    errs = dict(fq=rel(fq, fqo), att_fq=rel(att_fq, atto))
    print(f"MMN.forward: {errs}")
    assert max(errs.values()) < TOL, errs


def test_extract_mid_features(dev):
    """extract_features with rmid 'l34' (pspnet.py:172-181): the layer2/3/4 outputs beside the
    usual feature map, against the oracle's float64 backbone (bf16x3 convs: bar 1e-4)."""
    from few_shot_seg_cwt_amd import PSPNet
    from few_shot_seg_cwt_amd import synthetic as syn
    from oracle import match_oracle as M
    from oracle.cwt_oracle import to_torch_state
    sd = syn.make_pspnet_state(50, 2021)
    args = dict(layers=50, rmid="l34", all_lr="l")
    net = PSPNet(args)
    net.load_state_dict(sd)
    x = torch.from_numpy(syn.normal(2021, "mid_img", (2, 3, 65, 65), 1.0)).to(dev)
    f, lst = net.extract_features(x)
    plain = PSPNet(dict(layers=50))
    plain.load_state_dict(sd)
    f0, empty = plain.extract_features(x)
    torch.cuda.synchronize()
    assert empty == [] and sorted(lst) == [2, 3, 4]
    assert torch.equal(f, f0)
    sd64 = {k: v.double() for k, v in to_torch_state(sd).items()}
    ref = M.feat_list(x.double().cpu(), sd64, 50)
    errs = {k: rel(lst[k][0], ref[k]) for k in (2, 3, 4)}
    print(f"mid features: {errs}")
    assert max(errs.values()) < 1e-4, errs


@pytest.mark.parametrize("use_ig,use_cyc", [(True, False), (False, True), (True, True)])
def test_forward_support_masks(dev, use_ig, use_cyc):
    """MatchNet.forward's ig_mask and cycle mask (match.py:117-126, 165-182).  The masks are
    checked on the device's own corr2d (argmax decisions on float64 values would differ only at
    ties the fp32 rounding creates): the oracle applies support_masks to the unmasked corr2d the
    device returns, the inconsistent mask must match exactly, the masked corr2d and weighted_v at
    2e-5 (weighted_v against the float64 softmax readout of the oracle's masked corr2d)."""
    from few_shot_seg_cwt_amd.match import MatchNet, init_match_params
    from oracle import match_oracle as M
    B, C, h, w, Cv = 2, 64, 9, 11, 48
    g = torch.Generator().manual_seed(31)
    fq = torch.rand(B, C, h, w, generator=g).to(dev)
    fs = torch.rand(B, C, h, w, generator=g).to(dev)
    v = torch.randn(B, Cv, h, w, generator=g).to(dev)
    ig = (torch.rand(B, h * w, generator=g) < 0.2) if use_ig else None
    # a support label map of two regions, so some cycles land on the other label
    sm = (torch.rand(B, h, w, generator=g) < 0.4).long() if use_cyc else None
    net = MatchNet(temp=20.0, cyc=use_cyc, device=dev).eval()
    init_match_params(net, 5)
    _, corr_plain = net(fq, fs, v, ret_corr=True)
    out = net(fq, fs, v, s_mask=sm.to(dev) if use_cyc else None, ig_mask=ig.to(dev) if use_ig else None,
              ret_corr=True, use_cyc=use_cyc, ret_cyc=use_cyc)
    wv, corr = out[0], out[1]
    c_ref, inc_ref = M.support_masks(corr_plain.reshape(B, h * w, h * w).double().cpu(),
                                     ig if use_ig else None, sm if use_cyc else None)
    if use_cyc:
        inc = out[2]
        assert tuple(inc.shape) == (B, 1, h * w)
        assert torch.equal(inc[:, 0].cpu().double(), inc_ref), "inconsistent mask"
        assert 0 < int(inc_ref.sum()) < B * h * w
    e_c = rel(corr.reshape(B, h * w, h * w), c_ref)
    attn = torch.softmax(c_ref * 20.0, dim=-1)
    wv_ref = torch.bmm(v.double().cpu().reshape(B, Cv, h * w), attn.transpose(1, 2)).reshape(B, Cv, h, w)
    e_v = rel(wv, wv_ref)
    print(f"MatchNet masks ig={use_ig} cyc={use_cyc}: corr2d {e_c:.2e} weighted_v {e_v:.2e}")
    assert e_c < 1e-6 and e_v < TOL


def test_forward_masks_errors(dev):
    from few_shot_seg_cwt_amd.match import MatchNet
    net = MatchNet(temp=20.0, cyc=True, device=dev)
    f = torch.rand(1, 8, 4, 4, device=dev)
    # training mode: Dropout(0.1) of the cycle mask (built since round 5): entries 0 or 1 / 0.9
    _, inc = net(f, f, f, s_mask=(torch.rand(1, 4, 4, device=dev) < 0.5).long(), use_cyc=True, ret_cyc=True)
    vals = set(round(float(x), 5) for x in inc.flatten().cpu())
    assert vals <= {0.0, round(1 / 0.9, 5)}, vals
    net.eval()
    with pytest.raises(ValueError):
        net(f, f, f, s_mask=None, use_cyc=True)
    with pytest.raises(UnboundLocalError):
        MatchNet(temp=20.0, device=dev).eval()(f, f, f, ret_cyc=True)


@pytest.mark.parametrize("L,h,w,sym", [(1, 6, 7, True), (2, 5, 5, True), (1, 7, 4, False)])
def test_corr_forward_cv4(dev, L, h, w, sym):
    """NeighConsensus over full Conv4d layers (conv='cv4', conv4d.py:64-138) through
    corr_forward, against the oracle's per-slice conv3d restatement in float64."""
    from few_shot_seg_cwt_amd.match import MatchNet, init_match_params
    from oracle import match_oracle as M
    net = MatchNet(temp=20.0, cv_type="cv4", in_channel=L, sym_mode=sym, device=dev)
    init_match_params(net, 13)
    sd = {k: t.detach().double().cpu() for k, t in net.state_dict().items()}
    assert tuple(sd["NeighConsensus.conv.0.weight"].shape) == (3, 10, L, 3, 3, 3)
    assert set(sd) == {f"NeighConsensus.conv.{i}.{n}" for i in (0, 2, 4) for n in ("weight", "bias")}
    B, Cv = 1, 24
    corr = _corr(dev, B, L, h, w, 17)
    g = torch.Generator().manual_seed(18)
    v = torch.randn(B, Cv, h, w, generator=g).to(dev)
    corr2d, wv = net.corr_forward(corr, v, ret_attn=True)
    rc, rwv = M.corr_forward(corr.double().cpu(), v.double().cpu(), M.layers_from_state(sd), 20.0, sym)
    e_c, e_v = rel(corr2d, rc), rel(wv, rwv)
    print(f"corr_forward cv4 L={L} {h}x{w} sym={sym}: corr2d {e_c:.2e} weighted_v {e_v:.2e}")
    assert e_c < TOL and e_v < TOL


@pytest.mark.parametrize("C,h,w,k", [(2048, 13, 11, 25), (64, 9, 8, 5)])
def test_spatial_context_encoder(dev, C, h, w, k):
    """SpatialContextEncoder (spatial_context.py:13-110) against the float64 oracle: the
    window descriptor, featureL2Norm, the concatenation and the 1x1 conv + ReLU."""
    from few_shot_seg_cwt_amd.match import SpatialContextEncoder, init_match_params
    from oracle import match_oracle as M
    hidden = 2048 if C == 2048 else 96
    enc = SpatialContextEncoder(kernel_size=k, input_dim=k * k + C, hidden_dim=hidden, device=dev)
    init_match_params(enc, 21)
    g = torch.Generator().manual_seed(22)
    x = torch.nn.functional.normalize(torch.rand(2, C, h, w, generator=g), dim=1)
    y = enc(x.to(dev))
    sd = {n: t.detach().double().cpu() for n, t in enc.state_dict().items()}
    assert set(sd) == {"embeddingFea.0.weight", "embeddingFea.0.bias"}
    ref = M.spatial_context_encoder(x.double(), k, sd["embeddingFea.0.weight"], sd["embeddingFea.0.bias"])
    e = rel(y, ref)
    print(f"SpatialContextEncoder C={C} {h}x{w} k={k}: {e:.2e}")
    assert e < 1e-5


def test_matchnet_forward_sce(dev):
    """MatchNet(sce=True).forward (match.py:95-97,108-113) against the oracle chain:
    normalize -> encoder -> get_corr -> run_match_model -> softmax readout."""
    from few_shot_seg_cwt_amd.match import MatchNet, init_match_params
    from oracle import match_oracle as M
    B, C, h, w, Cv = 1, 2048, 8, 9, 32
    net = MatchNet(temp=20.0, sce=True, device=dev).eval()
    init_match_params(net, 23)
    g = torch.Generator().manual_seed(24)
    fq, fs = torch.rand(B, C, h, w, generator=g), torch.rand(B, C, h, w, generator=g)
    v = torch.randn(B, Cv, h, w, generator=g)
    wv, corr = net(fq.to(dev), fs.to(dev), v.to(dev), ret_corr=True)
    sd = {n: t.detach().double().cpu() for n, t in net.state_dict().items()}
    W, b = sd["SpatialContextEncoder.embeddingFea.0.weight"], sd["SpatialContextEncoder.embeddingFea.0.bias"]
    eq = M.spatial_context_encoder(torch.nn.functional.normalize(fq.double(), dim=1), 25, W, b)
    es = M.spatial_context_encoder(torch.nn.functional.normalize(fs.double(), dim=1), 25, W, b)
    nq = torch.nn.functional.normalize(eq, dim=1).reshape(B, -1, h * w)
    ns = torch.nn.functional.normalize(es, dim=1).reshape(B, -1, h * w)
    corr0 = torch.bmm(nq.transpose(1, 2), ns).reshape(B, 1, h, w, h, w)
    rc, rwv = M.corr_forward(corr0, v.double(), M.layers_from_state(sd), 20.0, True)
    e_c, e_v = rel(corr.reshape(B, h * w, h * w), rc), rel(wv, rwv)
    print(f"MatchNet sce: corr2d {e_c:.2e} weighted_v {e_v:.2e}")
    # the encoder's ReLU features are nearly parallel (cosines near 1), so corr2d carries the
    # chain's fp32 rounding at ~1e-5 and the temp-20 softmax scales it by up to 20 in weighted_v
    # (measured 6.8e-6 / 2.8e-5); each stage alone is within 1e-5 (tests above)
    assert e_c < TOL and e_v < 5 * TOL


@pytest.mark.parametrize("agg,wa,red_dim", [("sum", True, False), ("cat", True, 512), ("sum", False, 256)])
def test_mmn_forward_agg_red_dim(dev, agg, wa, red_dim):
    """MMN with agg 'sum' (mmn.py:62-63) and red_dim (the rd_<layer> 1x1 conv + ReLU, mmn.py:
    28-31,49-51; the wa_ modules exist whenever red_dim does) against the oracle chain."""
    from few_shot_seg_cwt_amd.match import MMN, init_match_params
    from oracle import match_oracle as M
    args = dict(rmid="l34", layers=50, all_lr="l", temp=20.0, att_wt=0.2, conv4d="red")
    net = MMN(args, agg=agg, wa=wa, red_dim=red_dim, device=dev)
    init_match_params(net, seed=6)
    sd = {k: t.cpu() for k, t in net.state_dict().items()}
    if red_dim:
        assert tuple(sd["rd_3.0.weight"].shape) == (red_dim, 1024, 1, 1) and "wa_4.conv_theta.weight" in sd
    g = torch.Generator().manual_seed(25)
    h = 8
    fq_lst = {3: [torch.rand(1, 1024, h, h, generator=g).to(dev)], 4: [torch.rand(1, 2048, h, h, generator=g).to(dev)]}
    fs_lst = {3: [torch.rand(2, 1024, h, h, generator=g).to(dev)], 4: [torch.rand(2, 2048, h, h, generator=g).to(dev)]}
    f_q = torch.rand(1, 512, h, h, generator=g).to(dev)
    f_s = torch.rand(2, 512, h, h, generator=g).to(dev)
    fq, att_fq = net(fq_lst, fs_lst, f_q, f_s)
    wap = {b: M.wa_params_from_state(sd, f"wa_{b}.") for b in (3, 4)} if wa else None
    rdw = {b: sd[f"rd_{b}.0.weight"].double() for b in (3, 4)} if red_dim else None
    layers = M.layers_from_state(sd, prefix="corr_net.NeighConsensus.conv.")
    d = lambda t: t.double().cpu()  # noqa: E731
    fqo, atto = M.mmn_forward({k: d(v[0]) for k, v in fq_lst.items()}, {k: d(v[0]) for k, v in fs_lst.items()},
                              d(f_q), d(f_s), [3, 4], wap, layers, 20.0, 0.2, agg=agg, rd_weights=rdw)
    errs = dict(fq=rel(fq, fqo), att_fq=rel(att_fq, atto))
    print(f"MMN agg={agg} wa={wa} red_dim={red_dim}: {errs}")
    assert max(errs.values()) < TOL, errs

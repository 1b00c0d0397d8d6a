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


def test_mutual_matching(dev):
    from few_shot_seg_cwt_amd.match import MutualMatching
    from oracle import match_oracle as M
    g = torch.Generator().manual_seed(7)
    x = (torch.rand(2, 3, 5, 7, 6, 4, generator=g) * 2 - 1).to(dev)
    y = MutualMatching(x)
    e = rel(y, M.mutual_matching(x.double().cpu()))
    print(f"MutualMatching: {e:.2e}")
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

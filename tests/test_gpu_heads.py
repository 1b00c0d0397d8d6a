"""Variant heads on HIP (few_shot_seg_cwt_amd.heads: csrc/heads.hip) against the reference's
own CosCls / get_corr outputs (tests/golden/variants_small.npz, made by make_golden.py) and the
oracle at full size.  Bars: fp32 kernels, 1e-5 relative on outputs, 1e-4 on the parameter
gradients (fixed-order sums over the pixels in another order than the CPU's)."""
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from few_shot_seg_cwt_amd import synthetic as syn  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_oracle_golden import COS_TYPES, cos_params  # noqa: E402

SEED = 2021


def rel(a, b):
    a = a.detach().double().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a, np.float64)
    b = b.detach().double().cpu().numpy() if isinstance(b, torch.Tensor) else np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


@pytest.fixture(scope="module")
def gold(golden_dir):
    return dict(np.load(os.path.join(golden_dir, "variants_small.npz")))


@pytest.mark.parametrize("ct", COS_TYPES)
@pytest.mark.parametrize("n", [2, 16])
def test_cos_cls_vs_reference(dev, gold, ct, n):
    from few_shot_seg_cwt_amd.heads import CosCls
    tag = f"cos_{ct}_{n}"
    m = CosCls(512, n, ct)
    sd = dict(m.named_parameters())
    with torch.no_grad():
        for name, v in cos_params(ct, n).items():
            sd[name].copy_(v.to(dev).reshape(sd[name].shape))
    x = torch.from_numpy(syn.normal(SEED, "cosx", (2, 512, 5, 7), 1.0)).to(dev)
    y = m(x)
    assert tuple(y.shape) == (2, n, 5, 7)
    assert rel(y, gold[f"{tag}_out"]) < 1e-5
    G = torch.from_numpy(syn.normal(SEED, tag + "G", tuple(y.shape), 1.0)).to(dev)
    (y * G).sum().backward()
    for name, p in m.named_parameters():
        assert rel(p.grad, gold[f"{tag}_grad_{name}"]) < 1e-4, name
    if ct[1] == "n" and ct[0] != "r":   # weight_norm rewrote the stored weight, as the reference does
        assert rel(m.cls.weight, gold[f"{tag}_after_cls.weight"]) < 1e-6


def test_cos_cls_state_dict_keys_match_reference():
    from few_shot_seg_cwt_amd.heads import CosCls
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    assert sorted(CosCls(512, 2, "rnbt").state_dict()) == ["cls.bias", "cls.weight_g", "cls.weight_v", "scale_factor"]
    assert sorted(CosCls(512, 2, "0000").state_dict()) == ["cls.weight"]


def test_get_corr_vs_reference(dev, gold):
    from few_shot_seg_cwt_amd.heads import get_corr
    q = torch.from_numpy(syn.normal(SEED, "corrq", (2, 512, 5, 7), 1.0)).to(dev)
    k = torch.from_numpy(syn.normal(SEED, "corrk", (2, 512, 5, 7), 1.0)).to(dev)
    assert rel(get_corr(q, k), gold["corr_small"]) < 1e-5
    q = torch.from_numpy(syn.normal(SEED, "corrQ", (1, 512, 60, 60), 1.0)).abs().to(dev)
    k = torch.from_numpy(syn.normal(SEED, "corrK", (1, 512, 60, 60), 1.0)).abs().to(dev)
    sim = get_corr(q, k)
    assert tuple(sim.shape) == (1, 3600, 3600)
    assert rel(sim.reshape(-1)[::9973], gold["corr60_sample"]) < 1e-5
    np.testing.assert_allclose(np.array([sim.double().sum().item()]), gold["corr60_stat"][:1], rtol=1e-6)


@pytest.mark.parametrize("shape", [(1, 512, 81, 81, 81, 81), (3, 64, 9, 13, 7, 5)])
def test_get_corr_sizes_vs_oracle(dev, shape):
    """Ragged token counts (6561 = 81^2, partial 128-tiles, other C) against the oracle."""
    from few_shot_seg_cwt_amd.heads import get_corr
    from oracle import cwt_oracle as O
    B, C, h, w, hk, wk = shape
    q = torch.from_numpy(syn.normal(SEED, "cq" + str(shape), (B, C, h, w), 1.0))
    k = torch.from_numpy(syn.normal(SEED, "ck" + str(shape), (B, C, hk, wk), 1.0))
    ref = O.get_corr(q, k) if (h, w) == (hk, wk) else torch.bmm(
        torch.nn.functional.normalize(q.flatten(2).transpose(1, 2), dim=-1),
        torch.nn.functional.normalize(k.flatten(2), dim=-2))
    got = get_corr(q.to(dev), k.to(dev))
    assert rel(got, ref) < 1e-5

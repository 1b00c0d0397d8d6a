"""The bf16 conv stack (cwt_backbone_set_precision(CWT_CONV_BF16), BASELINE.json config #5:
"mixed-precision bf16 conv + fp32 CWT").  Its bar is not fp32 parity
but |delta mIoU| against the fp32 path over >= 100 synthetic episodes, reported, with the
CWT / classifier still fp32 on its inputs.  The mIoU here is on synthetic weights and
episodes (no pretrained weights or datasets exist offline), so it is a numerics check of the
bf16 path, not an accuracy claim."""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from few_shot_seg_cwt_amd import synthetic as syn  # noqa: E402

SEED = 2021
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


def _models(layers, sd):
    from few_shot_seg_cwt_amd import get_model
    m32 = get_model(syn.cfg_defaults(layers=layers)).load_state_dict(sd)
    m16 = get_model(syn.cfg_defaults(layers=layers, conv_dtype="bf16")).load_state_dict(sd)
    return m32, m16


def _transformer():
    from few_shot_seg_cwt_amd import MultiHeadAttentionOne
    t = MultiHeadAttentionOne(4, 512, 512, 512, dropout=0.5)
    t.load_state_dict(syn.make_transformer_state(4, 512, SEED))
    return t


@pytest.mark.parametrize("layers,S", [(50, 129), (101, 65)])
def test_bf16_features_close_to_fp32(dev, layers, S):
    sd = syn.make_pspnet_state(layers, SEED)
    m32, m16 = _models(layers, sd)
    ep = syn.make_episode(SEED, 11, S, 2)
    x = torch.from_numpy(np.concatenate([ep["spprt_imgs"][0], ep["qry_img"]])).to(dev)
    f32, _ = m32.extract_features(x)
    f16, _ = m16.extract_features(x)
    torch.cuda.synchronize()
    assert f16.dtype == torch.float32 and f16.shape == f32.shape
    err = float((f16 - f32).abs().max() / f32.abs().max())
    cos = float(torch.nn.functional.cosine_similarity(f16.flatten(1), f32.flatten(1)).min())
    print(f"R{layers}@{S}: bf16 vs fp32 features max rel {err:.3e}, min cosine {cos:.6f}")
    assert err < 0.1 and cos > 0.995
    # switching back restores the fp32 path exactly
    m16.set_conv_dtype("fp32")
    f16b, _ = m16.extract_features(x)
    assert torch.equal(f16b, f32)


def test_bf16_miou_delta_100_episodes(dev):
    """validate_transformer over 100 synthetic PASCAL 1-shot R50@473 episodes, fp32 vs bf16
    conv stack, identical W0 draws: |delta mIoU| reported (and written to
    gpurun_out/bf16_miou.json when that directory exists)."""
    from few_shot_seg_cwt_amd.episode import SyntheticEpisodes, validate_transformer
    n = 100
    sd = syn.make_pspnet_state(50, SEED)
    m32, m16 = _models(50, sd)
    t = _transformer()
    cfg = syn.cfg_defaults(test_num=n, n_runs=1)
    res = {}
    for name, m in (("fp32", m32), ("bf16", m16)):
        torch.manual_seed(SEED)
        miou, loss = validate_transformer(cfg, SyntheticEpisodes(n, start=500), m, t)
        res[name] = dict(mIoU=miou, loss=loss)
    d = abs(res["bf16"]["mIoU"] - res["fp32"]["mIoU"])
    res["abs_delta_mIoU"] = d
    res["episodes"] = n
    print(json.dumps(res))
    out = os.path.join(ROOT, "gpurun_out")
    if os.path.isdir(out):
        with open(os.path.join(out, "bf16_miou.json"), "w") as f:
            json.dump(res, f, indent=1)
    assert d < 0.02, res

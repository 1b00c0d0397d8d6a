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


def _argmax_up(pred, S):
    up = torch.nn.functional.interpolate(pred.float(), size=(S, S), mode="bilinear", align_corners=True)
    return up.argmax(1)


def _cached_loader(n, S, shot, start, classes):
    """SyntheticEpisodes with the n episodes built once, in parallel (a 641^2 5-shot episode
    takes ~1 s of host PRNG work), and replayed for both precisions."""
    from concurrent.futures import ThreadPoolExecutor
    from few_shot_seg_cwt_amd.episode import SyntheticEpisodes

    class Cached(SyntheticEpisodes):
        def __init__(self):
            super().__init__(n, S=S, shot=shot, start=start, classes=classes)
            with ThreadPoolExecutor(16) as ex:
                self.cache = list(ex.map(super().episode, range(n)))

        def episode(self, i):
            return self.cache[i]
    return Cached()


def _miou_run(layers, S, shot, n, start, classes=None):
    """validate_transformer over n synthetic episodes with the fp32 and the bf16 conv stack,
    identical W0 draws.  Returns the report: mIoU / loss per precision, |delta mIoU|, and the
    per-episode argmax flips of the upsampled mask (bf16 vs fp32, S x S pixels)."""
    from few_shot_seg_cwt_amd.episode import validate_transformer
    loader = _cached_loader(n, S, shot, start, classes)
    sd = syn.make_pspnet_state(layers, SEED)
    m32, m16 = _models(layers, sd)
    t = _transformer()
    cfg = syn.cfg_defaults(test_num=n, n_runs=1, layers=layers, image_size=S, shot=shot)
    res, outs = {}, {}
    for name, m in (("fp32", m32), ("bf16", m16)):
        torch.manual_seed(SEED)
        eps = []
        miou, loss = validate_transformer(cfg, loader, m, t, episodes_out=eps)
        res[name] = dict(mIoU=miou, loss=loss)
        outs[name] = eps
    flips = [int((_argmax_up(a["pred_q"], S) != _argmax_up(b["pred_q"], S)).sum())
             for a, b in zip(outs["fp32"], outs["bf16"])]
    res.update(abs_delta_mIoU=abs(res["bf16"]["mIoU"] - res["fp32"]["mIoU"]), episodes=n, layers=layers, S=S,
               shot=shot, flips_per_episode_mean=float(np.mean(flips)), flips_max=int(np.max(flips)),
               flip_fraction_mean=float(np.mean(flips)) / (S * S))
    print(json.dumps(res))
    out = os.path.join(ROOT, "gpurun_out")
    if os.path.isdir(out):
        with open(os.path.join(out, f"bf16_miou_r{layers}_{S}_{shot}shot.json"), "w") as f:
            json.dump(res, f, indent=1)
    return res


# Bars (|dmIoU| vs the fp32 path over >= 100 episodes, reported).  Measured on
# the MI355X (profiles/r2/bf16_miou_*.json): R50@473 1-shot |dmIoU| 7.5e-5; the bar is set a
# small multiple above the measurement so a precision regression in the bf16 stack fails it.
BF16_MIOU_BAR = 1e-3


def test_bf16_miou_delta_100_episodes(dev):
    """PASCAL 1-shot R50@473, 100 episodes: |delta mIoU| and argmax flips, bf16 vs fp32."""
    res = _miou_run(50, 473, 1, 100, 500)
    assert res["abs_delta_mIoU"] < BF16_MIOU_BAR, res


def test_bf16_config5_miou_delta_100_episodes(dev):
    """BASELINE config #5 as configured: COCO 5-shot R101@641, bf16 conv stack + fp32 CWT, 100
    episodes: |delta mIoU| and argmax flips against the fp32 stack on the same episodes."""
    res = _miou_run(101, 641, 5, 100, 500, syn.coco_val_classes(0))
    assert res["abs_delta_mIoU"] < BF16_MIOU_BAR, res


def test_bf16_config5_cwt_fp32_parity(dev):
    """Config #5's "fp32 CWT": on the bf16 stack's own inputs (its f_q and inner-loop W), the
    normalise + CWT + classifier must match the fp32 oracle to the fp32 kernel bar (1e-4)."""
    from few_shot_seg_cwt_amd.episode import EpisodeEngine
    from oracle import cwt_oracle as O
    sd = syn.make_pspnet_state(101, SEED)
    _, m16 = _models(101, sd)
    t = _transformer().eval()
    cfg = syn.cfg_defaults(layers=101, image_size=641, shot=5)
    ep = syn.make_episode(SEED, 3, 641, 5, syn.coco_val_classes(0))
    imgs = torch.from_numpy(np.concatenate([ep["spprt_imgs"][0], ep["qry_img"]])).to(dev)
    W0 = torch.from_numpy(syn.normal(SEED, "c5W0", (2, 512), 0.04)).to(dev)
    r = EpisodeEngine(m16, t, cfg).run(imgs, torch.from_numpy(ep["s_label"][0]).to(dev),
                                       torch.from_numpy(ep["q_label"]).to(dev), W0)
    torch.cuda.synchronize()
    tsd = O.to_torch_state(syn.make_transformer_state(4, 512, SEED))
    f_q = r["f_q"].detach().cpu().float().contiguous()
    W = r["W"].detach().cpu().reshape(1, 2, 512)
    fqn = O.normalize(f_q)
    W2 = O.cwt_forward(W, fqn, fqn, tsd, 4)
    pred_q = O.classify(W2, fqn)
    pred_q0 = torch.nn.functional.conv2d(f_q, W.reshape(2, 512, 1, 1))

    def rel(a, b):
        a, b = a.detach().double().cpu(), b.detach().double().cpu()
        return float((a - b).abs().max() / b.abs().max())
    errs = dict(W2=rel(r["W2"], W2), pred_q=rel(r["pred_q"], pred_q), pred_q0=rel(r["pred_q0"], pred_q0))
    print("config #5 fp32 CWT on bf16 inputs:", errs)
    assert max(errs.values()) < 1e-4, errs

"""HIP path (libcwt.so through the C ABI) vs the oracle and the reference's golden vectors.

Tolerances (BASELINE.json north_star): fp32 logits within 1e-3 relative
(max|d| / max|ref|), W and W' within 1e-3; argmax identical except on pixels whose
reference logit margin is below 1e-3 * max|logit| (IoU counts compared within the
count of such pixels)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from few_shot_seg_cwt_amd import synthetic as syn  # noqa: E402

SEED = 2021
TOL = 1e-3


def rel(a, b):
    a = a.detach().double().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a, np.float64)
    b = b.detach().double().cpu().numpy() if isinstance(b, torch.Tensor) else np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


_models = {}


def model(layers):
    from few_shot_seg_cwt_amd import get_model
    if layers not in _models:
        m = get_model(syn.cfg_defaults(layers=layers))
        m.load_state_dict(syn.make_pspnet_state(layers, SEED))
        _models[layers] = m
    return _models[layers]


def transformer(heads=4):
    from few_shot_seg_cwt_amd import MultiHeadAttentionOne
    t = MultiHeadAttentionOne(heads, 512, 512, 512, dropout=0.5)
    t.load_state_dict(syn.make_transformer_state(heads, 512, SEED))
    return t.eval()   # eval semantics: the oracle and the fixtures have no dropout


@pytest.fixture(scope="module")
def small(golden_dir):
    return dict(np.load(os.path.join(golden_dir, "modules_small.npz")))


# ---------------------------------------------------------------- feature extractor
@pytest.mark.parametrize("layers", [50, 101])
def test_extract_features_small_vs_reference(dev, small, layers):
    ep = syn.make_episode(SEED, 7, 33, 2)
    x = torch.from_numpy(ep["spprt_imgs"][0]).to(dev)
    f, lst = model(layers).extract_features(x)
    torch.cuda.synchronize()
    assert lst == [] and tuple(f.shape) == (2, 512, 5, 5)
    assert rel(f, small[f"feat_r{layers}_S33"]) < 1e-4


ARITH_X3S, ARITH_F32, ARITH_X6 = 0, 1, 2   # CWT_CONV_ARITH_*; the context default is X6


class conv_arith:
    """the default context's conv stack in another arithmetic for the duration
    (cwt_ctx_set_conv_arith): F32 = conv_igemm_f32d (the LDS-DMA body on v_mfma_f32_16x16x4_f32),
    X3S = the bf16x3 approximation over S-layout activations; restores the default (X6)"""

    def __init__(self, arith):
        self.arith = arith

    def __enter__(self):
        from few_shot_seg_cwt_amd import _lib
        _lib.check(_lib.lib().cwt_ctx_set_conv_arith(_lib.ctx(0), self.arith), "cwt_ctx_set_conv_arith")

    def __exit__(self, *exc):
        from few_shot_seg_cwt_amd import _lib
        _lib.check(_lib.lib().cwt_ctx_set_conv_arith(_lib.ctx(0), ARITH_X6), "cwt_ctx_set_conv_arith")
        return False


def exact_fp32():
    return conv_arith(ARITH_F32)


# x6 and f32: fp32-width products, fp32 sums in another order (the reference's own arithmetic,
# bar 1e-5); x3s: 16-bit operands (the declared approximation, bar 1e-3)
BAR = {ARITH_X6: 1e-5, ARITH_F32: 1e-5, ARITH_X3S: TOL}


@pytest.mark.parametrize("arith", [ARITH_X6, ARITH_X3S], ids=["x6", "x3s"])
def test_extract_features_full_vs_oracle(dev, arith):
    from oracle import cwt_oracle as O
    ep = syn.make_episode(SEED, 0, 473, 1)
    x = torch.from_numpy(ep["qry_img"])
    with conv_arith(arith):
        f, _ = model(50).extract_features(x.to(dev))
        torch.cuda.synchronize()
    ref = O.extract_features(x, O.to_torch_state(syn.make_pspnet_state(50, SEED)))
    err = rel(f, ref)
    print(f"extract_features 473 arith {arith}: {err:.3e}")
    assert err < BAR[arith]


@pytest.mark.parametrize("arith", [ARITH_X6, ARITH_F32], ids=["x6", "f32"])
@pytest.mark.parametrize("layers", [50, 101])
def test_extract_features_exact_fp32_small_vs_reference(dev, small, layers, arith):
    ep = syn.make_episode(SEED, 7, 33, 2)
    x = torch.from_numpy(ep["spprt_imgs"][0]).to(dev)
    with conv_arith(arith):
        f, _ = model(layers).extract_features(x)
        torch.cuda.synchronize()
    assert rel(f, small[f"feat_r{layers}_S33"]) < BAR[arith]


@pytest.mark.parametrize("arith", [ARITH_X6, ARITH_F32], ids=["x6", "f32"])
def test_extract_features_exact_fp32_full_vs_oracle(dev, arith):
    from oracle import cwt_oracle as O
    ep = syn.make_episode(SEED, 0, 473, 1)
    x = torch.from_numpy(np.concatenate([ep["spprt_imgs"][0], ep["qry_img"]]))
    with conv_arith(arith):
        f, _ = model(50).extract_features(x.to(dev))
        torch.cuda.synchronize()
    ref = O.extract_features(x, O.to_torch_state(syn.make_pspnet_state(50, SEED)))
    err = rel(f, ref)
    print(f"extract_features 473 x2 arith {arith}: {err:.3e}")
    assert err < BAR[arith]


def test_extract_batch_independent(dev):
    # batching support + query in one pass must equal separate passes (eval-mode BN)
    ep = syn.make_episode(SEED, 3, 129, 2)
    x = torch.from_numpy(np.concatenate([ep["spprt_imgs"][0], ep["qry_img"]])).to(dev)
    fa, _ = model(50).extract_features(x)
    fb, _ = model(50).extract_features(x[2:].contiguous())
    assert rel(fa[2:], fb) < 1e-5


# ---------------------------------------------------------------- inner loop
def test_inner_loop_small_vs_reference(dev, small):
    from few_shot_seg_cwt_amd.episode import inner_adapt
    ep = syn.make_episode(SEED, 7, 33, 2)
    f_s = torch.from_numpy(small["feat_r50_S33"]).to(dev).contiguous(memory_format=torch.channels_last)
    W = torch.from_numpy(small["inner_W0"]).reshape(2, 512).to(dev).contiguous()
    inner_adapt(f_s, torch.from_numpy(ep["s_label"][0]).to(dev), W, 0.1, 200)
    assert rel(W, small["inner_W200"].reshape(2, 512)) < TOL


@pytest.mark.parametrize("iters", [0, 1, 5])
def test_inner_loop_few_steps_vs_oracle(dev, iters):
    from few_shot_seg_cwt_amd.episode import inner_adapt
    from oracle import cwt_oracle as O
    ep = syn.make_episode(SEED, 11, 65, 1)
    f_s = torch.from_numpy(syn.normal(SEED, "fs", (1, 512, 9, 9), 0.1))
    W0 = torch.from_numpy(syn.normal(SEED, "w0", (2, 512), 0.05))
    ref = O.inner_adapt(f_s, torch.from_numpy(ep["s_label"][0]), W0.reshape(2, 512, 1, 1), 0.1, iters,
                        O.class_weight(ep["s_label"]))
    W = W0.clone().to(dev)
    inner_adapt(f_s.to(dev).contiguous(memory_format=torch.channels_last), torch.from_numpy(ep["s_label"][0]).to(dev),
                W, 0.1, iters)
    assert rel(W, ref.reshape(2, 512)) < 1e-4


# ---------------------------------------------------------------- CWT
@pytest.mark.parametrize("heads", [1, 4])
def test_cwt_forward_vs_reference(dev, small, heads):
    t = transformer(heads)
    k = torch.nn.functional.normalize(torch.from_numpy(small["feat_r50_S33"][:1]), dim=1).to(dev)
    q = torch.from_numpy(small[f"mha_h{heads}_q"]).to(dev)
    with torch.no_grad():
        out = t(q, k, k)
    assert rel(out, small[f"mha_h{heads}_out"]) < 1e-4


def test_cwt_forward_full_vs_oracle(dev):
    from oracle import cwt_oracle as O
    k = torch.nn.functional.normalize(torch.from_numpy(syn.normal(SEED, "fq", (1, 512, 60, 60))), dim=1)
    q = torch.from_numpy(syn.normal(SEED, "q", (1, 2, 512), 0.3))
    tsd = O.to_torch_state(syn.make_transformer_state(4, 512, SEED))
    ref = O.cwt_forward(q, k, k, tsd, 4)
    kd = k.to(dev)
    with torch.no_grad():
        out = transformer(4)(q.to(dev), kd, kd)
    assert rel(out, ref) < 1e-4


@pytest.mark.parametrize("heads", [1, 4])
def test_cwt_backward_vs_oracle_autograd(dev, heads):
    from oracle import cwt_oracle as O
    k = torch.nn.functional.normalize(torch.from_numpy(syn.normal(SEED, "fk", (1, 512, 7, 9))), dim=1)
    q = torch.from_numpy(syn.normal(SEED, "qb", (1, 2, 512), 0.3))
    gout = torch.from_numpy(syn.normal(SEED, "go", (1, 2, 512), 1.0))
    tsd = {n: v.clone().requires_grad_(True) for n, v in
           O.to_torch_state(syn.make_transformer_state(heads, 512, SEED)).items()}
    ref_out = O.cwt_forward(q, k, k, tsd, heads)
    ref_g = torch.autograd.grad(ref_out, list(tsd.values()), gout)
    t = transformer(heads)
    kd = k.to(dev)
    out = t(q.to(dev), kd, kd)
    out.backward(gout.to(dev))
    g = t.flat.grad
    for (n, _), rg in zip(t.named_views(), ref_g):
        assert rel(t.view(n, g), rg) < 1e-4, n


# ---------------------------------------------------------------- metrics
def test_seg_metrics_vs_oracle(dev):
    from few_shot_seg_cwt_amd.util import seg_metrics
    from oracle import cwt_oracle as O
    logits = torch.from_numpy(syn.normal(SEED, "lg", (2, 2, 60, 60), 1.0))
    ep = syn.make_episode(SEED, 5, 473, 2)
    tgt = torch.from_numpy(ep["s_label"][0])
    iut, ce = seg_metrics(logits.to(dev), tgt.to(dev))
    up = O.upsample(logits, 473)
    for b in range(2):
        i, u, t = O.intersection_union(up.argmax(1)[b], tgt[b])
        np.testing.assert_array_equal(iut[b].cpu().numpy(), np.stack([i.numpy(), u.numpy(), t.numpy()]))
        l = torch.nn.functional.cross_entropy(up[b:b + 1], tgt[b:b + 1], ignore_index=255).item()
        c = ce[b].cpu().numpy()
        assert abs(c[0] / c[1] - l) < 1e-4 * abs(l)


def test_seg_metrics_pair_equals_two_calls(dev):
    """The fused pred_q / pred_q0 scoring (cwt_seg_metrics_pair) against two single calls:
    integer counts and the fixed-order double CE sum, bit for bit."""
    from few_shot_seg_cwt_amd.util import seg_metrics, seg_metrics_pair
    lg = torch.from_numpy(syn.normal(SEED, "lg", (2, 2, 60, 60), 1.0)).to(dev)
    lg0 = torch.from_numpy(syn.normal(SEED, "lg0", (2, 2, 60, 60), 1.0)).to(dev)
    tgt = torch.from_numpy(syn.make_episode(SEED, 5, 473, 2)["s_label"][0]).to(dev)
    iut, ce, iut0 = seg_metrics_pair(lg, lg0, tgt)
    r_iut, r_ce = seg_metrics(lg, tgt)
    r_iut0, _ = seg_metrics(lg0, tgt, with_ce=False)
    assert torch.equal(iut, r_iut) and torch.equal(ce, r_ce) and torch.equal(iut0, r_iut0)
    assert not torch.equal(iut, iut0)   # the two tensors really are scored separately


def test_iou_preds_vs_reference(dev, small):
    from few_shot_seg_cwt_amd.util import intersectionAndUnionGPU
    i, u, t = intersectionAndUnionGPU(torch.from_numpy(small["iou_preds"]).to(dev),
                                      torch.from_numpy(small["iou_target"]).to(dev), 2, 255)
    np.testing.assert_array_equal(torch.stack([i, u, t]).cpu().numpy(), small["iou_out"])


def test_sgd_nesterov_vs_torch(dev):
    from few_shot_seg_cwt_amd.optimizer import HipSGD
    p0 = torch.from_numpy(syn.normal(SEED, "p", (1000,), 1.0))
    grads = [torch.from_numpy(syn.normal(SEED, f"g{i}", (1000,), 1.0)) for i in range(3)]
    pr = p0.clone().requires_grad_(True)
    opt_r = torch.optim.SGD([pr], lr=0.01, momentum=0.9, weight_decay=1e-4, nesterov=True)
    pd = torch.nn.Parameter(p0.clone().to(dev))
    opt = HipSGD([pd], lr=0.01, momentum=0.9, weight_decay=1e-4, nesterov=True)
    for g in grads:
        pr.grad = g.clone()
        opt_r.step()
        pd.grad = g.clone().to(dev)
        opt.step()
    assert rel(pd.data, pr.detach()) < 1e-6


# ---------------------------------------------------------------- full episodes vs golden
def _low_margin(pred_ref, S):
    up = torch.nn.functional.interpolate(torch.from_numpy(pred_ref)[None], size=(S, S), mode="bilinear",
                                         align_corners=True)[0]
    m = (up[1] - up[0]).abs()
    return int((m < 1e-3 * up.abs().max()).sum())


def flip_report(pred, pred_ref, S, tag=""):
    """Argmax flips of the upsampled S x S mask (test.py:214-219) between our logits and the
    reference's [2,h,w]: (all flips, flips on pixels whose reference margin exceeds
    1e-3 * max|logit|).  The second must be 0; the first is reported.  Appended
    to gpurun_out/flips.jsonl when that directory exists."""
    up = lambda x: torch.nn.functional.interpolate(torch.as_tensor(np.asarray(x, np.float32))[None], size=(S, S),
                                                   mode="bilinear", align_corners=True)[0]
    a, b = up(pred.detach().cpu().numpy() if isinstance(pred, torch.Tensor) else pred), up(pred_ref)
    diff = a.argmax(0) != b.argmax(0)
    margin = (b[1] - b[0]).abs()
    big = margin >= 1e-3 * b.abs().max()
    rep = {"test": tag, "S": S, "flips": int(diff.sum()), "flips_above_margin": int((diff & big).sum()),
           "low_margin_pixels": int((~big).sum())}
    print("argmax flips:", rep)
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    if os.path.isdir(out):
        import json
        with open(os.path.join(out, "flips.jsonl"), "a") as f:
            f.write(json.dumps(rep) + "\n")
    return rep["flips"], rep["flips_above_margin"]


@pytest.mark.parametrize("name,layers,S,shot,n_ep", [
    ("episode_pascal_r50_1shot.npz", 50, 473, 1, 3),
    ("episode_pascal_r50_5shot.npz", 50, 473, 5, 1),
    ("episode_coco_r101_1shot.npz", 101, 641, 1, 1),
    ("episode_coco_r101_5shot.npz", 101, 641, 5, 1),     # BASELINE config #5's shapes, fp32 stack
])
def test_episode_vs_reference(dev, golden_dir, name, layers, S, shot, n_ep):
    from few_shot_seg_cwt_amd.episode import EpisodeEngine
    g = dict(np.load(os.path.join(golden_dir, name)))
    cfg = syn.cfg_defaults(layers=layers, image_size=S, shot=shot)
    eng = EpisodeEngine(model(layers), transformer(4), cfg)
    classes = syn.coco_val_classes(0) if layers == 101 else None
    for e in range(n_ep):
        ep = syn.make_episode(SEED, e, S, shot, classes)
        imgs = torch.from_numpy(np.concatenate([ep["spprt_imgs"][0], ep["qry_img"]])).to(dev)
        W0 = torch.from_numpy(g[f"e{e}_W0"]).to(dev).contiguous()
        r = eng.run(imgs, torch.from_numpy(ep["s_label"][0]).to(dev), torch.from_numpy(ep["q_label"]).to(dev), W0)
        torch.cuda.synchronize()
        assert rel(r["W"], g[f"e{e}_W"]) < TOL
        assert rel(r["W2"][0], g[f"e{e}_W2"]) < TOL
        assert rel(r["pred_q"][0], g[f"e{e}_pred_q"]) < TOL
        assert rel(r["pred_q0"][0], g[f"e{e}_pred_q0"]) < TOL
        low = _low_margin(g[f"e{e}_pred_q"], S)
        iu = r["iut"][0].cpu().numpy()
        assert np.abs(iu - g[f"e{e}_iu"]).max() <= low, (iu, g[f"e{e}_iu"], low)
        for key in ("pred_q", "pred_q0"):
            _, hard = flip_report(r[key][0], g[f"e{e}_{key}"], S, f"{name}:e{e}:{key}")
            assert hard == 0


@pytest.mark.parametrize("arith", [ARITH_F32, ARITH_X3S], ids=["f32", "x3s"])
@pytest.mark.parametrize("name,layers,S,shot", [
    ("episode_pascal_r50_1shot.npz", 50, 473, 1),
    ("episode_coco_r101_1shot.npz", 101, 641, 1),
])
def test_episode_exact_fp32_vs_reference(dev, golden_dir, name, layers, S, shot, arith):
    """The conv stack's other arithmetics (bench.py's exact_fp32 and bf16x3 legs; the default x6
    runs in test_episode_vs_reference) against the reference's episode fixture: W, W', logits
    and IoU counts; no argmax flip above the margin."""
    from few_shot_seg_cwt_amd.episode import EpisodeEngine
    g = dict(np.load(os.path.join(golden_dir, name)))
    cfg = syn.cfg_defaults(layers=layers, image_size=S, shot=shot)
    eng = EpisodeEngine(model(layers), transformer(4), cfg)
    classes = syn.coco_val_classes(0) if layers == 101 else None
    ep = syn.make_episode(SEED, 0, S, shot, classes)
    imgs = torch.from_numpy(np.concatenate([ep["spprt_imgs"][0], ep["qry_img"]])).to(dev)
    W0 = torch.from_numpy(g["e0_W0"]).to(dev).contiguous()
    with conv_arith(arith):
        r = eng.run(imgs, torch.from_numpy(ep["s_label"][0]).to(dev), torch.from_numpy(ep["q_label"]).to(dev), W0)
        torch.cuda.synchronize()
    assert rel(r["W"], g["e0_W"]) < TOL
    assert rel(r["W2"][0], g["e0_W2"]) < TOL
    assert rel(r["pred_q"][0], g["e0_pred_q"]) < TOL
    low = _low_margin(g["e0_pred_q"], S)
    iu = r["iut"][0].cpu().numpy()
    assert np.abs(iu - g["e0_iu"]).max() <= low
    _, hard = flip_report(r["pred_q"][0], g["e0_pred_q"], S, f"{name}:arith{arith}")
    assert hard == 0


def _check_episode_outputs(r, g, e, S, tag):
    """One episode of the product path (validate_transformer's episodes_out: the pipelined, fused
    loop + tail on the adapt context, or the drain's whole-chip loop for a run's last episode)
    against the reference's fixture: W, W', pred_q, pred_q0 (1e-3), IoU counts of both logits
    within the low-margin pixel count, no argmax flip above the margin (test.py:164-219)."""
    errs = dict(W=rel(r["W"], g[f"e{e}_W"]), W2=rel(r["W2"][0], g[f"e{e}_W2"]),
                pred_q=rel(r["pred_q"][0], g[f"e{e}_pred_q"]), pred_q0=rel(r["pred_q0"][0], g[f"e{e}_pred_q0"]))
    print(f"{tag} e{e}: " + ", ".join(f"{k} {v:.1e}" for k, v in errs.items()))
    assert max(errs.values()) < TOL, errs
    for key, iu_key in (("pred_q", "iut"), ("pred_q0", "iut0")):
        low = _low_margin(g[f"e{e}_{key}"], S)
        iu = r[iu_key][0].numpy()
        ref = g[f"e{e}_iu" if key == "pred_q" else f"e{e}_iu0"]
        assert np.abs(iu - ref).max() <= low, (key, iu, ref, low)
        _, hard = flip_report(r[key][0], g[f"e{e}_{key}"], S, f"{tag}:e{e}:{key}")
        assert hard == 0


def test_validate_transformer_vs_reference(dev, golden_dir):
    """validate_transformer (test.py:103-254) through the episode pipeline, against the
    reference's own run: run-level mIoU and loss, and per episode the product path's W, W',
    pred_q, pred_q0 and IoU counts.  Episodes 0 and 1 run the fused loop + tail on the pipeline's
    adapt context, episode 2 (the run's last) the drain's whole-chip loop."""
    from few_shot_seg_cwt_amd import _lib
    from few_shot_seg_cwt_amd.episode import EpisodeEngine, EpisodePipeline, SyntheticEpisodes, validate_transformer
    import ctypes
    g = dict(np.load(os.path.join(golden_dir, "episode_pascal_r50_1shot.npz")))
    cfg = syn.cfg_defaults(test_num=3, n_runs=1)
    torch.manual_seed(SEED)
    eps = []
    m, t = model(50), transformer(4)
    miou, loss = validate_transformer(cfg, SyntheticEpisodes(3), m, t, episodes_out=eps)
    assert abs(miou - float(g["mIoU"])) < 2e-3
    assert abs(loss - float(g["loss"])) < 1e-3 * abs(float(g["loss"]))
    pipe = EpisodePipeline.shared(EpisodeEngine(m, t, cfg), extract_streams=2)
    fz = ctypes.c_int(0)
    _lib.check(_lib.lib().cwt_adapt_fuses_tail(pipe.c_adapt, 1, 60, 60, 200, ctypes.byref(fz)), "cwt_adapt_fuses_tail")
    assert fz.value == 1   # the product path under test is the fused one
    for e in range(3):   # W0 drawn from the torch RNG exactly as the reference draws it
        _check_episode_outputs(eps[e], g, e, 473, "validate_transformer pascal 1-shot")


@pytest.mark.parametrize("name,layers,S,shot", [
    ("episode_pascal_r50_5shot.npz", 50, 473, 5),
    ("episode_coco_r101_1shot.npz", 101, 641, 1),
])
def test_validate_transformer_pipelined_vs_reference(dev, golden_dir, name, layers, S, shot):
    """BASELINE configs #3 / #4's shapes through validate_transformer's pipeline: the fixture holds
    one episode (the reference's run of test_num 1), so the run here has two and episode 0 -- the
    one with the fixture's W0, the first torch draw after manual_seed -- runs on the pipeline's adapt
    context (not the drain): its W, W', pred_q, pred_q0 and IoU counts against the fixture."""
    from few_shot_seg_cwt_amd.episode import SyntheticEpisodes, validate_transformer
    g = dict(np.load(os.path.join(golden_dir, name)))
    cfg = syn.cfg_defaults(layers=layers, image_size=S, shot=shot, test_num=2, n_runs=1)
    classes = syn.coco_val_classes(0) if layers == 101 else None
    torch.manual_seed(SEED)
    eps = []
    validate_transformer(cfg, SyntheticEpisodes(2, S=S, shot=shot, classes=classes), model(layers), transformer(4),
                         episodes_out=eps)
    assert len(eps) == 2
    _check_episode_outputs(eps[0], g, 0, S, f"validate_transformer {name}")


@pytest.mark.parametrize("name", ["train_pascal_r50_1shot.npz", "train_coco_r101_1shot.npz"])
def test_do_epoch_vs_reference(dev, golden_dir, name):
    """do_epoch (train.py:166-288) against the reference's own run, dropout off and BN eval:
    PASCAL R50@473 and BASELINE config #4's COCO 1-shot R101@641.  Losses, W, W', pred_q0,
    the CWT gradients of the first step and the parameters after both SGD steps."""
    from few_shot_seg_cwt_amd.episode import SyntheticEpisodes, do_epoch
    from few_shot_seg_cwt_amd.optimizer import get_optimizer
    g = dict(np.load(os.path.join(golden_dir, name)))
    layers, S = int(g.get("layers", 50)), int(g.get("S", 473))
    classes = syn.coco_val_classes(0) if layers == 101 else None
    cfg = syn.cfg_defaults(layers=layers, image_size=S)
    t = transformer(4)
    t.attention.dropout.p = 0.0   # dropout off, as make_golden.py does on the reference module
    t.dropout.p = 0.0
    opt = get_optimizer(cfg, [dict(params=[t.flat], lr=cfg["trans_lr"] * cfg["scale_lr"])])
    torch.manual_seed(SEED)
    recs = []
    m = model(layers)
    m.bn_train_mode = False   # the fixture excludes the first-episode BN quirk (test_gpu_bn_train.py has it)
    try:
        ious, losses = do_epoch(cfg, SyntheticEpisodes(2, S=S, start=int(g["start"]), classes=classes), m, t, opt,
                                epoch=1, iter_per_epoch=2, log_iter=2, records=recs)
    finally:
        m.bn_train_mode = True
    np.testing.assert_allclose(losses.numpy(), g["train_losses"], rtol=TOL)
    for e in range(2):
        assert rel(recs[e]["W"], g[f"e{e}_W"]) < TOL
        assert rel(recs[e]["W2"][0], g[f"e{e}_W2"]) < TOL
        if f"e{e}_pred_q0" in g:
            assert rel(recs[e]["pred_q0"][0], g[f"e{e}_pred_q0"]) < TOL
            _, hard = flip_report(recs[e]["pred_q0"][0], g[f"e{e}_pred_q0"], S, f"{name}:e{e}:pred_q0")
            assert hard == 0
    # LayerNorm/fc-bias gradients are sums over the two query rows whose d_out cancel exactly
    # (dW'[0] = -dW'[1]), i.e. pure rounding noise: their error is scaled by the whole gradient.
    gmax = max(float(np.abs(g[f"e0_grad_{n}_sample"]).max()) for n, _ in t.named_views())
    errs = {}
    for n, v in t.named_views():
        gv = t.view(n, recs[0]["grad"]).reshape(-1)[::101].double().numpy()
        ref = g[f"e0_grad_{n}_sample"].astype(np.float64)
        errs[n] = np.abs(gv - ref).max() / max(np.abs(ref).max(), 1e-3 * gmax)
        assert rel(v.reshape(-1)[::101], g[f"final_{n}_sample"]) < 1e-4, n
    print("gradient errors (relative, bar 1e-3):", errs)
    assert max(errs.values()) < TOL, errs

"""Episodes in flight (cwt_inner_adapt_batch, EpisodeEngine.run_batch): E independent
episodes sharing the backbone pass and the inner loop's step launches give each episode the
result it gets alone.  Only the fp32 rounding of the inner loop's per-workgroup partial sums
differs between the two runs (their workgroup geometries differ), so the bar is 1e-5 relative, and IoU counts may differ only on pixels whose
logit margin is at that rounding level."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from few_shot_seg_cwt_amd import synthetic as syn  # noqa: E402

SEED = 2021
TOL = 1e-5
TOL_RUN = 5e-5


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


@pytest.mark.parametrize("E,n,S,iters", [(3, 2, 65, 20), (2, 1, 129, 200), (4, 1, 33, 5), (8, 1, 65, 20)])
def test_inner_adapt_batch_equals_single(dev, E, n, S, iters):
    from few_shot_seg_cwt_amd.episode import inner_adapt, inner_adapt_batch
    h = (S - 1) // 8 + 1
    f = torch.from_numpy(syn.normal(5, f"fb{E}{n}{S}", (E * n, 512, h, h), 0.5)).abs().to(dev)
    f = f.contiguous(memory_format=torch.channels_last)
    lbl = torch.stack([torch.from_numpy(syn.make_episode(SEED, 40 + e, S, n)["s_label"][0]) for e in range(E)]).to(dev)
    W0 = torch.from_numpy(syn.normal(6, f"wb{E}{n}{S}", (E, 2, 512), 0.04)).to(dev)
    Wb = inner_adapt_batch(f, lbl, W0.clone(), 0.1, iters)
    for e in range(E):
        We = inner_adapt(f[e * n:(e + 1) * n], lbl[e], W0[e].clone(), 0.1, iters)
        assert rel(Wb[e], We) < TOL, e


@pytest.mark.parametrize("E", [3, 6])
def test_run_batch_equals_run(dev, E):
    from few_shot_seg_cwt_amd import MultiHeadAttentionOne, get_model
    from few_shot_seg_cwt_amd.episode import EpisodeEngine
    S, shot = 129, 1
    cfg = syn.cfg_defaults(image_size=S)
    m = get_model(cfg).load_state_dict(syn.make_pspnet_state(50, SEED))
    t = MultiHeadAttentionOne(4, 512, 512, 512, dropout=0.5)
    t.load_state_dict(syn.make_transformer_state(4, 512, SEED))
    eng = EpisodeEngine(m, t, cfg)
    eps = [syn.make_episode(SEED, 60 + e, S, shot) for e in range(E)]
    W0 = torch.from_numpy(syn.normal(7, "wrb", (E, 2, 512), 0.04)).to(dev)
    imgs = torch.from_numpy(np.concatenate([ep["spprt_imgs"][0] for ep in eps] + [ep["qry_img"] for ep in eps])).to(dev)
    sl = torch.from_numpy(np.stack([ep["s_label"][0] for ep in eps])).to(dev)
    ql = torch.from_numpy(np.concatenate([ep["q_label"] for ep in eps])).to(dev)
    rb = eng.run_batch(imgs, sl, ql, W0.clone())
    for e, ep in enumerate(eps):
        x = torch.from_numpy(np.concatenate([ep["spprt_imgs"][0], ep["qry_img"]])).to(dev)
        r = eng.run(x, sl[e], ql[e:e + 1], W0[e].clone())
        # the batched pass picks its conv plans (split-K) for its own M: features round
        # differently at the 1e-7 level, which 200 SGD steps lift to ~1e-5
        assert rel(rb["W"][e], r["W"]) < TOL_RUN
        assert rel(rb["W2"][e], r["W2"][0]) < TOL_RUN
        assert rel(rb["pred_q"][e], r["pred_q"][0]) < TOL_RUN
        assert rel(rb["pred_q0"][e], r["pred_q0"][0]) < TOL_RUN
        assert float((rb["iut"][e] - r["iut"][0]).abs().max()) <= 2


@pytest.mark.parametrize("streams,overlap", [(1, True), (2, True), (2, False)])
def test_pipeline_equals_run(dev, streams, overlap):
    """EpisodePipeline (extractor of episode i+1 on one stream beside episode i's inner loop and
    CWT on another) gives every episode what EpisodeEngine.run gives it alone -- the burst's last
    episode through the drain (its loop on the whole-chip context; overlap: on a stream of its own
    beside the previous episode's loop and tail)."""
    from few_shot_seg_cwt_amd import MultiHeadAttentionOne, get_model
    from few_shot_seg_cwt_amd.episode import EpisodeEngine, EpisodePipeline
    S, shot, n = 129, 1, 4
    cfg = syn.cfg_defaults(image_size=S)
    m = get_model(cfg).load_state_dict(syn.make_pspnet_state(50, SEED))
    t = MultiHeadAttentionOne(4, 512, 512, 512, dropout=0.5)
    t.load_state_dict(syn.make_transformer_state(4, 512, SEED))
    eng = EpisodeEngine(m, t, cfg)
    pipe = EpisodePipeline(eng, extract_streams=streams)
    pipe.drain_overlap = overlap
    eps = [syn.make_episode(SEED, 80 + e, S, shot) for e in range(n)]
    W0 = torch.from_numpy(syn.normal(8, "wpl", (n, 2, 512), 0.04)).to(dev)
    ins = []
    for ep in eps:
        imgs = torch.from_numpy(np.concatenate([ep["spprt_imgs"][0], ep["qry_img"]])).to(dev)
        ins.append((imgs, torch.from_numpy(ep["s_label"][0]).to(dev), torch.from_numpy(ep["q_label"]).to(dev)))
    outs = [pipe.submit(i, s, q, W0[e].clone(), last=e == n - 1) for e, (i, s, q) in enumerate(ins)]
    pipe.wait()
    torch.cuda.synchronize()
    if overlap:
        assert pipe.s_drain is not None   # the 17x17 grids fit beside each other
    for e, (i, s, q) in enumerate(ins):
        r = eng.run(i, s, q, W0[e].clone())
        torch.cuda.synchronize()
        assert rel(outs[e]["W"], r["W"]) < TOL, e
        assert rel(outs[e]["pred_q"], r["pred_q"]) < TOL_RUN, e
        assert torch.equal(outs[e]["iut0"], r["iut0"]), e
    pipe.close()


@pytest.mark.gpu
def test_pipeline_batch_equals_run(dev):
    """EpisodePipeline.submit_batch (two episodes sharing one extractor pass, their inner loops in
    one persistent launch, the tails batched) gives every episode what EpisodeEngine.run gives it
    alone, pair after pair through the pipeline's streams."""
    from few_shot_seg_cwt_amd import MultiHeadAttentionOne, get_model
    from few_shot_seg_cwt_amd.episode import EpisodeEngine, EpisodePipeline
    S, shot, n, E = 129, 1, 4, 2
    cfg = syn.cfg_defaults(image_size=S)
    m = get_model(cfg).load_state_dict(syn.make_pspnet_state(50, SEED))
    t = MultiHeadAttentionOne(4, 512, 512, 512, dropout=0.5)
    t.load_state_dict(syn.make_transformer_state(4, 512, SEED))
    eng = EpisodeEngine(m, t, cfg)
    pipe = EpisodePipeline(eng, extract_streams=2)
    eps = [syn.make_episode(SEED, 90 + e, S, shot) for e in range(n)]
    W0 = torch.from_numpy(syn.normal(9, "wpb", (n, 2, 512), 0.04)).to(dev)
    outs = []
    for b in range(0, n, E):
        grp = eps[b:b + E]
        imgs = torch.from_numpy(np.concatenate([ep["spprt_imgs"][0] for ep in grp] + [ep["qry_img"] for ep in grp]))
        sl = torch.from_numpy(np.stack([ep["s_label"][0] for ep in grp]))
        ql = torch.from_numpy(np.concatenate([ep["q_label"] for ep in grp]))
        outs.append(pipe.submit_batch(imgs.to(dev), sl.to(dev), ql.to(dev), W0[b:b + E].clone(), last=b + E >= n))
    pipe.wait()
    torch.cuda.synchronize()
    for e, ep in enumerate(eps):
        o = outs[e // E]
        j = e % E
        imgs = torch.from_numpy(np.concatenate([ep["spprt_imgs"][0], ep["qry_img"]])).to(dev)
        r = eng.run(imgs, torch.from_numpy(ep["s_label"][0]).to(dev), torch.from_numpy(ep["q_label"]).to(dev),
                    W0[e].clone())
        torch.cuda.synchronize()
        # the shared pass picks its conv plans for its own M (as run_batch): ~1e-5 after 200 steps
        assert rel(o["W"][j], r["W"]) < TOL_RUN, e
        assert rel(o["W2"][j], r["W2"][0]) < TOL_RUN, e
        assert rel(o["pred_q"][j], r["pred_q"][0]) < TOL_RUN, e
        assert float((o["iut"][j] - r["iut"][0]).abs().max()) <= 2, e
    pipe.close()


def test_validate_transformer_reuses_its_pipeline(dev):
    """validate_transformer runs every epoch: its EpisodePipeline (and the libcwt contexts it
    holds) is created once per device and reused, so repeated calls do not pile up contexts."""
    from few_shot_seg_cwt_amd import MultiHeadAttentionOne, _lib, get_model
    from few_shot_seg_cwt_amd.episode import EpisodePipeline, SyntheticEpisodes, validate_transformer
    S = 65
    cfg = syn.cfg_defaults(image_size=S)
    cfg.update(test_num=2, n_runs=1, pipeline=2, adapt_iter=5)
    m = get_model(cfg).load_state_dict(syn.make_pspnet_state(50, SEED))
    t = MultiHeadAttentionOne(4, 512, 512, 512, dropout=0.5)
    t.load_state_dict(syn.make_transformer_state(4, 512, SEED))
    torch.manual_seed(0)
    a = validate_transformer(cfg, SyntheticEpisodes(2, S), m, t)
    n_ctx = len(_lib.all_ctx())
    torch.manual_seed(0)
    b = validate_transformer(cfg, SyntheticEpisodes(2, S), m, t)
    assert len(_lib.all_ctx()) == n_ctx
    assert abs(a[0] - b[0]) < 1e-2 and abs(a[1] - b[1]) < 1e-3 * max(1.0, abs(a[1]))
    pipe = EpisodePipeline._shared[(torch.cuda.current_device(), 2)]
    owned = 2 + (pipe.c_solo is not None)
    pipe.close()
    assert len(_lib.all_ctx()) == n_ctx - owned   # its second extractor context, the adapt context(s)

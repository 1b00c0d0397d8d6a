"""The fused inference tail (test.py:190-204): cwt_attention_infer (F.normalize fused into the single
token pass, baseline logits W . f_q in the same pass, the CWT with its projections folded per head)
+ cwt_classify_scaled, against the module-by-module kernels it replaces (cwt_normalize,
cwt_attention_fwd, cwt_classify) and against the oracle (oracle/cwt_oracle.py, pinned by the
reference's fixtures).  The fused form is the same function re-associated, so the bar is fp32
rounding: 1e-5 relative.  Also: the folded weights follow every parameter change (load_state_dict,
the optimiser's step) -- a stale fold would be a silent error."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from few_shot_seg_cwt_amd import synthetic as syn  # noqa: E402

SEED = 2021
TOL = 1e-5


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


def _inputs(dev, B, h, tag):
    f = torch.from_numpy(syn.normal(3, "tf" + tag, (B, 512, h, h), 1.0)).abs().to(dev)
    f = f.contiguous(memory_format=torch.channels_last)
    W = torch.from_numpy(syn.normal(4, "tw" + tag, (B, 2, 512), 0.05)).to(dev)
    return f, W


def _modules(t, W, f):
    from few_shot_seg_cwt_amd.episode import classify, normalize
    fqn, pred_q0 = normalize(f, W)
    W2 = t.infer(W, fqn)
    return W2, classify(W2, fqn), pred_q0, fqn


@pytest.mark.parametrize("B,h", [(1, 60), (1, 81), (2, 60), (4, 33), (3, 9), (1, 2)])
def test_fused_tail_equals_modules(dev, B, h):
    from few_shot_seg_cwt_amd import MultiHeadAttentionOne
    from few_shot_seg_cwt_amd.episode import cwt_tail
    t = MultiHeadAttentionOne(4, 512, 512, 512, dropout=0.5)
    t.load_state_dict(syn.make_transformer_state(4, 512, SEED))
    t.eval()
    f, W = _inputs(dev, B, h, f"{B}_{h}")
    W2, pq, pq0 = cwt_tail(t, W, f)
    W2r, pqr, pq0r, fqn = _modules(t, W, f)
    _, inv, _ = t.infer_raw(W, f, with_logits0=False)
    torch.cuda.synchronize()
    fn_fused = f.permute(0, 2, 3, 1).reshape(B, h * h, 512) * inv[..., None]
    errs = dict(W2=rel(W2, W2r), pred_q=rel(pq, pqr), pred_q0=rel(pq0, pq0r),
                f_hat=rel(fn_fused, fqn.permute(0, 2, 3, 1).reshape(B, h * h, 512)))
    print(f"fused tail B={B} h={h}: {errs}")
    assert max(errs.values()) < TOL, errs


def test_fused_tail_vs_oracle(dev):
    """One 473-shaped tail against the oracle's normalize / cwt_forward / classify (float64)."""
    from few_shot_seg_cwt_amd import MultiHeadAttentionOne
    from few_shot_seg_cwt_amd.episode import cwt_tail
    from oracle import cwt_oracle as O
    tsd = syn.make_transformer_state(4, 512, SEED)
    t = MultiHeadAttentionOne(4, 512, 512, 512, dropout=0.5)
    t.load_state_dict(tsd)
    f, W = _inputs(dev, 1, 60, "or")
    W2, pq, pq0 = cwt_tail(t, W, f)
    tsd64 = {k: torch.from_numpy(np.asarray(v, np.float64)) for k, v in tsd.items()}
    f64, W64 = f.double().cpu().contiguous(), W.double().cpu()
    with torch.no_grad():
        fh = O.normalize(f64)
        W2o = O.cwt_forward(W64, fh, fh, tsd64, 4)
        pqo = O.classify(W2o, fh)
        pq0o = O.classify(W64, f64)
    errs = dict(W2=rel(W2, W2o), pred_q=rel(pq, pqo), pred_q0=rel(pq0, pq0o))
    print(f"fused tail vs oracle: {errs}")
    assert max(errs.values()) < 1e-5, errs


def test_fold_follows_parameter_changes(dev):
    from few_shot_seg_cwt_amd import MultiHeadAttentionOne
    from few_shot_seg_cwt_amd.episode import cwt_tail
    from few_shot_seg_cwt_amd.optimizer import HipSGD
    t = MultiHeadAttentionOne(4, 512, 512, 512, dropout=0.5)
    t.load_state_dict(syn.make_transformer_state(4, 512, SEED))
    f, W = _inputs(dev, 1, 33, "fold")
    a = cwt_tail(t, W, f)[0].clone()
    # new parameters through load_state_dict
    t.load_state_dict(syn.make_transformer_state(4, 512, SEED + 1))
    b = cwt_tail(t, W, f)[0].clone()
    assert rel(b, _modules(t, W, f)[0]) < TOL and rel(a, b) > 1e-3
    # an optimiser step writes the parameters in place (a kernel): the fold must follow it
    t.flat.grad = torch.from_numpy(syn.normal(9, "g", (t.flat.numel(),), 1.0)).to(dev)
    HipSGD([t.flat], lr=0.05).step()
    c = cwt_tail(t, W, f)[0].clone()
    assert rel(c, _modules(t, W, f)[0]) < TOL and rel(b, c) > 1e-4
    # a second module at a recycled address with the same version number does not hit the cache
    del t
    t2 = MultiHeadAttentionOne(4, 512, 512, 512, dropout=0.5)
    t2.load_state_dict(syn.make_transformer_state(4, 512, SEED + 2))
    assert rel(cwt_tail(t2, W, f)[0], _modules(t2, W, f)[0]) < TOL


# ---------------------------------------------------------------- the one-launch tail
def _labels(B, S, tag, p_ignore=0.05):
    lab = (syn.uniform01(9, "tl" + tag, B * S * S) < 0.3).astype(np.int64).reshape(B, S, S)
    lab[syn.uniform01(10, "ti" + tag, B * S * S).reshape(B, S, S) < p_ignore] = 255
    return torch.from_numpy(lab)


@pytest.mark.parametrize("B,h", [(1, 60), (1, 81), (2, 60), (4, 33), (3, 9), (1, 2), (2, 17)])
def test_episode_tail_one_launch_equals_modules(dev, B, h):
    """cwt_episode_tail (one launch, in-kernel grid barriers) against the module kernels it
    replaces: cwt_attention_infer + cwt_classify_scaled + cwt_seg_metrics_pair (W', pred_q,
    pred_q0 at fp32 rounding; integer counts equal except on pixels whose two upsampled logits
    are within rounding of each other; the CE sums to double rounding)."""
    from few_shot_seg_cwt_amd import MultiHeadAttentionOne
    from few_shot_seg_cwt_amd.episode import cwt_tail, episode_tail
    from few_shot_seg_cwt_amd.util import seg_metrics_pair
    t = MultiHeadAttentionOne(4, 512, 512, 512, dropout=0.5)
    t.load_state_dict(syn.make_transformer_state(4, 512, SEED))
    t.eval()
    S = 8 * (h - 1) + 1
    f, W = _inputs(dev, B, h, f"1l{B}_{h}")
    ql = _labels(B, S, f"{B}_{h}").to(dev)
    for rep in range(2):   # the second launch runs on the counters the first advanced
        W2, pq, pq0, iut, ce, iut0 = episode_tail(t, W, f, ql)
        W2r, pqr, pq0r = cwt_tail(t, W, f)
        iutr, cer, iut0r = seg_metrics_pair(pqr, pq0r, ql)
        torch.cuda.synchronize()
        errs = dict(W2=rel(W2, W2r), pred_q=rel(pq, pqr), pred_q0=rel(pq0, pq0r))
        print(f"one-launch tail B={B} h={h} rep={rep}: {errs}")
        assert max(errs.values()) < TOL, errs
        # pq / pqr differ at fp32 rounding: a pixel whose two upsampled logits tie within it may flip
        assert float((iut - iutr).abs().max()) <= 2 and float((iut0 - iut0r).abs().max()) <= 2
        assert float(ce[:, 1].sub(cer[:, 1]).abs().max()) == 0.0           # valid-pixel counts
        assert float(((ce[:, 0] - cer[:, 0]).abs() / cer[:, 0].abs().clamp_min(1e-30)).max()) < 1e-5


def test_episode_tail_status_clean(dev):
    """No grid-barrier timeout on a normal launch (the context's status word stays clear)."""
    from few_shot_seg_cwt_amd import MultiHeadAttentionOne, _lib
    from few_shot_seg_cwt_amd.episode import episode_tail
    t = MultiHeadAttentionOne(4, 512, 512, 512, dropout=0.5)
    t.load_state_dict(syn.make_transformer_state(4, 512, SEED))
    f, W = _inputs(dev, 1, 60, "st")
    episode_tail(t, W, f, _labels(1, 473, "st").to(dev))
    torch.cuda.synchronize()
    _lib.check_status()


def test_episode_tail_barrier_timeout_is_raised(dev):
    """A tail whose grid barrier gives up (spin bound 1 through cwt_debug_adapt_spin_limit) drains
    its grid, reports CWT_STATUS_TAIL_BARRIER and the host raises CwtError at its next check; the
    check re-arms the context (its counters are re-zeroed before the next tail), after which the
    same call is clean and equals the module kernels."""
    from few_shot_seg_cwt_amd import MultiHeadAttentionOne, _lib
    from few_shot_seg_cwt_amd.episode import cwt_tail, episode_tail
    t = MultiHeadAttentionOne(4, 512, 512, 512, dropout=0.5)
    t.load_state_dict(syn.make_transformer_state(4, 512, SEED))
    f, W = _inputs(dev, 1, 60, "to")
    ql = _labels(1, 473, "to").to(dev)
    _lib.check_status()
    c = _lib.ctx(dev.index)
    _lib.check(_lib.lib().cwt_debug_adapt_spin_limit(c, 1), "spin limit")
    try:
        episode_tail(t, W, f, ql)
        torch.cuda.synchronize()
        with pytest.raises(_lib.CwtError, match="episode tail's grid barrier timed out"):
            _lib.check_status()
    finally:
        _lib.check(_lib.lib().cwt_debug_adapt_spin_limit(c, 0), "spin limit")
    W2, pq, pq0, iut, ce, iut0 = episode_tail(t, W, f, ql)
    torch.cuda.synchronize()
    _lib.check_status()
    W2r, pqr, _ = cwt_tail(t, W, f)
    assert rel(W2, W2r) < TOL and rel(pq, pqr) < TOL


# ---------------------------------------------------------------- the tail fused behind the inner loop
def _episode_inputs(dev, shot, h, tag):
    S = 8 * (h - 1) + 1
    f_s = torch.from_numpy(syn.normal(11, "fs" + tag, (shot, 512, h, h), 1.0)).abs().to(dev)
    f_s = f_s.contiguous(memory_format=torch.channels_last)
    f_q = torch.from_numpy(syn.normal(12, "fq" + tag, (1, 512, h, h), 1.0)).abs().to(dev)
    f_q = f_q.contiguous(memory_format=torch.channels_last)
    s_lab = _labels(shot, S, "s" + tag).to(dev)
    q_lab = _labels(1, S, "q" + tag).to(dev)
    W0 = torch.from_numpy(syn.normal(13, "w0" + tag, (2, 512), 0.05)).to(dev)
    return f_s, f_q, s_lab, q_lab, W0


@pytest.mark.parametrize("shot,h", [(1, 60), (1, 33), (2, 60)])
def test_loop_tail_fused_equals_two_calls(dev, shot, h):
    """cwt_inner_adapt_tail on a context set for the pipeline's two-unit loop (the fused launch:
    the loop's workgroups run the tail behind its last step) against inner_adapt + episode_tail
    on the same context.  The loop's dW exchange is 64-bit fixed point (integer sums: exact and
    order-free), so W is bitwise the same, and so are W', pred_q, pred_q0 and
    the IoU counts (the tail's arithmetic does not depend on its grid); only the CE sum's
    per-workgroup grouping differs (1e-5).  Twice, so the second launch runs on the counters the
    first advanced, and the fused call repeated is bitwise identical in every output; the status
    word stays clear."""
    from few_shot_seg_cwt_amd import MultiHeadAttentionOne, _lib
    from few_shot_seg_cwt_amd.episode import adapt_and_tail, episode_tail, inner_adapt
    t = MultiHeadAttentionOne(4, 512, 512, 512, dropout=0.5)
    t.load_state_dict(syn.make_transformer_state(4, 512, SEED))
    t.eval()
    f_s, f_q, s_lab, q_lab, W0 = _episode_inputs(dev, shot, h, f"{shot}_{h}")
    c = _lib.new_ctx(dev.index)
    _lib.check(_lib.lib().cwt_ctx_set_adapt_units(c, 2), "adapt units")
    with _lib.using_ctx(c):
        for rep in range(2):
            Wf, (W2f, pqf, pq0f, iutf, cef, iut0f) = adapt_and_tail(t, f_s, s_lab, W0.clone(), 0.1, 50, f_q, q_lab)
            Wr = inner_adapt(f_s, s_lab, W0.clone(), 0.1, 50)
            W2r, pqr, pq0r, iutr, cer, iut0r = episode_tail(t, Wr.view(1, 2, -1), f_q, q_lab)
            torch.cuda.synchronize()
            _lib.check_status()
            errs = dict(W=rel(Wf, Wr), W2=rel(W2f, W2r), pred_q=rel(pqf, pqr), pred_q0=rel(pq0f, pq0r))
            print(f"loop+tail fused shot={shot} h={h} rep={rep}: {errs}")
            assert torch.equal(Wf, Wr) and torch.equal(W2f, W2r), errs
            assert torch.equal(pqf, pqr) and torch.equal(pq0f, pq0r), errs
            assert torch.equal(iutf, iutr) and torch.equal(iut0f, iut0r)
            assert float(cef[:, 1].sub(cer[:, 1]).abs().max()) == 0.0
            assert float(((cef[:, 0] - cer[:, 0]).abs() / cer[:, 0].abs().clamp_min(1e-30)).max()) < 1e-5
            if rep == 0:
                first = (Wf, W2f, pqf, pq0f, iutf, cef, iut0f)
            else:   # the same fused call again: every output bitwise the same, the CE sums included
                for x0, x1 in zip(first, (Wf, W2f, pqf, pq0f, iutf, cef, iut0f)):
                    assert torch.equal(x0, x1)


def test_loop_tail_fused_profile_split(dev):
    """The profile of a fused launch: a loop part and a tail part from the kernel's stamps, both
    positive and together within the launch's own event bracket."""
    from few_shot_seg_cwt_amd import MultiHeadAttentionOne, _lib
    from few_shot_seg_cwt_amd.episode import adapt_and_tail
    t = MultiHeadAttentionOne(4, 512, 512, 512, dropout=0.5)
    t.load_state_dict(syn.make_transformer_state(4, 512, SEED))
    t.eval()
    f_s, f_q, s_lab, q_lab, W0 = _episode_inputs(dev, 1, 60, "prof")
    c = _lib.new_ctx(dev.index)
    _lib.check(_lib.lib().cwt_ctx_set_adapt_units(c, 2), "adapt units")
    with _lib.using_ctx(c):
        adapt_and_tail(t, f_s, s_lab, W0.clone(), 0.1, 200, f_q, q_lab)
        torch.cuda.synchronize()
    _lib.profile_enable(1)   # (outside using_ctx: all_ctx lists the default context and the extra ones)
    with _lib.using_ctx(c):
        adapt_and_tail(t, f_s, s_lab, W0.clone(), 0.1, 200, f_q, q_lab)
        torch.cuda.synchronize()
    recs = _lib.profile_records()
    _lib.profile_enable(0)
    names = [r[0] for r in recs]
    print(recs)
    loop = [r for r in recs if r[0].startswith("inner_adapt_kernel [adapt_persist_tail_kernel<5")]
    tail = [r for r in recs if r[0] == "episode_tail_kernel"]
    brk = [r for r in recs if r[0].startswith("inner_adapt x")]
    assert len(loop) == 1 and len(tail) == 1 and len(brk) == 1, names
    assert loop[0][3] > 0.1 and 0.0 < tail[0][3] < 1.0
    assert loop[0][3] + tail[0][3] <= brk[0][3] * 1.05 + 0.05


def test_loop_tail_fused_barrier_timeout_is_raised(dev):
    """A fused launch whose loop barrier gives up (spin bound 1) skips the tail, reports
    CWT_STATUS_ADAPT_BARRIER and the host raises at its next check; the check re-arms the tail's
    counters too (the skipped tail never arrived on them), after which the same call is clean and
    equals the two separate calls."""
    from few_shot_seg_cwt_amd import MultiHeadAttentionOne, _lib
    from few_shot_seg_cwt_amd.episode import adapt_and_tail, episode_tail, inner_adapt
    t = MultiHeadAttentionOne(4, 512, 512, 512, dropout=0.5)
    t.load_state_dict(syn.make_transformer_state(4, 512, SEED))
    t.eval()
    f_s, f_q, s_lab, q_lab, W0 = _episode_inputs(dev, 1, 60, "to")
    c = _lib.new_ctx(dev.index)
    _lib.check(_lib.lib().cwt_ctx_set_adapt_units(c, 2), "adapt units")
    with _lib.using_ctx(c):
        adapt_and_tail(t, f_s, s_lab, W0.clone(), 0.1, 20, f_q, q_lab)   # the counters advanced once
        torch.cuda.synchronize()
        _lib.check_status()
        _lib.check(_lib.lib().cwt_debug_adapt_spin_limit(c, 1), "spin limit")
        try:
            adapt_and_tail(t, f_s, s_lab, W0.clone(), 0.1, 20, f_q, q_lab)
            torch.cuda.synchronize()
            with pytest.raises(_lib.CwtError, match="barrier timed out"):
                _lib.check_status()
        finally:
            _lib.check(_lib.lib().cwt_debug_adapt_spin_limit(c, 0), "spin limit")
        Wf, (W2f, pqf, _, _, _, _) = adapt_and_tail(t, f_s, s_lab, W0.clone(), 0.1, 20, f_q, q_lab)
        torch.cuda.synchronize()
        _lib.check_status()
        Wr = inner_adapt(f_s, s_lab, W0.clone(), 0.1, 20)
        W2r, pqr, _, _, _, _ = episode_tail(t, Wr.view(1, 2, -1), f_q, q_lab)
        torch.cuda.synchronize()
    assert rel(Wf, Wr) < TOL and rel(W2f, W2r) < TOL and rel(pqf, pqr) < TOL

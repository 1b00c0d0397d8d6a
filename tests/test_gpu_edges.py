"""Edge cases of the episode path on the device, with the reference's behaviour as the oracle:

* a support mask without foreground: test.py:169-175 / train.py:197-199 divide #bg by #fg in
  Python and raise ZeroDivisionError before any device work;
* a query whose every pixel is 255: CrossEntropyLoss(ignore_index=255) gives a NaN loss
  (test.py:222-224, train.py:261-265) and ZERO gradients, so the CWT step that follows is the
  optimiser step on a zero gradient, and the IoU counts of that episode are all zero
  (util.py:237-277 drops ignored pixels);
* partially ignored query labels through the weighted query CE, against torch's own loss and
  gradient (class weight [1, #bg/(#fg + 1e-12)], train.py:237-243).
torch's CrossEntropyLoss stands in for the reference here: it is the call the reference makes."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from few_shot_seg_cwt_amd import synthetic as syn  # noqa: E402

SEED = 2021


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


def _model():
    from few_shot_seg_cwt_amd import get_model
    m = get_model(syn.cfg_defaults(layers=50))
    m.load_state_dict(syn.make_pspnet_state(50, SEED))
    return m


def _transformer():
    from few_shot_seg_cwt_amd import MultiHeadAttentionOne
    t = MultiHeadAttentionOne(4, 512, 512, 512, dropout=0.5)
    t.load_state_dict(syn.make_transformer_state(4, 512, SEED))
    return t


class _Edited:
    """A SyntheticEpisodes stream with one episode's labels rewritten."""

    def __init__(self, base, index, edit):
        self.base, self.index, self.edit = base, index, edit

    def __len__(self):
        return len(self.base)

    def __iter__(self):
        outer = self

        class _It:
            i = 0

            def next(self):
                r = list(outer.base.episode(self.i % len(outer.base)))
                if self.i == outer.index:
                    r = outer.edit(r)
                self.i += 1
                return tuple(r)

            __next__ = next

        return _It()


def _no_fg_support(r):
    s = r[3].clone()
    s[s == 1] = 0
    r[3] = s
    return r


def _ignored_query(r):
    r[1] = torch.full_like(r[1], 255)
    return r


def test_validate_raises_without_support_foreground(dev):
    from few_shot_seg_cwt_amd.episode import SyntheticEpisodes, validate_transformer
    cfg = syn.cfg_defaults(test_num=2, n_runs=1)
    with pytest.raises(ZeroDivisionError):
        validate_transformer(cfg, _Edited(SyntheticEpisodes(2), 0, _no_fg_support), _model(), _transformer().eval())


def test_train_raises_without_support_foreground(dev):
    from few_shot_seg_cwt_amd.episode import SyntheticEpisodes, do_epoch
    from few_shot_seg_cwt_amd.optimizer import get_optimizer
    cfg = syn.cfg_defaults()
    t = _transformer()
    opt = get_optimizer(cfg, [dict(params=[t.flat], lr=cfg["trans_lr"] * cfg["scale_lr"])])
    with pytest.raises(ZeroDivisionError):
        do_epoch(cfg, _Edited(SyntheticEpisodes(1), 0, _no_fg_support), _model(), t, opt, epoch=1,
                 iter_per_epoch=1, log_iter=1)


def test_validate_with_an_ignored_query(dev):
    """Episode 1 of 3 has an all-255 query: its loss is NaN (so the mean loss is NaN, as the
    reference's AverageMeter gives), its IoU counts and CE count are zero, and the other
    episodes are those of the unedited stream."""
    from few_shot_seg_cwt_amd.episode import SyntheticEpisodes, validate_transformer
    cfg = syn.cfg_defaults(test_num=3, n_runs=1)
    m, t = _model(), _transformer().eval()
    torch.manual_seed(SEED)
    base = []
    miou0, loss0 = validate_transformer(cfg, SyntheticEpisodes(3), m, t, episodes_out=base)
    torch.manual_seed(SEED)
    eps = []
    miou, loss = validate_transformer(cfg, _Edited(SyntheticEpisodes(3), 1, _ignored_query), m, t, episodes_out=eps)
    assert math.isfinite(loss0) and math.isnan(loss)
    assert float(eps[1]["ce"][0, 1]) == 0.0
    assert float(eps[1]["iut"].abs().sum()) == 0.0 and float(eps[1]["iut0"].abs().sum()) == 0.0
    for e in (0, 2):
        for k in ("W", "pred_q", "iut", "ce"):
            a, b = eps[e][k].double(), base[e][k].double()
            assert float((a - b).abs().max()) <= 1e-6 * max(float(b.abs().max()), 1e-30), (e, k)
    # the run's mIoU is the per-class FG sums without episode 1 (test.py:227-235)
    sums = {}
    for e in (0, 2):
        c = syn.make_episode(SEED, e, 473, 1, syn.pascal_val_classes(0))["subcls"][0]
        iut = eps[e]["iut"].double().numpy()[0]
        sums.setdefault(c, np.zeros(2))
        sums[c] += (iut[0, 1], iut[1, 1])
    c1 = syn.make_episode(SEED, 1, 473, 1, syn.pascal_val_classes(0))["subcls"][0]
    sums.setdefault(c1, np.zeros(2))
    want = float(np.mean([s[0] / (s[1] + 1e-10) for s in sums.values()]))
    assert abs(miou - want) < 1e-6, (miou, want, miou0)


@pytest.mark.parametrize("frac_ignored", [1.0, 0.5, 0.0])
def test_query_ce_vs_torch(dev, frac_ignored):
    """seg_ce_fwd_bwd (the training query CE) against torch's weighted CrossEntropyLoss on the
    upsampled logits: loss and d logits, including the all-ignored case (NaN loss, zero grad)."""
    from few_shot_seg_cwt_amd.episode import seg_ce_fwd_bwd
    g = torch.Generator().manual_seed(5)
    B, h, w, S = 1, 60, 60, 473
    logits = torch.randn(B, 2, h, w, generator=g)
    target = (torch.rand(B, S, S, generator=g) > 0.7).long()
    target[torch.rand(B, S, S, generator=g) < frac_ignored] = 255
    loss, dl = seg_ce_fwd_bwd(logits.to(dev), target.to(dev))
    x = logits.double().requires_grad_(True)
    up = torch.nn.functional.interpolate(x, size=(S, S), mode="bilinear", align_corners=True)
    nb, nf = int((target == 0).sum()), int((target == 1).sum())
    crit = torch.nn.CrossEntropyLoss(weight=torch.tensor([1.0, nb / (nf + 1e-12)], dtype=torch.float64),
                                     ignore_index=255)
    ref = crit(up, target)
    ref.backward()
    dl = dl.double().cpu()
    if frac_ignored == 1.0:
        assert math.isnan(float(loss.item())) and math.isnan(float(ref.detach()))
        assert float(dl.abs().max()) == 0.0 and float(x.grad.abs().max()) == 0.0
    else:
        assert abs(float(loss.item()) - float(ref.detach())) <= 1e-5 * abs(float(ref.detach()))
        assert float((dl - x.grad).abs().max()) <= 1e-4 * float(x.grad.abs().max())


def test_train_step_with_an_ignored_query(dev):
    """do_epoch on an episode whose query is all 255: NaN loss (train.py:261-265) and a CWT step
    on a zero gradient -- the parameters equal the optimiser's step from a zero gradient, and
    stay finite."""
    from few_shot_seg_cwt_amd.episode import SyntheticEpisodes, do_epoch
    from few_shot_seg_cwt_amd.optimizer import get_optimizer
    cfg = syn.cfg_defaults()
    t = _transformer()
    t.attention.dropout.p = 0.0
    t.dropout.p = 0.0
    t_ref = _transformer()
    lr = cfg["trans_lr"] * cfg["scale_lr"]
    opt = get_optimizer(cfg, [dict(params=[t.flat], lr=lr)])
    opt_ref = get_optimizer(cfg, [dict(params=[t_ref.flat], lr=lr)])
    m = _model()
    m.bn_train_mode = False
    torch.manual_seed(SEED)
    _, losses = do_epoch(cfg, _Edited(SyntheticEpisodes(1), 0, _ignored_query), m, t, opt, epoch=1,
                         iter_per_epoch=1, log_iter=1)
    assert math.isnan(float(losses[0]))
    assert bool(torch.isfinite(t.flat).all())
    t_ref.flat.grad = torch.zeros_like(t_ref.flat)
    opt_ref.step()
    assert float((t.flat.detach().cpu() - t_ref.flat.detach().cpu()).abs().max()) == 0.0

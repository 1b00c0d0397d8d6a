"""The persistent inner loop (adapt_persist_kernel: all 200 SGD steps in one launch, in-kernel
grid barrier) against the per-step launches it replaces (CWT_ADAPT_PERSIST=0) on the same
inputs, at the BASELINE shapes and in batched / multi-unit-per-workgroup geometries.  Both
are fp32; the step launches sum the gradient with float atomics and the persistent loop with
64-bit fixed-point atomics (exact), so they agree to rounding; the oracle and
reference fixtures pin the absolute result (test_gpu_parity.py, test_gpu_shapes.py)."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

from few_shot_seg_cwt_amd import synthetic as syn  # noqa: E402

SEED = 2021


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


def _run(persist, f, lbl, W0, iters, uc=None, upw=None, stream=None, res1=None):
    """persist: "0" per-step launches, "2" the persistent loop also where units are streamed;
    upw: units per workgroup ("1": f in registers; "2": two units in lockstep, both in registers
    (adapt_persist_kernel<5>); "2lds": the same with the second unit's f in LDS (<2>));
    stream: "1" the LDS-streamed form from 3 units per workgroup, "0" never; res1: "1" the first
    unit of each workgroup resident in registers (<6>, opt-in), default every unit streamed (<3>)."""
    from few_shot_seg_cwt_amd.episode import inner_adapt_batch
    breg = None
    if upw == "2lds":
        upw, breg = "2", "0"
    env = {"CWT_ADAPT_PERSIST": persist, "CWT_ADAPT_UC": uc, "CWT_ADAPT_UPW": upw, "CWT_ADAPT_STREAM": stream,
           "CWT_ADAPT_BREG": breg, "CWT_ADAPT_RES1": res1}
    old = {k: os.environ.get(k) for k in env}
    for k, v in env.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    try:
        W = inner_adapt_batch(f, lbl, W0.clone(), 0.1, iters)
        torch.cuda.synchronize()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return W


@pytest.mark.parametrize("E,n,S,iters,uc", [
    (1, 1, 473, 200, None),  # config #2: 236 15-column units, one per workgroup (f resident in registers)
    (1, 1, 473, 200, "31"),  # ... as 118 31-column units
    (1, 5, 473, 200, None),  # config #3: 590 units, three per workgroup in lockstep (197 workgroups)
    (8, 5, 129, 20, None),   # 640 units, three per workgroup, workgroups spanning two episodes
    (1, 1, 641, 200, None),  # config #4 shapes: 240 units
    (1, 5, 641, 50, None),   # config #5 shapes: 1200 units
    (4, 1, 473, 50, None),   # episodes in flight: workgroups span two episodes
    (16, 1, 129, 20, None),
    (3, 2, 65, 20, None),
    (2, 1, 33, 5, None),
])
@pytest.mark.parametrize("upw", ["1", "2", "2lds"])
def test_persist_equals_step_launches(dev, E, n, S, iters, uc, upw):
    h = (S - 1) // 8 + 1
    f = torch.from_numpy(syn.normal(5, f"fp{E}{n}{S}", (E * n, 512, h, h), 0.1)).to(dev)
    f = f.contiguous(memory_format=torch.channels_last)
    lbl = torch.stack([torch.from_numpy(syn.make_episode(SEED, 70 + e, S, n)["s_label"][0]) for e in range(E)]).to(dev)
    W0 = torch.from_numpy(syn.normal(6, f"wp{E}{n}{S}", (E, 2, 512), 0.04)).to(dev)
    Wp = _run("2", f, lbl, W0, iters, uc, upw)
    Ws = _run("0", f, lbl, W0, iters)
    errs = [rel(Wp[e], Ws[e]) for e in range(E)]
    print(f"E={E} n={n} S={S} iters={iters} upw={upw}: max rel {max(errs):.3e}")
    assert max(errs) < 1e-4, errs
    assert torch.isfinite(Wp).all()


@pytest.mark.parametrize("E,n,S,iters", [
    (1, 5, 473, 50),   # 590 units over 256 workgroups: 2-3 streamed units each
    (1, 5, 641, 20),   # 1200 units: 4-5 each
    (2, 3, 129, 20),   # workgroups spanning two episodes
    (6, 1, 65, 10),
])
@pytest.mark.parametrize("res1", ["0", "1"])
def test_lds_streamed_units_equal_step_launches(dev, E, n, S, iters, res1):
    """The LDS-streamed form (each wave DMAs its 32-channel slice of the next unit into its own
    LDS while the current unit is computed; per-episode register sums of the butterfly results)
    forced on from 3 units per workgroup; res1 "1": the first unit of each workgroup resident in
    registers (adapt_persist_kernel<6>), "0": every unit streamed (<3>)."""
    h = (S - 1) // 8 + 1
    f = torch.from_numpy(syn.normal(7, f"fs{E}{n}{S}", (E * n, 512, h, h), 0.1)).to(dev)
    f = f.contiguous(memory_format=torch.channels_last)
    lbl = torch.stack([torch.from_numpy(syn.make_episode(SEED, 90 + e, S, n)["s_label"][0]) for e in range(E)]).to(dev)
    W0 = torch.from_numpy(syn.normal(8, f"ws{E}{n}{S}", (E, 2, 512), 0.04)).to(dev)
    Wp = _run("2", f, lbl, W0, iters, upw="1" if E * n * ((h - 1) * ((h - 2) // 31 + 1)) > 256 else "2",
              stream="1", res1=res1)
    Ws = _run("0", f, lbl, W0, iters)
    errs = [rel(Wp[e], Ws[e]) for e in range(E)]
    print(f"stream E={E} n={n} S={S} res1={res1}: max rel {max(errs):.2e}")
    assert max(errs) < 1e-4, errs


@pytest.mark.parametrize("upw", ["1", "2"])
def test_barrier_timeout_is_raised(dev, upw):
    """A persistent loop whose grid barrier gives up (cwt_debug_adapt_spin_limit = 1: nearly
    every poll exhausts its bound) drains the grid, reports CWT_STATUS_ADAPT_BARRIER in the
    context's status word, and the host raises CwtError at its next check (the readbacks of
    validate_transformer / do_epoch call _lib.check_status); with the default bound restored
    the same call is clean and matches the step launches."""
    from few_shot_seg_cwt_amd import _lib
    from few_shot_seg_cwt_amd.episode import inner_adapt_batch
    S, n = 473, 1
    h = (S - 1) // 8 + 1
    f = torch.from_numpy(syn.normal(3, "fto", (n, 512, h, h), 0.1)).to(dev)
    f = f.contiguous(memory_format=torch.channels_last)
    lbl = torch.from_numpy(syn.make_episode(SEED, 9, S, n)["s_label"][0]).to(dev)[None]
    W0 = torch.from_numpy(syn.normal(4, "wto", (1, 2, 512), 0.04)).to(dev)
    _lib.check_status()   # clean before
    c = _lib.ctx(dev.index)
    _lib.check(_lib.lib().cwt_debug_adapt_spin_limit(c, 1), "spin limit")
    old = os.environ.get("CWT_ADAPT_UPW")
    os.environ["CWT_ADAPT_UPW"] = upw
    try:
        inner_adapt_batch(f, lbl, W0.clone(), 0.1, 200)
        torch.cuda.synchronize()
        with pytest.raises(_lib.CwtError, match="grid barrier timed out"):
            _lib.check_status()
        _lib.check_status()   # the check cleared the word
    finally:
        _lib.check(_lib.lib().cwt_debug_adapt_spin_limit(c, 0), "spin limit")
        if old is None:
            os.environ.pop("CWT_ADAPT_UPW", None)
        else:
            os.environ["CWT_ADAPT_UPW"] = old
    W = _run("1", f, lbl, W0, 200, upw=upw)
    _lib.check_status()
    Wr = _run("0", f, lbl, W0, 200)
    assert rel(W, Wr) < 1e-4


@pytest.mark.parametrize("E,n,S,iters,upw,stream", [
    (1, 1, 473, 200, "1", None),    # config #2 sequential geometry (adapt_persist_kernel<1>)
    (1, 1, 473, 200, "2", None),    # the pipeline's two-unit register form (<5>)
    (1, 1, 473, 50, "2lds", None),  # <2>
    (1, 5, 473, 50, None, None),    # config #3: three units in lockstep (<4>)
    (1, 5, 641, 20, None, "1"),     # the LDS-streamed form (<3>)
    (4, 1, 129, 20, None, None),    # workgroups spanning two episodes
])
def test_persist_loop_is_deterministic(dev, E, n, S, iters, upw, stream):
    """The persistent loop's dW exchange sums 64-bit fixed-point integers (exact, order-free:
    AdaptScalars.fx_scale), so the same call twice gives bitwise the same W whatever order the
    workgroups' atomics land in -- as the reference's CPU path is bitwise deterministic (SURVEY
    §0).  Five repeats, every geometry form."""
    h = (S - 1) // 8 + 1
    f = torch.from_numpy(syn.normal(9, f"fd{E}{n}{S}", (E * n, 512, h, h), 0.1)).to(dev)
    f = f.contiguous(memory_format=torch.channels_last)
    lbl = torch.stack([torch.from_numpy(syn.make_episode(SEED, 40 + e, S, n)["s_label"][0]) for e in range(E)]).to(dev)
    W0 = torch.from_numpy(syn.normal(10, f"wd{E}{n}{S}", (E, 2, 512), 0.04)).to(dev)
    W1 = _run("2", f, lbl, W0, iters, upw=upw, stream=stream)
    for _ in range(4):
        assert torch.equal(_run("2", f, lbl, W0, iters, upw=upw, stream=stream), W1)
    Ws = _run("0", f, lbl, W0, iters)   # and still the float-atomic step launches' result to rounding
    assert max(rel(W1[e], Ws[e]) for e in range(E)) < 1e-4


def test_persist_loop_nonfinite_features(dev):
    """A NaN in the support features makes the adapted W NaN (the fixed-point scale cannot be
    formed: fx_inv NaN), as the reference's float sums would, instead of garbage integers."""
    S, n = 129, 1
    h = (S - 1) // 8 + 1
    f = torch.from_numpy(syn.normal(11, "fnan", (n, 512, h, h), 0.1)).to(dev)
    f[0, 7, 3, 4] = float("nan")
    f = f.contiguous(memory_format=torch.channels_last)
    lbl = torch.from_numpy(syn.make_episode(SEED, 12, S, n)["s_label"][0]).to(dev)[None]
    W0 = torch.from_numpy(syn.normal(12, "wnan", (1, 2, 512), 0.04)).to(dev)
    W = _run("2", f, lbl, W0, 5, upw="1")
    assert torch.isnan(W).all()

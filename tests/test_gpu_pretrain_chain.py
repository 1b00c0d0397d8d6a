"""Teacher-forced per-stage parity of the pretraining backward (reference
src/pretrain.py:104-121 -- ``loss.backward()`` through PSPNet.forward, pspnet.py:147-156).

The whole-network gradient of the synthetic, untrained PSPNet under training-mode BN is
ill-conditioned at fp32: the oracle's own fp32 and float64 gradients differ by 10-20 % on deep
layer3/4 tensors (tests/test_gpu_pretrain.py prints that spread), so a whole-step comparison can
only bound the chain.  This test pins every stage of the chain instead.  One HIP training step
runs with its transient gradients captured (cwt_debug_pretrain_capture); then, for every stage,
the oracle (float64 torch autograd of the reference's modules, cwt_oracle / pretrain_oracle)
recomputes that stage's backward from the HIP forward's OWN inputs and the HIP backward's OWN
upstream gradient -- its input activation, its ReLU masks and max-pool choices (so a rounding-level
mask flip cannot move the comparison), the Dropout2d mask -- and every parameter gradient and
the stage's input gradient must match at BAR.  Errors cannot compound across stages.

Stages: the loss (smoothed CE of the upsampled logits -> dlogits), the head (classifier, bottleneck
conv + BN + ReLU + Dropout2d, the four PPM branches -> dcat), every ResNet bottleneck block
(resnet.py:74-96, with the dilation surgery of pspnet.py:103-112 -> the block input gradient), and
the stem (three conv + BN + ReLU, max-pool; resnet.py:110-118).  Printed: the worst relative error
per stage.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from few_shot_seg_cwt_amd import synthetic as syn  # noqa: E402
from dropout_ref import dropout_scale  # noqa: E402

SEED = 2021
BAR = 1e-4       # max |HIP - oracle| / max |oracle| per tensor
BN_EPS = 1e-5


def rel(a, b):
    a = a.detach().double().cpu().numpy()
    b = b.detach().double().cpu().numpy()
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


def _tensor(model, name, shape):
    """A captured / forward tensor of the last HIP step as float64, NHWC rows -> [N, C, H, W]."""
    from few_shot_seg_cwt_amd import _lib
    N, H, W, C = shape
    out = np.empty((N * H * W * C,), np.float32)
    _lib.check(_lib.lib().cwt_debug_pretrain_tensor(model._h, name.encode(), out.ctypes.data, out.size), name)
    return torch.from_numpy(out).double().reshape(N, H, W, C).permute(0, 3, 1, 2).contiguous()


def _bn(x, P, p):
    # training-mode nn.BatchNorm2d: batch statistics (running statistics do not enter the gradient)
    return F.batch_norm(x, None, None, P[p + ".weight"], P[p + ".bias"], training=True, eps=BN_EPS)


def _block(x, P, li, bi, m):
    """Bottleneck.forward (resnet.py:74-96) with the HIP forward's ReLU masks m[1..3]."""
    from oracle.cwt_oracle import block_geometry
    p = f"layer{li}.{bi}"
    s, d, ds = block_geometry(li, bi)
    o = _bn(F.conv2d(x, P[p + ".conv1.weight"]), P, p + ".bn1") * m[1]
    o = _bn(F.conv2d(o, P[p + ".conv2.weight"], None, s, d, d), P, p + ".bn2") * m[2]
    o = _bn(F.conv2d(o, P[p + ".conv3.weight"]), P, p + ".bn3")
    res = _bn(F.conv2d(x, P[p + ".downsample.0.weight"], None, ds), P, p + ".downsample.1") if bi == 0 else x
    return (o + res) * m[3]


def _report(stage, errs, worst):
    w = max(errs.values())
    worst[stage] = w
    bad = {k: v for k, v in errs.items() if not v < BAR}
    assert not bad, f"{stage}: " + ", ".join(f"{k} {v:.3g}" for k, v in sorted(bad.items(), key=lambda t: -t[1])[:8])


@pytest.mark.parametrize("layers,N,S,nc,drop", [(50, 4, 65, 16, 0.1), (101, 2, 65, 16, 0.0), (50, 2, 129, 61, 0.0)])
def test_pretrain_backward_teacher_forced(dev, layers, N, S, nc, drop):
    from few_shot_seg_cwt_amd import _lib
    from few_shot_seg_cwt_amd.pretrain import PretrainPSPNet
    from oracle.cwt_oracle import RESNET_BLOCKS
    from oracle.pretrain_oracle import smoothed_ce
    a = dict(layers=layers, num_classes_tr=nc, lr=0.0025, scale_lr=2.0, momentum=0.9, weight_decay=1e-4,
             nesterov=True, smoothing=True, dropout=drop)
    state = syn.make_pspnet_state(layers, SEED, num_classes_tr=nc)
    model = PretrainPSPNet(a, state, dev)
    x = torch.from_numpy(syn.normal(SEED, "ptc_img", (N, 3, S, S), 1.0))
    t = (syn.uniform01(SEED, "ptc_lbl", N * S * S) * nc).astype(np.int64).reshape(N, S, S)
    t[syn.uniform01(SEED, "ptc_ign", N * S * S).reshape(N, S, S) < 0.05] = 255
    t = torch.from_numpy(t)
    seed = 77
    _lib.check(_lib.lib().cwt_debug_pretrain_capture(model._h, 1), "capture")
    model.train_step(x.to(dev), t.to(dev), seed=seed)
    torch.cuda.synchronize()
    # the step's gradients were taken at the initial parameters (the SGD update came after)
    P = {k: torch.from_numpy(np.asarray(v, np.float64)).requires_grad_(True) for k, v in state.items()
         if not (k.endswith(("running_mean", "running_var", "num_batches_tracked")) or k == "gamma")}
    G = {k: model.grad(k).double() for k in P}
    Hs = (S - 1) // 2 + 1
    H1 = (Hs - 1) // 2 + 1
    h = (H1 - 1) // 2 + 1
    worst = {}

    # ---- loss: smoothed CE of the upsampled HIP logits (pretrain.py:163-219) -> dlogits ----
    lg = _tensor(model, "logits", (N, h, h, nc)).requires_grad_(True)
    up = F.interpolate(lg, size=(S, S), mode="bilinear", align_corners=True)
    smoothed_ce(up, t, nc, True).backward()
    dlog = _tensor(model, "dlogits", (N, h, h, nc))
    _report("loss", {"dlogits": rel(dlog, lg.grad)}, worst)

    # ---- head: PPM (pspnet.py:19-38) + bottleneck conv/BN/ReLU/Dropout2d + classifier ----
    cat = _tensor(model, "cat", (N, h, h, 2048)).requires_grad_(True)
    outs = [cat]
    for i, b in enumerate((1, 2, 3, 6)):
        y = F.conv2d(F.adaptive_avg_pool2d(cat, b), P[f"ppm.features.{i}.1.weight"])
        mb = (_tensor(model, f"a:ppm{i}", (N, b, b, 512)) > 0).double()
        y = _bn(y, P, f"ppm.features.{i}.2") * mb
        outs.append(F.interpolate(y, (h, h), mode="bilinear", align_corners=True))
    f = _bn(F.conv2d(torch.cat(outs, 1), P["bottleneck.0.weight"], None, 1, 1), P, "bottleneck.1")
    f = f * (_tensor(model, "fpre", (N, h, h, 512)) > 0).double()
    if drop > 0:
        ds = dropout_scale(drop, seed, 3, np.arange(N * 512, dtype=np.uint64)).reshape(N, 512)
        f = f * torch.from_numpy(ds)[:, :, None, None]
    logits = F.conv2d(f, P["classifier.weight"])
    (logits * dlog).sum().backward()
    head = [k for k in P if k.startswith(("ppm.", "bottleneck.", "classifier."))]
    errs = {k: rel(G[k], P[k].grad) for k in head}
    errs["dcat"] = rel(_tensor(model, "dcat", (N, h, h, 2048)), cat.grad)
    _report("head", errs, worst)

    # ---- ResNet blocks, each from its HIP input, masks and output gradient ----
    nblocks = RESNET_BLOCKS[layers]
    dims = []
    H = H1
    cin = 128
    for li, planes in enumerate((64, 128, 256, 512), start=1):
        for bi in range(nblocks[li - 1]):
            Ho = (H - 1) // 2 + 1 if (li == 2 and bi == 0) else H
            dims.append((li, bi, H, Ho, cin, planes))
            cin, H = planes * 4, Ho
    for k, (li, bi, H, Ho, ci, planes) in enumerate(dims):
        xin = _tensor(model, f"in:l{li}.{bi}", (N, H, H, ci)).requires_grad_(True)
        m = {1: (_tensor(model, f"a:l{li}.{bi}.c1", (N, H, H, planes)) > 0).double(),
             2: (_tensor(model, f"a:l{li}.{bi}.c2", (N, Ho, Ho, planes)) > 0).double(),
             3: (_tensor(model, f"a:l{li}.{bi}.c3", (N, Ho, Ho, planes * 4)) > 0).double()}
        out = _block(xin, P, li, bi, m)
        if k + 1 < len(dims):
            nli, nbi = dims[k + 1][:2]
            dout = _tensor(model, f"dx:l{nli}.{nbi}", (N, Ho, Ho, planes * 4))
        else:
            dout = _tensor(model, "dcat", (N, Ho, Ho, planes * 4))
        (out * dout).sum().backward()
        pre = f"layer{li}.{bi}."
        errs = {kk: rel(G[kk], P[kk].grad) for kk in P if kk.startswith(pre)}
        errs["dx"] = rel(_tensor(model, f"dx:l{li}.{bi}", (N, H, H, ci)), xin.grad)
        _report(f"layer{li}.{bi}", errs, worst)

    # ---- stem (resnet.py:110-118) from the image, with the HIP ReLU masks and max-pool choices ----
    xs = x.double()
    a0 = _bn(F.conv2d(xs, P["layer0.0.weight"], None, 2, 1), P, "layer0.1") * \
        (_tensor(model, "a:stem0", (N, Hs, Hs, 64)) > 0).double()
    a1 = _bn(F.conv2d(a0, P["layer0.3.weight"], None, 1, 1), P, "layer0.4") * \
        (_tensor(model, "a:stem1", (N, Hs, Hs, 64)) > 0).double()
    a2h = _tensor(model, "a:stem2", (N, Hs, Hs, 128))
    a2 = _bn(F.conv2d(a1, P["layer0.6.weight"], None, 1, 1), P, "layer0.7") * (a2h > 0).double()
    _, idx = F.max_pool2d(a2h, 3, 2, 1, return_indices=True)   # the HIP forward's argmax (first maximum)
    mp = a2.flatten(2).gather(2, idx.flatten(2)).view(N, 128, H1, H1)
    (mp * _tensor(model, "dx:l1.0", (N, H1, H1, 128))).sum().backward()
    _report("stem", {k: rel(G[k], P[k].grad) for k in P if k.startswith("layer0.")}, worst)

    _lib.check(_lib.lib().cwt_debug_pretrain_capture(model._h, 0), "capture")
    print(f"teacher-forced R{layers} N={N} S={S} nc={nc} drop={drop}: worst per stage " +
          ", ".join(f"{k} {v:.2e}" for k, v in worst.items()))

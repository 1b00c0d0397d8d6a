"""ORACLE — test infrastructure only.  CPU fp32 restatement of the reference CWT path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker / the timed CPU baseline.  The product path
(``few_shot_seg_cwt_amd``) never imports it and has no CPU fallback.

This is a functional restatement in plain PyTorch (CPU, fp32) of the reference
TeamOfProfGuo/Few_Shot_Seg_CWT episode path; every function cites the reference
file:line it follows.  Parity of this restatement is PINNED against golden vectors that
``tests/golden/make_golden.py`` produced by running the reference's own modules and
drivers (``validate_transformer``, ``do_epoch``, ``MultiHeadAttentionOne``) in the survey
container; ``tests/test_oracle_golden.py`` checks it.

State dicts use the reference key names (see few_shot_seg_cwt_amd/synthetic.py).
"""
from __future__ import annotations

import math
from typing import Dict, List, Tuple

import numpy as np
import torch
import torch.nn.functional as F

RESNET_BLOCKS = {50: (3, 4, 6, 3), 101: (3, 4, 23, 3)}
BN_EPS = 1e-5


def to_torch_state(sd) -> Dict[str, torch.Tensor]:
    return {k: (v if isinstance(v, torch.Tensor) else torch.from_numpy(np.asarray(v))) for k, v in sd.items()}


def _bn(x, sd, p, mom=None):
    # nn.BatchNorm2d in eval mode (running statistics), eps 1e-5; mom != None: training mode
    # (batch statistics, running statistics of sd moved in place by mom, unbiased variance)
    return F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"], sd[p + ".weight"],
                        sd[p + ".bias"], training=mom is not None, momentum=0.0 if mom is None else mom,
                        eps=BN_EPS)


def _conv(x, sd, name, stride=1, padding=0, dilation=1):
    return F.conv2d(x, sd[name], None, stride, padding, dilation)


def stem(x, sd, mom=None):
    """layer0 (pspnet.py:93-95; resnet.py:110-118): 3x[conv3x3+BN+ReLU] (first stride 2) + maxpool 3/2/1."""
    x = F.relu(_bn(_conv(x, sd, "layer0.0.weight", 2, 1), sd, "layer0.1", mom))
    x = F.relu(_bn(_conv(x, sd, "layer0.3.weight", 1, 1), sd, "layer0.4", mom))
    x = F.relu(_bn(_conv(x, sd, "layer0.6.weight", 1, 1), sd, "layer0.7", mom))
    return F.max_pool2d(x, 3, 2, 1)


def block_geometry(layer: int, block: int) -> Tuple[int, int, int]:
    """(conv2 stride, conv2 dilation, downsample stride) after the dilation surgery of
    pspnet.py:103-112 applied to resnet.py:133-147 (stride on conv2, resnet.py:65)."""
    if layer == 1:
        return 1, 1, 1
    if layer == 2:
        return (2, 1, 2) if block == 0 else (1, 1, 1)
    if layer == 3:
        return 1, 2, 1
    return 1, 4, 1


def bottleneck(x, sd, layer: int, block: int, mom=None):
    """Bottleneck.forward (resnet.py:74-96)."""
    p = f"layer{layer}.{block}"
    s, d, ds = block_geometry(layer, block)
    out = F.relu(_bn(_conv(x, sd, p + ".conv1.weight"), sd, p + ".bn1", mom))
    out = F.relu(_bn(_conv(out, sd, p + ".conv2.weight", s, d, d), sd, p + ".bn2", mom))
    out = _bn(_conv(out, sd, p + ".conv3.weight"), sd, p + ".bn3", mom)
    if block == 0:
        res = _bn(_conv(x, sd, p + ".downsample.0.weight", ds), sd, p + ".downsample.1", mom)
    else:
        res = x
    return F.relu(out + res)


def backbone(x, sd, layers: int = 50, mom=None):
    """get_feat_list (pspnet.py:272-287): layer0..layer4, returns the layer4 output."""
    x = stem(x, sd, mom)
    for li, nblk in enumerate(RESNET_BLOCKS[layers], start=1):
        for b in range(nblk):
            x = bottleneck(x, sd, li, b, mom)
    return x


def ppm(x, sd, bins=(1, 2, 3, 6), mom=None):
    """PPM.forward (pspnet.py:33-38): AdaptiveAvgPool -> 1x1 conv -> BN -> ReLU ->
    bilinear(align_corners=True) back to h x w; concat [x, b1..b4]."""
    h, w = x.shape[-2:]
    outs = [x]
    for i, b in enumerate(bins):
        y = F.adaptive_avg_pool2d(x, b)
        y = F.relu(_bn(_conv(y, sd, f"ppm.features.{i}.1.weight"), sd, f"ppm.features.{i}.2", mom))
        outs.append(F.interpolate(y, (h, w), mode="bilinear", align_corners=True))
    return torch.cat(outs, 1)


def extract_features(x, sd, layers: int = 50, train_bn_momentum=None, drop2d_scale=None):
    """PSPNet.extract_features (pspnet.py:172-181) in eval mode: backbone -> PPM ->
    bottleneck conv3x3 4096->512 + BN + ReLU (+Dropout2d, identity in eval) (pspnet.py:124-129).
    train_bn_momentum: the module in train mode (train.py:184): every BN on batch statistics,
    sd's running statistics updated in place; drop2d_scale [N,512]: the Dropout2d mask x 1/(1-p)."""
    with torch.no_grad():
        f = backbone(x, sd, layers, train_bn_momentum)
        f = ppm(f, sd, mom=train_bn_momentum)
        f = F.relu(_bn(_conv(f, sd, "bottleneck.0.weight", 1, 1), sd, "bottleneck.1", train_bn_momentum))
        if drop2d_scale is not None:
            f = f * drop2d_scale[:, :, None, None]
    return f


def class_weight(labels: np.ndarray, train_query: bool = False) -> torch.Tensor:
    """Dynamic CE class weight [1, #bg/#fg] from the host copy of the labels
    (test.py:169-175; train.py:211-217). The query variant adds 1e-12 (train.py:237-243)."""
    nb = int(np.count_nonzero(labels == 0))
    nf = int(np.count_nonzero(labels == 1))
    r = nb / (nf + 1e-12) if train_query else nb / nf
    return torch.tensor([1.0, r])


def inner_adapt(f_s, s_label, W0, lr: float, iters: int, weight: torch.Tensor):
    """Support-set inner loop (test.py:164-187; train.py:206-231): 1x1 conv classifier,
    bilinear(align_corners) upsample to the label size, weighted CE (ignore 255, mean
    reduction), plain SGD W <- W - lr*dW.  W0 is [2, C, 1, 1]."""
    W = W0.detach().clone().requires_grad_(True)
    S = s_label.shape[-2:]
    for _ in range(iters):
        out = F.conv2d(f_s, W)
        out = F.interpolate(out, size=S, mode="bilinear", align_corners=True)
        loss = F.cross_entropy(out, s_label, weight=weight, ignore_index=255)
        g, = torch.autograd.grad(loss, W)
        with torch.no_grad():
            W -= lr * g
    return W.detach()


def cwt_forward(q, k, v, tsd, heads: int, dropout: bool = False):
    """MultiHeadAttentionOne.forward (transformer.py:54-83) + ScaledDotProductAttention
    (transformer.py:23-30), eval mode (dropouts identity).  q [B,2,C], k/v [B,C,h,w]."""
    B, C = k.shape[0], k.shape[1]
    k = k.reshape(B, C, -1).permute(0, 2, 1)
    v = v.reshape(B, C, -1).permute(0, 2, 1)
    Wq = tsd["w_qkvs.weight"]
    lq, lk = q.shape[1], k.shape[1]
    residual = q
    qp = (q @ Wq.t()).view(B, lq, heads, C).permute(2, 0, 1, 3).reshape(-1, lq, C)
    kp = (k @ Wq.t()).view(B, lk, heads, C).permute(2, 0, 1, 3).reshape(-1, lk, C)
    vp = (v @ Wq.t()).view(B, lk, heads, C).permute(2, 0, 1, 3).reshape(-1, lk, C)
    attn = torch.softmax(torch.bmm(qp, kp.transpose(1, 2)) / math.sqrt(C), dim=2)
    out = torch.bmm(attn, vp).view(heads, B, lq, C).permute(1, 2, 0, 3).reshape(B, lq, -1)
    out = out @ tsd["fc.weight"].t() + tsd["fc.bias"]
    return F.layer_norm(out + residual, (C,), tsd["layer_norm.weight"], tsd["layer_norm.bias"], 1e-5)


def normalize(f):
    """F.normalize(f, dim=1) (test.py:194; train.py:250): x / max(||x||_2, 1e-12)."""
    return F.normalize(f, dim=1)


def classify(W, f):
    """1x1 conv / matmul classifier (test.py:200-204; train.py:259-261): W [B,2,C], f [B,C,h,w]."""
    B, C, h, w = f.shape
    return torch.bmm(W, f.reshape(B, C, h * w)).view(B, -1, h, w)


def upsample(logits, S: int):
    """F.interpolate(bilinear, align_corners=True) to S x S (test.py:214-215)."""
    return F.interpolate(logits, size=(S, S), mode="bilinear", align_corners=True)


def intersection_union(preds, target, num_classes: int = 2, ignore_index: int = 255):
    """intersectionAndUnionGPU (util.py:280-308): histc-based per-class counts."""
    preds = preds.reshape(-1).clone()
    target = target.reshape(-1)
    preds[target == ignore_index] = ignore_index
    inter = preds[preds == target]
    ai = torch.histc(inter.float(), bins=num_classes, min=0, max=num_classes - 1)
    ao = torch.histc(preds.float(), bins=num_classes, min=0, max=num_classes - 1)
    at = torch.histc(target.float(), bins=num_classes, min=0, max=num_classes - 1)
    return ai, ao + at - ai, at


def run_inference_episode(ep: dict, sd, tsd, W0, cfg: dict) -> dict:
    """One episode of validate_transformer (test.py:138-219) for batch_size_val = 1."""
    S = cfg["image_size"]
    spprt = torch.from_numpy(ep["spprt_imgs"])[0]
    s_label = torch.from_numpy(ep["s_label"])[0]
    qry = torch.from_numpy(ep["qry_img"])
    q_label = torch.from_numpy(ep["q_label"])
    weight = class_weight(ep["s_label"])
    f_s = extract_features(spprt, sd, cfg["layers"])
    W = inner_adapt(f_s, s_label, W0, cfg["cls_lr"], cfg["adapt_iter"], weight)
    with torch.no_grad():
        f_q = extract_features(qry, sd, cfg["layers"])
        pred_q0 = F.conv2d(f_q, W)
        fqn = normalize(f_q)
        Wr = W.reshape(1, 2, -1)
        W2 = cwt_forward(Wr, fqn, fqn, tsd, cfg["heads"])
        pred_q = classify(W2, fqn)
        up = upsample(pred_q, S)
        up0 = upsample(pred_q0, S)
        i, u, t = intersection_union(up.argmax(1)[0], q_label[0])
        i0, u0, t0 = intersection_union(up0.argmax(1)[0], q_label[0])
    return dict(f_s=f_s, f_q=f_q, W=W.reshape(2, -1), W2=W2.reshape(2, -1), pred_q=pred_q, pred_q0=pred_q0,
                inter=i, union=u, target=t, inter0=i0, union0=u0, target0=t0)


def cwt_train_step_grads(W, f_q, q_label, tsd, heads: int):
    """Outer-loop loss + gradients of the CWT params for one training episode
    (train.py:237-267) with dropout off: query CE weight [1, #bg/(#fg+1e-12)], logits
    W'.f_hat upsampled to the label size.  Returns (loss, {name: grad})."""
    params = {k: v.detach().clone().requires_grad_(True) for k, v in tsd.items()}
    fqn = normalize(f_q)
    W2 = cwt_forward(W.reshape(1, 2, -1), fqn, fqn, params, heads)
    B, C, h, w = fqn.shape
    pred = torch.matmul(W2, fqn.reshape(B, C, -1)).view(B, 2, h, w)
    pred = F.interpolate(pred, size=q_label.shape[-2:], mode="bilinear", align_corners=True)
    weight = class_weight(q_label.numpy(), train_query=True)
    loss = F.cross_entropy(pred, q_label, weight=weight, ignore_index=255)
    grads = torch.autograd.grad(loss, list(params.values()))
    return loss.detach(), dict(zip(params.keys(), grads)), pred.detach()


def sgd_nesterov(params: dict, grads: dict, bufs: dict, lr: float, momentum: float, wd: float):
    """torch.optim.SGD(momentum, nesterov, weight_decay) step (optimizer.py:8-15)."""
    out, nb = {}, {}
    for k, p in params.items():
        g = grads[k] + wd * p
        b = g.clone() if bufs.get(k) is None else momentum * bufs[k] + g
        nb[k] = b
        out[k] = p - lr * (g + momentum * b)
    return out, nb


# ---------------------------------------------------------------- variant heads (§8(f) rank 4)
def cos_cls(x, weight, g=None, bias=None, scale=2.0, weight_norm_r=False, weight_norm=False):
    """CosCls.forward (pspnet.py:300-309): x [B, C, h, w]; weight [n, C, 1, 1] (weight_v under
    WeightNorm, pspnet.py:294-295, W = g v / ||v|| per output channel, torch._weight_norm dim 0);
    weight_norm: the stored weight normalised (eps 1e-5) before use -- under WeightNorm the
    pre-forward hook recomputes the weight from (g, v) afterwards, so it has no effect there.
    Returns (scores [B, n, h, w], the weight the conv used)."""
    if weight_norm_r:
        v = weight
        w = v * (g / v.flatten(1).norm(dim=1).view(-1, 1, 1, 1))
    else:
        w = F.normalize(weight, p=2, dim=1, eps=1e-5) if weight_norm else weight
    x_norm = F.normalize(x, p=2, dim=1, eps=1e-5)
    return scale * F.conv2d(x_norm, w, bias), w


def get_corr(q, k):
    """model_util.py:101-109: cosine similarity of every (q token, k token) pair."""
    bs, ch, h, w = q.shape
    pq = F.normalize(q.view(bs, ch, h * w).permute(0, 2, 1), dim=-1)
    pk = F.normalize(k.view(bs, -1, k.shape[2] * k.shape[3]), dim=-2)
    return torch.bmm(pq, pk)

"""ORACLE — test infrastructure only.  CPU fp32 restatement of the reference's stage-1
pretraining iteration (src/pretrain.py).

Only ``tests/`` and ``bench.py``'s ``cpu_baseline`` leg may import this module.  The product
path (``few_shot_seg_cwt_amd.pretrain``) never imports it.

One iteration of pretrain.py:104-121: ``model.train()``; ``logits = model(images)`` (PSPNet
forward pspnet.py:147-156: extract_features -> classifier conv -> bilinear align_corners to
the input size); ``compute_loss`` with label smoothing (pretrain.py:182-219; ``cross_entropy``
:163-179: log_softmax, -(one_hot * logp).sum(1), masked_select of non-255 pixels, mean);
``zero_grad``; ``backward`` (torch autograd); ``optimizer.step()`` with the two parameter
groups of :60-72 (torch.optim.SGD momentum / weight decay / nesterov, optimizer.py:8-15).

The forward modules are cwt_oracle's (stem / bottleneck / ppm), which are pinned by the
reference-run fixtures (tests/golden); the backward is torch autograd of that
forward, the same algorithm the reference runs (``loss.backward()``).  Dropout2d masks are
injected (``drop2d_scale``) so the HIP path's counter-based masks can be reproduced; with the
reference's own torch RNG masks only the distribution matches.
"""
from __future__ import annotations

from typing import Dict, Tuple

import torch
import torch.nn.functional as F

from .cwt_oracle import backbone, ppm, _bn, _conv

HEAD_PREFIXES = ("ppm.", "bottleneck.", "classifier.")


def is_head(name: str) -> bool:
    """Parameter group 2 (pretrain.py:63,68-69: ppm, bottleneck, classifier at lr * scale_lr)."""
    return name.startswith(HEAD_PREFIXES)


def pspnet_logits(x, sd, layers: int = 50, train: bool = True, drop2d_scale=None, bn_momentum: float = 0.1):
    """PSPNet.forward (pspnet.py:147-156) before the upsample, autograd-enabled; train: every
    BN on batch statistics with the running statistics of sd moved in place (model.train())."""
    mom = bn_momentum if train else None
    f = backbone(x, sd, layers, mom)
    f = ppm(f, sd, mom=mom)
    f = F.relu(_bn(_conv(f, sd, "bottleneck.0.weight", 1, 1), sd, "bottleneck.1", mom))
    if drop2d_scale is not None:
        f = f * drop2d_scale[:, :, None, None]
    return F.conv2d(f, sd["classifier.weight"])


def smoothed_ce(logits_up, targets, num_classes: int, smoothing: bool = True, ignore_index: int = 255):
    """compute_loss + cross_entropy (pretrain.py:163-219) without mixup."""
    b, h, w = targets.shape
    one_hot = torch.zeros(b, num_classes, h, w)
    t = targets.clone().unsqueeze(1)
    t[t == ignore_index] = 0
    one_hot.scatter_(1, t, 1)
    if smoothing:
        eps = 0.1
        one_hot = one_hot * (1 - eps) + (1 - one_hot) * eps / (num_classes - 1)
    logp = F.log_softmax(logits_up, dim=1)
    loss = -(one_hot * logp).sum(dim=1)
    return loss.masked_select(targets.ne(ignore_index)).mean()


def pretrain_step(sd: Dict[str, torch.Tensor], images, targets, num_classes: int, layers: int = 50,
                  lr: float = 0.0025, scale_lr: float = 2.0, momentum: float = 0.9, weight_decay: float = 1e-4,
                  nesterov: bool = True, smoothing: bool = True, bufs: Dict[str, torch.Tensor] | None = None,
                  drop2d_scale=None) -> Tuple[torch.Tensor, Dict[str, torch.Tensor], Dict, Dict]:
    """One iteration.  sd: the model state (running statistics updated in place).  Returns
    (loss, grads, new params, new momentum buffers)."""
    names = [k for k, v in sd.items() if not (k.endswith("running_mean") or k.endswith("running_var")
                                               or k.endswith("num_batches_tracked") or k == "gamma")]
    params = {k: sd[k].detach().clone().requires_grad_(True) for k in names}
    work = dict(sd)
    work.update(params)
    logits = pspnet_logits(images, work, layers, True, drop2d_scale)
    up = F.interpolate(logits, size=targets.shape[-2:], mode="bilinear", align_corners=True)
    loss = smoothed_ce(up, targets, num_classes, smoothing)
    grads = dict(zip(names, torch.autograd.grad(loss, [params[k] for k in names])))
    new, nb = {}, {}
    bufs = bufs or {}
    with torch.no_grad():
        for k in names:
            p = sd[k]
            g = grads[k] + weight_decay * p
            b = g.clone() if bufs.get(k) is None else momentum * bufs[k] + g
            nb[k] = b
            d = g + momentum * b if nesterov else b
            new[k] = p - (lr * scale_lr if is_head(k) else lr) * d
    return loss.detach(), grads, new, nb

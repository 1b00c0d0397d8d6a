"""Metrics of the CWT drivers (reference src/util.py:199-308), on the device.

``intersectionAndUnionGPU`` / ``batch_intersectionAndUnionGPU`` keep the reference
signatures and return float tensors like ``torch.histc`` does, but the upsample, argmax
and histogram run as one HIP kernel (cwt_seg_metrics / cwt_iou_preds) instead of
materialising S x S logits.
"""
from __future__ import annotations

from typing import Tuple

import torch

from . import _lib


class AverageMeter:
    """util.py:199-214."""

    def __init__(self):
        self.reset()

    def reset(self):
        self.val = 0
        self.avg = 0
        self.sum = 0
        self.count = 0

    def update(self, val, n=1):
        self.val = val
        self.sum += val * n
        self.count += n
        self.avg = self.sum / self.count


_seed_state = [None, 0]


def dropout_seed() -> int:
    """Seed of one counter-based dropout draw (csrc/common.h dropout_uniform).  The reference's
    dropouts run on CUDA tensors and draw from the CUDA generator, so they never move the host
    RNG stream that the per-episode classifier init (nn.Conv2d, train.py:206) draws W0 from; to
    keep that stream identical this seed comes from the device generator's initial seed and a
    per-process counter (restarted when torch.manual_seed changes the initial seed)."""
    base = int(torch.cuda.initial_seed()) if torch.cuda.is_available() else int(torch.initial_seed())
    if _seed_state[0] != base:
        _seed_state[0], _seed_state[1] = base, 0
    n = _seed_state[1]
    _seed_state[1] += 1
    return (base * 0x9E3779B97F4A7C15 + n * 0xD1B54A32D192ED03 + 1) & ((1 << 62) - 1)


def intersectionAndUnionGPU(preds: torch.Tensor, target: torch.Tensor, num_classes: int,
                            ignore_index: int = 255) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """util.py:280-308 on argmax maps: returns (intersection, union, target) [num_classes] float."""
    assert preds.dim() in (1, 2, 3)
    assert preds.shape == target.shape
    _lib.require(preds, "preds", torch.int64)
    _lib.require(target, "target", torch.int64)
    p, t = preds.contiguous(), target.contiguous()
    out = torch.empty((3, num_classes), device=p.device, dtype=torch.float32)
    _lib.check(_lib.lib().cwt_iou_preds(_lib.ctx(p.device.index), _lib.ptr(p), _lib.ptr(t), p.numel(), num_classes,
                                        ignore_index, _lib.ptr(out), _lib.stream_ptr(p.device)), "cwt_iou_preds")
    return out[0], out[1], out[2]


def seg_metrics(logits: torch.Tensor, target: torch.Tensor, with_ce: bool = True):
    """Upsample [B,2,h,w] logits to the [B,S,S] target (bilinear, align_corners), argmax,
    histc (util.py:237-277) and the CE(ignore 255) sum (test.py:222-224).
    Returns iut [B,3,2] float32 and ce [B,2] float64 (sum nll, count) on the device."""
    _lib.require(logits, "logits")
    _lib.require(target, "target", torch.int64)
    B, nc, h, w = logits.shape
    if nc != 2:
        raise NotImplementedError("2-way episodes only (num_classes_tr = 2)")
    S = target.shape[-1]
    lg, tg = logits.contiguous(), target.contiguous()
    iut = torch.empty((B, 3, 2), device=lg.device, dtype=torch.float32)
    ce = torch.empty((B, 2), device=lg.device, dtype=torch.float64) if with_ce else None
    _lib.check(_lib.lib().cwt_seg_metrics(_lib.ctx(lg.device.index), _lib.ptr(lg), _lib.ptr(tg), B, h, w, S,
                                          _lib.ptr(iut), _lib.ptr(ce), _lib.stream_ptr(lg.device)),
               "cwt_seg_metrics")
    return iut, ce


def seg_metrics_pair(logits: torch.Tensor, logits0: torch.Tensor, target: torch.Tensor):
    """seg_metrics of an episode's adapted logits (with CE) and of its baseline logits0
    (test.py:192,200-204: pred_q0, without CE) against one target, in the same two launches.
    Returns (iut, ce, iut0); equal to two seg_metrics calls."""
    _lib.require(logits, "logits")
    _lib.require(logits0, "logits0")
    _lib.require(target, "target", torch.int64)
    B, nc, h, w = logits.shape
    if nc != 2:
        raise NotImplementedError("2-way episodes only (num_classes_tr = 2)")
    if tuple(logits0.shape) != tuple(logits.shape):
        raise ValueError("logits0 must have the shape of logits")
    S = target.shape[-1]
    lg, lg0, tg = logits.contiguous(), logits0.contiguous(), target.contiguous()
    iut = torch.empty((B, 3, 2), device=lg.device, dtype=torch.float32)
    iut0 = torch.empty_like(iut)
    ce = torch.empty((B, 2), device=lg.device, dtype=torch.float64)
    _lib.check(_lib.lib().cwt_seg_metrics_pair(_lib.ctx(lg.device.index), _lib.ptr(lg), _lib.ptr(lg0), _lib.ptr(tg),
                                               B, h, w, S, _lib.ptr(iut), _lib.ptr(ce), _lib.ptr(iut0),
                                               _lib.stream_ptr(lg.device)),
               "cwt_seg_metrics_pair")
    return iut, ce, iut0


def batch_intersectionAndUnionGPU(logits: torch.Tensor, target: torch.Tensor, num_classes: int,
                                  ignore_index: int = 255):
    """util.py:237-277: logits [n_task, shot, C, h, w], target [n_task, shot, H, W] ->
    (intersection, union, target) each [n_task, shot, C]."""
    assert ignore_index == 255
    n_task, shots, nc, h, w = logits.shape
    iut, _ = seg_metrics(logits.reshape(n_task * shots, nc, h, w), target.reshape(n_task * shots, *target.shape[-2:]),
                         with_ce=False)
    iut = iut.view(n_task, shots, 3, nc)
    return iut[:, :, 0], iut[:, :, 1], iut[:, :, 2]

"""Episode drivers: the build's counterparts of the reference's ``validate_transformer``
(src/test.py:103-254) and ``do_epoch`` (src/train.py:166-288), plus the device-resident
single-episode pipeline they (and bench.py) are built from.

Order of operations per inference episode (test.py:138-219):
  extract_features(support ++ query)   one backbone pass over shot+1 images (batching the
                                       query with the support is exact: eval-mode BN)
  inner_adapt(f_s, s_label, W0)        200 fused SGD steps            (test.py:180-187)
  normalize(f_q) + pred_q0 = W . f_q   one pass                        (test.py:190-194)
  W' = CWT(W, f_hat, f_hat)                                            (test.py:195-197)
  pred_q = W' . f_hat                                                  (test.py:200-204)
  upsample + argmax + IoU + CE         for pred_q and pred_q0          (test.py:214-224)
Everything stays on the device; the host reads back per-episode IoU counts only.
"""
from __future__ import annotations

import ctypes
import os
import time
from collections import defaultdict
from typing import Iterable, Tuple

import numpy as np
import torch

from . import _lib
from . import dist as cdist
from .synthetic import feature_side, make_episode, pascal_val_classes
from .util import AverageMeter, seg_metrics, seg_metrics_pair


def _a(args, k, default=None):
    if isinstance(args, dict):
        return args.get(k, default)
    return getattr(args, k, default)


# --------------------------------------------------------------------------------------
# device primitives
# --------------------------------------------------------------------------------------

def inner_adapt(f_s: torch.Tensor, s_label: torch.Tensor, W: torch.Tensor, lr: float, iters: int) -> torch.Tensor:
    """Support-set inner loop, in place on W [2,512] (test.py:164-187; train.py:206-231).
    f_s [n,512,h,w] channels_last; s_label [n,S,S] int64."""
    _lib.require(f_s, "f_s")
    _lib.require(s_label, "s_label", torch.int64)
    _lib.require(W, "W")
    n, Cc, h, w = f_s.shape
    if not f_s.is_contiguous(memory_format=torch.channels_last):
        f_s = f_s.contiguous(memory_format=torch.channels_last)
    S = s_label.shape[-1]
    lbl = s_label.reshape(n, S, S).contiguous()
    assert W.is_contiguous() and W.numel() == 2 * Cc
    _lib.check(_lib.lib().cwt_inner_adapt(_lib.ctx(W.device.index), _lib.ptr(f_s), _lib.ptr(lbl), n, h, w, Cc, S,
                                          float(lr), int(iters), _lib.ptr(W), _lib.stream_ptr(W.device)),
               "cwt_inner_adapt")
    return W


def inner_adapt_batch(f_s: torch.Tensor, s_label: torch.Tensor, W: torch.Tensor, lr: float, iters: int) -> torch.Tensor:
    """E independent inner loops in the same launches (cwt_inner_adapt_batch), in place on
    W [E,2,512].  f_s [E*n,512,h,w] channels_last (episode-major), s_label [E,n,S,S] or
    [E*n,S,S] int64.  Episode e gets exactly inner_adapt(f_s[e*n:(e+1)*n], s_label[e], W[e])."""
    _lib.require(f_s, "f_s")
    _lib.require(s_label, "s_label", torch.int64)
    _lib.require(W, "W")
    E = W.shape[0]
    En, Cc, h, w = f_s.shape
    if W.shape != (E, 2, Cc) or not W.is_contiguous() or En % E:
        raise ValueError(f"W must be a contiguous [E,2,{Cc}] tensor and f_s hold E*n images")
    n = En // E
    if not f_s.is_contiguous(memory_format=torch.channels_last):
        f_s = f_s.contiguous(memory_format=torch.channels_last)
    S = s_label.shape[-1]
    lbl = s_label.reshape(E * n, S, S).contiguous()
    _lib.check(_lib.lib().cwt_inner_adapt_batch(_lib.ctx(W.device.index), _lib.ptr(f_s), _lib.ptr(lbl), E, n, h, w,
                                                Cc, S, float(lr), int(iters), _lib.ptr(W),
                                                _lib.stream_ptr(W.device)), "cwt_inner_adapt_batch")
    return W


def normalize(f: torch.Tensor, W0: torch.Tensor | None = None):
    """F.normalize(f, dim=1) (+ baseline logits W0 . f). f [B,512,h,w] channels_last."""
    B, Cc, h, w = f.shape
    out = torch.empty_like(f, memory_format=torch.channels_last)
    logits0 = torch.empty((B, 2, h, w), device=f.device, dtype=torch.float32) if W0 is not None else None
    _lib.check(_lib.lib().cwt_normalize(_lib.ctx(f.device.index), _lib.ptr(f), B, h * w, Cc, _lib.ptr(out),
                                        _lib.ptr(W0), _lib.ptr(logits0), _lib.stream_ptr(f.device)), "cwt_normalize")
    return out, logits0


def classify(W: torch.Tensor, f: torch.Tensor) -> torch.Tensor:
    """W [B,2,512] . f [B,512,h,w] (channels_last) -> logits [B,2,h,w]."""
    B, Cc, h, w = f.shape
    logits = torch.empty((B, 2, h, w), device=f.device, dtype=torch.float32)
    W = W.contiguous()  # keep the (possible) copy alive until the call has been enqueued
    _lib.check(_lib.lib().cwt_classify(_lib.ctx(f.device.index), _lib.ptr(W), _lib.ptr(f), B, h * w, Cc,
                                       _lib.ptr(logits), _lib.stream_ptr(f.device)), "cwt_classify")
    return logits


def classify_scaled(W: torch.Tensor, f: torch.Tensor, inv_norm: torch.Tensor) -> torch.Tensor:
    """W [B,2,512] . F.normalize(f) with the normalisation as the per-pixel scale inv_norm [B,hw]
    (cwt_classify_scaled; f the RAW features [B,512,h,w] channels_last) -> logits [B,2,h,w]."""
    B, Cc, h, w = f.shape
    logits = torch.empty((B, 2, h, w), device=f.device, dtype=torch.float32)
    W = W.contiguous()
    _lib.check(_lib.lib().cwt_classify_scaled(_lib.ctx(f.device.index), _lib.ptr(W), _lib.ptr(f),
                                              _lib.ptr(inv_norm), B, h * w, Cc, _lib.ptr(logits),
                                              _lib.stream_ptr(f.device)), "cwt_classify_scaled")
    return logits


def cwt_tail(transformer, Wb: torch.Tensor, f_q: torch.Tensor):
    """test.py:190-204 after the inner loop: pred_q0 = W . f_q, f_hat = F.normalize(f_q),
    W' = CWT(W, f_hat, f_hat), pred_q = W' . f_hat.  4 heads: the fused form (one pass over the
    raw tokens, no normalised copy; cwt_attention_infer + cwt_classify_scaled); otherwise the
    module-by-module kernels.  Returns (W', pred_q, pred_q0).  The fused entry point takes
    d_model 512, at most 16384 tokens and 4 queries per call (cwt_attention_infer); any other
    shape takes the module path, as before it."""
    B, Cc, h, w = f_q.shape
    if transformer.n_head == 4 and transformer.d_model == 512 and Cc == 512 and h * w <= 16384 and B <= 4:
        if not f_q.is_contiguous(memory_format=torch.channels_last):
            f_q = f_q.contiguous(memory_format=torch.channels_last)
        W2, inv, pred_q0 = transformer.infer_raw(Wb, f_q)
        return W2, classify_scaled(W2, f_q, inv), pred_q0
    fqn, pred_q0 = normalize(f_q, Wb)
    W2 = transformer.infer(Wb, fqn)
    return W2, classify(W2, fqn), pred_q0


_FUSED_TAIL = os.environ.get("CWT_FUSED_TAIL", "1") != "0"   # 0: the module kernels (A/B)
# 0: inner loop and tail as two library calls (the library also honours CWT_FUSED_LOOP_TAIL=0)
_FUSED_LOOP_TAIL = os.environ.get("CWT_FUSED_LOOP_TAIL", "1") != "0"


def fused_tail_ok(transformer, f_q: torch.Tensor, S: int) -> bool:
    """The one-launch tail (cwt_episode_tail) takes 4 heads, d_model 512, <= 4 queries of
    <= 16384 tokens and labels of side S with S - 1 == 8 (h - 1) (the extractor's geometry);
    anything else takes the module path (cwt_tail + seg_metrics_pair, any S)."""
    B, Cc, h, w = f_q.shape
    return (_FUSED_TAIL and transformer.n_head == 4 and Cc == 512 and h * w <= 16384 and B <= 4 and h == w
            and S - 1 == 8 * (h - 1))


def episode_tail(transformer, Wb: torch.Tensor, f_q: torch.Tensor, q_label: torch.Tensor):
    """test.py:190-224 after the inner loop in ONE launch (cwt_episode_tail): pred_q0 = W . f_q,
    W' = CWT(W, F.normalize(f_q)), pred_q = W' . F.normalize(f_q), and the metrics of both
    against q_label.  Returns (W', pred_q, pred_q0, iut, ce, iut0) as cwt_tail + seg_metrics_pair
    do (the same function: tests/test_gpu_tail.py)."""
    if not f_q.is_contiguous(memory_format=torch.channels_last):
        f_q = f_q.contiguous(memory_format=torch.channels_last)
    B, Cc, h, w = f_q.shape
    S = q_label.shape[-1]
    t = transformer
    Wb = Wb.contiguous()
    tg = q_label.reshape(B, S, S).contiguous()
    dev = f_q.device
    out = torch.empty((B, 2, Cc), device=dev, dtype=torch.float32)
    logits = torch.empty((B, 2, h, w), device=dev, dtype=torch.float32)
    logits0 = torch.empty_like(logits)
    iut = torch.empty((B, 3, 2), device=dev, dtype=torch.float32)
    iut0 = torch.empty_like(iut)
    ce = torch.empty((B, 2), device=dev, dtype=torch.float64)
    wq, fw, fb, lw, lb = t._ptrs(t.flat)
    _lib.check(_lib.lib().cwt_episode_tail(_lib.ctx(dev.index), _lib.ptr(Wb), _lib.ptr(f_q), B, h, w, S, _lib.ptr(tg),
                                           wq, fw, fb, lw, lb, t.params_version(), _lib.ptr(out), _lib.ptr(logits),
                                           _lib.ptr(logits0), _lib.ptr(iut), _lib.ptr(ce), _lib.ptr(iut0),
                                           _lib.stream_ptr(dev)), "cwt_episode_tail")
    return out, logits, logits0, iut, ce, iut0


def tail_and_metrics(transformer, Wb: torch.Tensor, f_q: torch.Tensor, q_label: torch.Tensor):
    """(W', pred_q, pred_q0, iut, ce, iut0) of an episode group (B <= 4): the one-launch tail
    where it applies, else cwt_tail + seg_metrics_pair."""
    if fused_tail_ok(transformer, f_q, q_label.shape[-1]):
        return episode_tail(transformer, Wb, f_q, q_label)
    W2, pred_q, pred_q0 = cwt_tail(transformer, Wb, f_q)
    iut, ce, iut0 = seg_metrics_pair(pred_q, pred_q0, q_label)
    return W2, pred_q, pred_q0, iut, ce, iut0


def adapt_and_tail(transformer, f_s: torch.Tensor, s_label: torch.Tensor, W: torch.Tensor, lr: float, iters: int,
                   f_q: torch.Tensor, q_label: torch.Tensor):
    """inner_adapt(f_s, s_label, W) then tail_and_metrics(W, f_q, q_label) for one episode with
    one query -- as ONE call (cwt_inner_adapt_tail) where the one-launch tail applies: on the
    pipeline's adapt context the library fuses the tail behind the loop's last step in the same
    launch.  Returns (W, (W', pred_q, pred_q0, iut, ce, iut0))."""
    if f_q.shape[0] != 1 or not fused_tail_ok(transformer, f_q, q_label.shape[-1]) or not _FUSED_LOOP_TAIL:
        W = inner_adapt(f_s, s_label, W, lr, iters)
        return W, tail_and_metrics(transformer, W.view(1, 2, -1), f_q, q_label)
    _lib.require(f_s, "f_s")
    _lib.require(s_label, "s_label", torch.int64)
    _lib.require(W, "W")
    n, Cc, h, w = f_s.shape
    if not f_s.is_contiguous(memory_format=torch.channels_last):
        f_s = f_s.contiguous(memory_format=torch.channels_last)
    if not f_q.is_contiguous(memory_format=torch.channels_last):
        f_q = f_q.contiguous(memory_format=torch.channels_last)
    if f_q.shape[2:] != f_s.shape[2:]:
        raise ValueError("f_q and f_s must share h, w")
    S = s_label.shape[-1]
    lbl = s_label.reshape(n, S, S).contiguous()
    tg = q_label.reshape(1, S, S).contiguous()
    assert W.is_contiguous() and W.numel() == 2 * Cc
    dev = f_q.device
    out = torch.empty((1, 2, Cc), device=dev, dtype=torch.float32)
    logits = torch.empty((1, 2, h, w), device=dev, dtype=torch.float32)
    logits0 = torch.empty_like(logits)
    iut = torch.empty((1, 3, 2), device=dev, dtype=torch.float32)
    iut0 = torch.empty_like(iut)
    ce = torch.empty((1, 2), device=dev, dtype=torch.float64)
    t = transformer
    wq, fw, fb, lw, lb = t._ptrs(t.flat)
    _lib.check(_lib.lib().cwt_inner_adapt_tail(
        _lib.ctx(dev.index), _lib.ptr(f_s), _lib.ptr(lbl), n, h, w, Cc, S, float(lr), int(iters), _lib.ptr(W),
        _lib.ptr(f_q), _lib.ptr(tg), wq, fw, fb, lw, lb, t.params_version(), _lib.ptr(out), _lib.ptr(logits),
        _lib.ptr(logits0), _lib.ptr(iut), _lib.ptr(ce), _lib.ptr(iut0), _lib.stream_ptr(dev)), "cwt_inner_adapt_tail")
    return W, (out, logits, logits0, iut, ce, iut0)


def classify_bwd(dlogits: torch.Tensor, f: torch.Tensor, dW: torch.Tensor):
    B, Cc, h, w = f.shape
    dlogits = dlogits.contiguous()
    _lib.check(_lib.lib().cwt_classify_bwd(_lib.ctx(f.device.index), _lib.ptr(dlogits), _lib.ptr(f), B,
                                           h * w, Cc, _lib.ptr(dW), _lib.stream_ptr(f.device)), "cwt_classify_bwd")
    return dW


def seg_ce_fwd_bwd(logits: torch.Tensor, target: torch.Tensor):
    """Query CE with class weight [1, #bg/(#fg+1e-12)] (train.py:237-243,261-265):
    returns (loss [1] device, dlogits [B,2,h,w])."""
    B, _, h, w = logits.shape
    S = target.shape[-1]
    loss = torch.empty(1, device=logits.device, dtype=torch.float32)
    logits, target = logits.contiguous(), target.contiguous()
    dl = torch.empty_like(logits)
    _lib.check(_lib.lib().cwt_seg_ce_fwd_bwd(_lib.ctx(logits.device.index), _lib.ptr(logits),
                                             _lib.ptr(target), B, h, w, S, _lib.ptr(loss), _lib.ptr(dl),
                                             _lib.stream_ptr(logits.device)), "cwt_seg_ce_fwd_bwd")
    return loss, dl


class EpisodeEngine:
    """Device-resident CWT inference episode (batch_size_val = 1), no host syncs."""

    def __init__(self, model, transformer, args):
        self.model, self.transformer = model, transformer
        self.S = int(_a(args, "image_size", 473))
        self.h = feature_side(self.S)
        self.shot = int(_a(args, "shot", 1))
        self.lr = float(_a(args, "cls_lr", 0.1))
        self.iters = int(_a(args, "adapt_iter", 200))

    @torch.no_grad()
    def run(self, imgs: torch.Tensor, s_label: torch.Tensor, q_label: torch.Tensor, W0: torch.Tensor) -> dict:
        """imgs [shot+1,3,S,S] (supports then query), s_label [shot,S,S], q_label [1,S,S] int64,
        W0 [2,512] (consumed: adapted in place)."""
        shot = imgs.shape[0] - 1
        f_all, _ = self.model.extract_features(imgs)
        f_s, f_q = f_all[:shot], f_all[shot:]
        W = inner_adapt(f_s, s_label, W0, self.lr, self.iters)
        Wb = W.view(1, 2, -1)
        W2, pred_q, pred_q0, iut, ce, iut0 = tail_and_metrics(self.transformer, Wb, f_q, q_label)
        return dict(W=W, W2=W2, pred_q=pred_q, pred_q0=pred_q0, iut=iut, iut0=iut0, ce=ce, f_s=f_s, f_q=f_q)

    @torch.no_grad()
    def run_batch(self, imgs: torch.Tensor, s_label: torch.Tensor, q_label: torch.Tensor, W0: torch.Tensor) -> dict:
        """E independent episodes in flight at once (throughput form of ``run``; each
        episode's outputs are those ``run`` gives it alone: eval-mode BN makes the shared
        backbone pass exact, and the inner loops keep per-episode W, class weights and
        accumulators).  imgs [E*shot + E,3,S,S] = the E*shot supports (episode-major) then the
        E queries; s_label [E,shot,S,S]; q_label [E,S,S] int64; W0 [E,2,512] (adapted in
        place).  E <= 16; the CWT runs in groups of 4 episodes (its kernels' batch limit)."""
        E = W0.shape[0]
        shot = s_label.shape[1]
        if imgs.shape[0] != E * (shot + 1) or E > 16:
            raise ValueError("imgs must hold E*shot supports then E queries, E <= 16")
        f_all, _ = self.model.extract_features(imgs)
        f_s, f_q = f_all[:E * shot], f_all[E * shot:]
        W = inner_adapt_batch(f_s, s_label, W0, self.lr, self.iters)
        parts = [tail_and_metrics(self.transformer, W[i:i + 4], f_q[i:i + 4], q_label[i:i + 4]) for i in range(0, E, 4)]
        W2, pred_q, pred_q0, iut, ce, iut0 = (torch.cat([p[j] for p in parts]) for j in range(6))
        return dict(W=W, W2=W2, pred_q=pred_q, pred_q0=pred_q0, iut=iut, iut0=iut0, ce=ce, f_s=f_s, f_q=f_q)


class EpisodePipeline:
    """Consecutive independent episodes on two HIP streams: the extractor pass of episode i+1
    runs while episode i's inner loop (one persistent launch on ~118 of the 256 CUs, the rest
    idle) and its CWT / classifier / metrics run.  Every episode executes exactly the kernels
    ``EpisodeEngine.run`` launches, with the same inputs, so its outputs are the same (up to the
    fp32 rounding of the inner loop's per-workgroup partial sums, which depends on how many units a
    workgroup holds; the exchange itself is exact); only their placement in time changes.  Each
    episode is still processed alone (batch_size_val = 1): nothing is batched across episodes.

    Stream use: the extractor's workspaces are only touched by the extract stream, the inner
    loop's / CWT's by the adapt stream.  ``submit`` returns the episode's result tensors, valid
    on the adapt stream (``wait`` makes the current stream wait for them)."""

    _shared = {}   # (device, extract_streams) -> the process's pipeline (streams + contexts reused)

    @classmethod
    def shared(cls, engine: "EpisodeEngine", extract_streams: int = 1) -> "EpisodePipeline":
        """The pipeline of this device and stream count, created once per process and reused by
        every later caller (validate_transformer runs every epoch: a pipeline per call would
        leave its libcwt contexts and their workspaces behind each time)."""
        key = (torch.cuda.current_device(), max(1, int(extract_streams)))
        p = cls._shared.get(key)
        if p is None or p.closed:
            p = cls._shared[key] = cls(engine, extract_streams)
        p.eng = engine
        return p

    def __init__(self, engine: "EpisodeEngine", extract_streams: int = 1):
        """extract_streams > 1: consecutive episodes' extractor passes also overlap each other,
        round-robin over that many streams, each with its own libcwt context (workspaces)."""
        self.closed = False
        self.device = torch.cuda.current_device()
        self.eng = engine
        self.s_ext = [torch.cuda.Stream() for _ in range(max(1, int(extract_streams)))]
        self.c_ext = [None] + [_lib.new_ctx() for _ in range(len(self.s_ext) - 1)]
        self.s_extract = self.s_ext[0]
        # the adapt stream at high priority: its loop's grid is dispatched ahead of the extractor
        # pass's pending workgroups.  Rounds 2 and 5 measured no difference; round 6 (the fused
        # tail) 5 of 6 interleaved pairs higher, +0.9 % on average (profiles/r6/studies/adapt_prio/).
        # CWT_PIPE_ADAPT_PRIO=0 turns it off (A/B)
        prio = -1 if os.environ.get("CWT_PIPE_ADAPT_PRIO", "1") == "1" else 0
        self.s_adapt = torch.cuda.Stream(priority=prio)
        # the adapt stream's own context: its persistent inner loop holds two units per
        # workgroup (59 instead of 118 CUs at 1-shot 473^2), leaving the rest to the extractor
        # passes beside it -- 466 against 443 episodes/s (same session); results are unchanged
        self.c_adapt = _lib.new_ctx()
        upw = int(os.environ.get("CWT_PIPE_ADAPT_UNITS", "2"))   # (1, 2 or 3: A/B of the geometry)
        _lib.check(_lib.lib().cwt_ctx_set_adapt_units(self.c_adapt, upw), "cwt_ctx_set_adapt_units")
        self.k = 0
        # drain: submit(..., last=True) (the caller knows no episode follows before it reads the
        # results back) runs that episode's inner loop and tail on a context with the automatic
        # geometry (one unit per workgroup at 1-shot 473^2: 118 CUs, 1.05 instead of 1.4 ms), since
        # no extractor pass runs beside it any more.  Same kernels, same inputs, same results.
        # CWT_PIPE_DRAIN=0 turns it off (A/B).
        self.drain = os.environ.get("CWT_PIPE_DRAIN", "1") != "0"
        self.c_solo = None
        # Opt-in (CWT_PIPE_DRAIN_OVERLAP=1): that loop on a stream of its own beside the previous
        # episode's loop and tail (instead of after them) whenever the two persistent grids fit on
        # the chip together (1-shot 473^2: 59 + 118 of 256 CUs; not 5-shot: 197 + 197), its tail
        # then following on the adapt stream.  Measured no faster at the driver's 20 steps
        # (470.5 vs 472.2 episodes/s, 3 interleaved pairs, profiles/r4/run_r), so off.
        self.drain_overlap = os.environ.get("CWT_PIPE_DRAIN_OVERLAP", "0") == "1"
        self.s_drain = None
        self._fits = {}

    def _drain_fits(self, shot: int, h: int, w: int, iters: int) -> bool:
        key = (shot, h, w, iters)
        if key not in self._fits:
            gs = []
            for c in (self.c_adapt, self.c_solo):
                g = ctypes.c_int(0)
                _lib.check(_lib.lib().cwt_adapt_workgroups(c, 1, shot, h, w, iters, ctypes.byref(g)),
                           "cwt_adapt_workgroups")
                gs.append(g.value)
            # the previous episode's tail may run beside the drain loop as well: nothing extra where
            # the adapt context fuses it into its loop's own workgroups (cwt_inner_adapt_tail), else a
            # 64-workgroup co-resident grid (cwt_episode_tail)
            fz = ctypes.c_int(0)
            _lib.check(_lib.lib().cwt_adapt_fuses_tail(self.c_adapt, shot, h, w, iters, ctypes.byref(fz)),
                       "cwt_adapt_fuses_tail")
            tail_g = 0 if fz.value else min(64, _lib.cu_count(self.device))
            self._fits[key] = min(gs) > 0 and sum(gs) + tail_g <= _lib.cu_count(self.device)
        return self._fits[key]

    @torch.no_grad()
    def submit(self, imgs: torch.Tensor, s_label: torch.Tensor, q_label: torch.Tensor, W0: torch.Tensor,
               last: bool = False) -> dict:
        """Queue one episode; last=True: no episode follows before the caller reads the results
        (its inner loop then takes the whole-chip geometry; the results are the same)."""
        eng = self.eng
        cur = torch.cuda.current_stream()
        shot = imgs.shape[0] - 1
        i = self.k % len(self.s_ext)
        self.k += 1
        s_ex = self.s_ext[i]
        s_ex.wait_stream(cur)   # inputs were produced on the caller's stream
        self.s_adapt.wait_stream(cur)
        with torch.cuda.stream(s_ex):
            if self.c_ext[i] is None:
                f_all, _ = eng.model.extract_features(imgs)
            else:
                with _lib.using_ctx(self.c_ext[i]):
                    f_all, _ = eng.model.extract_features(imgs)
            done = torch.cuda.Event()
            done.record(s_ex)
        c_ad = self.c_adapt
        if last and self.drain:
            if self.c_solo is None:
                self.c_solo = _lib.new_ctx()   # automatic geometry (cwt_ctx_set_adapt_units 0)
            c_ad = self.c_solo
            if self.drain_overlap and self._drain_fits(shot, f_all.shape[2], f_all.shape[3], eng.iters):
                if self.s_drain is None:
                    self.s_drain = torch.cuda.Stream()
                self.s_drain.wait_stream(cur)
                with torch.cuda.stream(self.s_drain), _lib.using_ctx(self.c_solo):
                    self.s_drain.wait_event(done)
                    for t in (f_all, imgs, s_label, q_label, W0):
                        t.record_stream(self.s_drain)
                    W = inner_adapt(f_all[:shot], s_label, W0, eng.lr, eng.iters)
                    looped = torch.cuda.Event()
                    looped.record(self.s_drain)
                with torch.cuda.stream(self.s_adapt), _lib.using_ctx(self.c_adapt):
                    self.s_adapt.wait_event(looped)
                    for t in (f_all, q_label, W):
                        t.record_stream(self.s_adapt)
                    W2, pred_q, pred_q0, iut, ce, iut0 = tail_and_metrics(eng.transformer, W.view(1, 2, -1),
                                                                          f_all[shot:], q_label)
                    done_all = torch.cuda.Event()
                    done_all.record(self.s_adapt)
                return dict(W=W, W2=W2, pred_q=pred_q, pred_q0=pred_q0, iut=iut, iut0=iut0, ce=ce, done=done_all)
        if c_ad is self.c_solo and self.s_drain is not None:
            self.s_adapt.wait_stream(self.s_drain)     # c_solo's workspaces: one stream at a time
        with torch.cuda.stream(self.s_adapt), _lib.using_ctx(c_ad):
            self.s_adapt.wait_event(done)
            for t in (f_all, imgs, s_label, q_label, W0):
                t.record_stream(self.s_adapt)
            f_s, f_q = f_all[:shot], f_all[shot:]
            W, (W2, pred_q, pred_q0, iut, ce, iut0) = adapt_and_tail(eng.transformer, f_s, s_label, W0, eng.lr,
                                                                      eng.iters, f_q, q_label)
            done_all = torch.cuda.Event()
            done_all.record(self.s_adapt)
        return dict(W=W, W2=W2, pred_q=pred_q, pred_q0=pred_q0, iut=iut, iut0=iut0, ce=ce, done=done_all)

    @torch.no_grad()
    def submit_batch(self, imgs: torch.Tensor, s_label: torch.Tensor, q_label: torch.Tensor, W0: torch.Tensor,
                     last: bool = False) -> dict:
        """Queue E independent episodes that share ONE extractor pass (``EpisodeEngine.run_batch``
        in the pipeline): imgs [E*shot + E,3,S,S] (the supports episode-major, then the queries),
        s_label [E,shot,S,S], q_label [E,S,S], W0 [E,2,512] (adapted in place).  Eval-mode BN makes
        the shared pass exact, the E inner loops run in one persistent launch with per-episode W,
        class weights and accumulators, the tails in groups of 4: every episode's outputs are the
        ones ``run`` gives it alone (tests/test_gpu_batch.py).  A throughput form (bigger conv GEMMs,
        M = E*(shot+1)*h*w), reported beside the one-episode pipeline, not in place of it."""
        eng = self.eng
        cur = torch.cuda.current_stream()
        E = W0.shape[0]
        shot = s_label.shape[1]
        if imgs.shape[0] != E * (shot + 1) or E > 16:
            raise ValueError("imgs must hold E*shot supports then E queries, E <= 16")
        i = self.k % len(self.s_ext)
        self.k += 1
        s_ex = self.s_ext[i]
        s_ex.wait_stream(cur)
        self.s_adapt.wait_stream(cur)
        with torch.cuda.stream(s_ex):
            if self.c_ext[i] is None:
                f_all, _ = eng.model.extract_features(imgs)
            else:
                with _lib.using_ctx(self.c_ext[i]):
                    f_all, _ = eng.model.extract_features(imgs)
            done = torch.cuda.Event()
            done.record(s_ex)
        c_ad = self.c_adapt
        if last and self.drain:
            if self.c_solo is None:
                self.c_solo = _lib.new_ctx()
            c_ad = self.c_solo
        if c_ad is self.c_solo and self.s_drain is not None:
            self.s_adapt.wait_stream(self.s_drain)     # c_solo's workspaces: one stream at a time
        with torch.cuda.stream(self.s_adapt), _lib.using_ctx(c_ad):
            self.s_adapt.wait_event(done)
            for t in (f_all, imgs, s_label, q_label, W0):
                t.record_stream(self.s_adapt)
            f_s, f_q = f_all[:E * shot], f_all[E * shot:]
            W = inner_adapt_batch(f_s, s_label, W0, eng.lr, eng.iters)
            parts = [tail_and_metrics(eng.transformer, W[j:j + 4], f_q[j:j + 4], q_label[j:j + 4])
                     for j in range(0, E, 4)]
            W2, pred_q, pred_q0, iut, ce, iut0 = (torch.cat([p[j] for p in parts]) for j in range(6))
            done_all = torch.cuda.Event()
            done_all.record(self.s_adapt)
        return dict(W=W, W2=W2, pred_q=pred_q, pred_q0=pred_q0, iut=iut, iut0=iut0, ce=ce, done=done_all)

    def submit_train(self, tengine: "TrainEngine", imgs: torch.Tensor, s_label: torch.Tensor, q_label: torch.Tensor,
                     W0: torch.Tensor, after=None) -> dict:
        """A training episode (train.py:188-267): the extractor pass on an extractor stream, then
        on the adapt stream the inner loop, CWT forward, query CE and the CWT backward into
        transformer.flat.grad, then ``after()`` (the caller's gradient all-reduce and optimiser
        step) -- so the CWT parameter updates stay in episode order while the next episode's
        extractor pass and inner loop (which do not read them) already run."""
        cur = torch.cuda.current_stream()
        shot = imgs.shape[0] - 1
        i = self.k % len(self.s_ext)
        self.k += 1
        s_ex = self.s_ext[i]
        s_ex.wait_stream(cur)
        self.s_adapt.wait_stream(cur)
        with torch.no_grad(), torch.cuda.stream(s_ex):
            if self.c_ext[i] is None:
                f_all, _ = tengine.model.extract_features(imgs)
            else:
                with _lib.using_ctx(self.c_ext[i]):
                    f_all, _ = tengine.model.extract_features(imgs)
            done = torch.cuda.Event()
            done.record(s_ex)
        with torch.cuda.stream(self.s_adapt), _lib.using_ctx(self.c_adapt):
            self.s_adapt.wait_event(done)
            for t in (f_all, imgs, s_label, q_label, W0):
                t.record_stream(self.s_adapt)
            r = tengine.step_from_features(f_all[:shot], f_all[shot:], s_label, q_label, W0)
            if after is not None:
                after()
        return r

    def wait(self):
        """Make the caller's current stream wait for everything submitted so far."""
        cur = torch.cuda.current_stream()
        for s in self.s_ext:
            cur.wait_stream(s)
        if self.s_drain is not None:
            cur.wait_stream(self.s_drain)
        cur.wait_stream(self.s_adapt)

    def close(self):
        """Synchronise the pipeline's streams and destroy its libcwt contexts."""
        if self.closed:
            return
        for s in self.s_ext + [self.s_adapt] + ([self.s_drain] if self.s_drain is not None else []):
            s.synchronize()
        for c in [c for c in self.c_ext if c is not None] + [self.c_adapt] + ([self.c_solo] if self.c_solo else []):
            _lib.destroy_ctx(c, self.device)
        self.closed = True
        for k, v in list(EpisodePipeline._shared.items()):
            if v is self:
                del EpisodePipeline._shared[k]


class TrainEngine:
    """Device-resident CWT training episode (train.py:188-267 without the host-side batch
    transfer): the backbone and inner loop as in inference, then CWT forward with saved
    state, classifier, query CE forward/backward, classifier and CWT backward; gradients
    ACCUMULATE into transformer.flat.grad.  The all-reduce and the optimiser step are the
    caller's (do_epoch, bench.py --train)."""

    def __init__(self, model, transformer, args):
        self.model, self.transformer = model, transformer
        self.lr = float(_a(args, "cls_lr", 0.1))
        self.iters = int(_a(args, "adapt_iter", 200))

    def step(self, imgs: torch.Tensor, s_label: torch.Tensor, q_label: torch.Tensor, W0: torch.Tensor) -> dict:
        shot = imgs.shape[0] - 1
        with torch.no_grad():
            f_all, _ = self.model.extract_features(imgs)
        return self.step_from_features(f_all[:shot], f_all[shot:], s_label, q_label, W0)

    def step_from_features(self, f_s: torch.Tensor, f_q: torch.Tensor, s_label: torch.Tensor, q_label: torch.Tensor,
                           W0: torch.Tensor) -> dict:
        t = self.transformer
        if t.flat.grad is None:
            t.flat.grad = torch.zeros_like(t.flat)
        with torch.no_grad():
            W = inner_adapt(f_s, s_label, W0, self.lr, self.iters)
            Wb = W.view(1, 2, -1)
            fqn, pred_q0 = normalize(f_q, Wb)
            W2, state = t.forward_train(Wb, fqn)
            pred_q = classify(W2, fqn)
            loss, dl = seg_ce_fwd_bwd(pred_q, q_label)
            dW2 = torch.zeros_like(W2)
            classify_bwd(dl, fqn, dW2)
            t.backward_into(state, dW2)
        return dict(loss=loss, W=W, W2=W2, pred_q=pred_q, pred_q0=pred_q0)


def new_binary_classifier_weight(bottleneck_dim: int = 512, num_classes: int = 2) -> torch.Tensor:
    """W0 exactly as the reference draws it: nn.Conv2d(512, 2, 1, bias=False) constructed on the
    host from the global torch RNG (test.py:164; train.py:206), returned as [2,512]."""
    conv = torch.nn.Conv2d(bottleneck_dim, num_classes, kernel_size=1, bias=False)
    return conv.weight.detach().reshape(num_classes, bottleneck_dim).clone()


def _class_weight_check(s_label: torch.Tensor):
    # test.py:169-175: len(back_pix) / len(target_pix) raises ZeroDivisionError without FG
    # (host labels from the synthetic loader, device labels from dataset.EpisodicData)
    nf = int((s_label == 1).sum().item())
    nb = int((s_label == 0).sum().item())
    return nb / nf


# --------------------------------------------------------------------------------------
# loaders
# --------------------------------------------------------------------------------------

class SyntheticEpisodes:
    """Episode loader yielding the reference 7-tuple (dataset.py:326-327) as CPU tensors;
    its iterator has ``.next()`` like the torch-1.6 DataLoader iterators the reference uses."""

    def __init__(self, n: int, S: int = 473, shot: int = 1, seed: int = 2021, start: int = 0, classes=None,
                 stride: int = 1):
        self.n, self.S, self.shot, self.seed, self.start, self.classes, self.stride = n, S, shot, seed, start, \
            classes or pascal_val_classes(0), stride

    def __len__(self):
        return self.n

    def shard(self, rank: int, world: int) -> "SyntheticEpisodes":
        """This rank's share of the episode stream (episodes start + (rank + i*world)*stride):
        disjoint across ranks, like the DistributedSampler shard of the real loader."""
        return SyntheticEpisodes(self.n, self.S, self.shot, self.seed, self.start + rank * self.stride, self.classes,
                                 self.stride * world)

    def episode(self, i: int):
        ep = make_episode(self.seed, self.start + i * self.stride, self.S, self.shot, self.classes)
        t = torch.from_numpy
        return (t(ep["qry_img"]), t(ep["q_label"]), t(ep["spprt_imgs"]), t(ep["s_label"]),
                [torch.tensor([c]) for c in ep["subcls"]], "", "")

    def __iter__(self):
        outer = self

        class _It:
            def __init__(self):
                self.i = 0

            def next(self):
                r = outer.episode(self.i % outer.n)
                self.i += 1
                return r

            __next__ = next

        return _It()


# --------------------------------------------------------------------------------------
# validate_transformer (test.py:103-254)
# --------------------------------------------------------------------------------------

def validate_transformer(args, val_loader, model, transformer, episodes_out: list | None = None) -> Tuple[float, float]:
    """Mirror of the reference's validate_transformer for batch_size_val = 1.  Returns
    (mean mIoU over runs, mean loss).  With torch.distributed initialised, rank r runs the
    episodes e with e % world == r and the per-class intersection/union sums are all-reduced
    once at the end of each run.  Episodes run through an
    EpisodePipeline (``args.pipeline`` extractor streams, default 2; 0 = strictly one after the
    other); each is still computed alone and read back in order.  The runtime printed is the
    run's wall time (test.py:252 sums per-episode times, which overlap here)."""
    if int(_a(args, "batch_size_val", 1)) != 1:
        raise NotImplementedError("batch_size_val must be 1 (scripts/test.sh)")
    model.eval()
    transformer.eval()
    dev = torch.device("cuda", torch.cuda.current_device())
    engine = EpisodeEngine(model, transformer, args)
    nb_episodes = int(_a(args, "test_num", 1000))
    n_runs = int(_a(args, "n_runs", 1))
    rank, world = cdist.rank_world()
    runtimes = np.zeros(n_runs)
    val_IoUs = np.zeros(n_runs)
    val_losses = np.zeros(n_runs)
    it = iter(val_loader)
    # EpisodePipeline (args.pipeline extractor streams, 0 = one episode after the other): the
    # next episode is submitted before this one's results are read back (same results, same
    # accumulation order)
    n_pipe = int(_a(args, "pipeline", 2))
    pipe = EpisodePipeline.shared(engine, extract_streams=n_pipe) if n_pipe > 0 else None
    for run in range(n_runs):
        loss_meter = AverageMeter()
        t_run = time.time()
        cls_iu = defaultdict(lambda: np.zeros(2))
        cls_iu0 = defaultdict(lambda: np.zeros(2))
        pending = []

        def finish(r, subcls):
            if "done" in r:
                torch.cuda.current_stream().wait_event(r["done"])
            iut = r["iut"].cpu().numpy()[0]
            iut0 = r["iut0"].cpu().numpy()[0]
            ce = r["ce"].cpu().numpy()[0]
            _lib.check_status()     # the readback synchronised: surface an inner-loop barrier timeout
            # CE mean over the non-ignored pixels; a query with every pixel 255 gives NaN, as
            # CrossEntropyLoss(ignore_index=255) does in the reference (test.py:222-224)
            loss_meter.update(float(ce[0] / ce[1]) if ce[1] > 0 else float("nan"))
            for c in [int(x.item()) for x in subcls]:
                cls_iu[c] += (iut[0, 1], iut[1, 1])       # FG only (test.py:227-228)
                cls_iu0[c] += (iut0[0, 1], iut0[1, 1])
            if episodes_out is not None:
                episodes_out.append({k: (v.detach().cpu() if isinstance(v, torch.Tensor) else v)
                                     for k, v in r.items() if k not in ("f_s", "f_q", "done")})

        for e in range(nb_episodes):
            qry_img, q_label, spprt_imgs, s_label, subcls, _, _ = it.next() if hasattr(it, "next") else next(it)
            W0 = new_binary_classifier_weight()          # consumes the torch RNG like test.py:164
            new_binary_classifier_weight()               # ... and like Pseudo_cls (test.py:200)
            if e % world != rank:
                continue
            _class_weight_check(s_label)
            imgs = torch.cat([spprt_imgs[0], qry_img], 0).to(dev, non_blocking=True)
            sl = s_label[0].to(dev, non_blocking=True)
            ql = q_label.to(dev, non_blocking=True)
            last = e + world >= nb_episodes   # this rank's last episode of the run
            r = (pipe.submit(imgs, sl, ql, W0.to(dev), last=last) if pipe is not None
                 else engine.run(imgs, sl, ql, W0.to(dev)))
            pending.append((r, subcls))
            if len(pending) > (1 if pipe is not None else 0):
                finish(*pending.pop(0))
        while pending:
            finish(*pending.pop(0))
        runtime = time.time() - t_run
        classes = sorted(set(cls_iu) | set(cls_iu0))
        if world > 1:
            classes = cdist.union_keys(classes)
            table = np.array([[*cls_iu[c], *cls_iu0[c]] for c in classes], dtype=np.float64)
            table = cdist.all_reduce_sum_np(table)
            for c, row in zip(classes, table):
                cls_iu[c] = row[:2]
                cls_iu0[c] = row[2:]
            tot = cdist.all_reduce_sum_np(np.array([loss_meter.sum, loss_meter.count], dtype=np.float64))
            loss_meter.sum, loss_meter.count = float(tot[0]), int(tot[1])
            loss_meter.avg = loss_meter.sum / max(loss_meter.count, 1)
        IoU = {c: cls_iu[c][0] / (cls_iu[c][1] + 1e-10) for c in classes}
        mIoU = float(np.mean(list(IoU.values()))) if IoU else 0.0
        if rank == 0:
            print("mIoU---Val result: mIoU {:.4f}.".format(mIoU))
            for c in classes:
                print("Class {} : {:.4f}".format(c, IoU[c]))
        runtimes[run] = runtime
        val_IoUs[run] = mIoU
        val_losses[run] = loss_meter.avg
    if rank == 0:
        print("Average mIoU over {} runs --- {:.4f}.".format(n_runs, val_IoUs.mean()))
        print("Average runtime / run --- {:.4f}.".format(runtimes.mean()))
    return float(val_IoUs.mean()), float(val_losses.mean())


# --------------------------------------------------------------------------------------
# do_epoch (train.py:166-288)
# --------------------------------------------------------------------------------------

def train_episode(model, transformer, args, batch, W0: torch.Tensor, dev) -> dict:
    """Forward/backward of one training episode (train.py:188-267) without the optimiser
    step; gradients are ACCUMULATED into transformer.flat.grad.  CWT dropouts follow
    transformer.training.  In eval mode the 1-shot support is not duplicated: the reference's
    two identical copies (train.py:199-201) give exactly the same inner-loop loss and gradient
    as one, and support + query share one extractor pass.  With the model in train mode (the
    first episode of an epoch, train.py:184) the support pass runs train-mode BN over the
    duplicated batch (batch statistics of both copies, Dropout2d masks differ per copy), then
    model.eval() (train.py:245) and the query pass sees the updated running statistics."""
    qry_img, q_label, spprt_imgs, s_label, subcls = batch[:5]
    S = int(_a(args, "image_size", 473))
    shot = spprt_imgs.shape[1]
    _class_weight_check(s_label)
    sl = s_label[0].to(dev, non_blocking=True).long()
    ql = q_label.to(dev, non_blocking=True).long()
    if getattr(model, "training", False):
        sp = spprt_imgs[0].to(dev, non_blocking=True)
        if shot == 1:
            sp = sp.expand(2, -1, -1, -1)
            sl = sl.expand(2, -1, -1)
        f_s, _ = model.extract_features(sp.contiguous())
        model.eval()
        if cdist.rank_world()[1] > 1:
            # every rank moved its own running statistics; take rank 0's before the query pass
            # so all replicas extract identical features from here on (dist.broadcast_backbone_bn_)
            cdist.broadcast_backbone_bn_(model)
        f_q, _ = model.extract_features(qry_img.to(dev, non_blocking=True))
        sl = sl.contiguous()
    else:
        imgs = torch.cat([spprt_imgs[0], qry_img], 0).to(dev, non_blocking=True)
        f_all, _ = model.extract_features(imgs)
        f_s, f_q = f_all[:shot], f_all[shot:]
    W = inner_adapt(f_s, sl, W0.to(dev), float(_a(args, "cls_lr", 0.1)), int(_a(args, "adapt_iter", 200)))
    Wb = W.view(1, 2, -1)
    fqn, pred_q0 = normalize(f_q, Wb)
    W2, state = transformer.forward_train(Wb, fqn)
    pred_q = classify(W2, fqn)
    loss, dl = seg_ce_fwd_bwd(pred_q, ql)
    dW2 = torch.zeros_like(W2)
    classify_bwd(dl, fqn, dW2)
    transformer.backward_into(state, dW2)
    iut, _ = seg_metrics(pred_q, ql, with_ce=False)
    iut0, _ = seg_metrics(pred_q0, ql, with_ce=False)
    return dict(loss=loss, W=W, W2=W2, pred_q=pred_q, pred_q0=pred_q0, iut=iut, iut0=iut0)


def do_epoch(args, train_loader, model, transformer, optimizer_trans, epoch: int, iter_per_epoch: int,
             log_iter: int, records: list | None = None):
    """Mirror of train.py:166-288 (batch_size 1).  With torch.distributed initialised each
    rank runs its own episode per iteration -- ``train_loader`` must then be this rank's shard
    (``get_train_loader`` returns one; ``SyntheticEpisodes.shard``) and the host RNGs seeded per
    rank (``dist.seed_everything``), so ranks draw different episodes and W0 -- the parameters
    are broadcast from rank 0 once at the start, and the CWT gradient bucket is all-reduced
    (mean) before the identical SGD step on every rank."""
    if int(_a(args, "batch_size", 1)) != 1:
        raise NotImplementedError("batch_size must be 1 (scripts/train.sh)")
    # (the HIP calls in train_episode raise without a device; the loop itself is host logic)
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    loss_meter = AverageMeter()
    train_losses = torch.zeros(log_iter)
    train_Ious = torch.zeros(log_iter)
    train_Ious0 = torch.zeros(log_iter)
    it = iter(train_loader)
    model.train()
    transformer.train()
    rank, world = cdist.rank_world()
    if world > 1:   # identical starting parameters on every rank (DDP's construction-time broadcast)
        cdist.broadcast_params_(transformer.flat)
    for i in range(iter_per_epoch):
        batch = it.next() if hasattr(it, "next") else next(it)
        W0 = new_binary_classifier_weight()              # train.py:206
        optimizer_trans.zero_grad()
        if transformer.flat.grad is None:    # torch optimisers zero_grad to None
            transformer.flat.grad = torch.zeros_like(transformer.flat)
        r = train_episode(model, transformer, args, batch, W0, dev)
        if world > 1:
            cdist.all_reduce_mean_(transformer.flat.grad)
        optimizer_trans.step()
        loss = float(r["loss"].item())
        if dev.type == "cuda":
            _lib.check_status()     # after the .item() sync: surface an inner-loop barrier timeout
        iut = r["iut"].cpu().numpy()[0]
        iut0 = r["iut0"].cpu().numpy()[0]
        IoUb, IoUf = iut[0] / (iut[1] + 1e-10)
        IoUb0, IoUf0 = iut0[0] / (iut0[1] + 1e-10)
        loss_meter.update(loss / 1)
        train_losses[i] = loss_meter.avg
        train_Ious[i] = float((IoUb + IoUf) / 2)
        train_Ious0[i] = float((IoUb0 + IoUf0) / 2)
        if records is not None:
            records.append(dict(loss=loss, W=r["W"].detach().cpu(), W2=r["W2"].detach().cpu(),
                                pred_q0=None if r.get("pred_q0") is None else r["pred_q0"].detach().cpu(),
                                grad=transformer.flat.grad.detach().cpu().clone()))
        if ((epoch == 0 and i % 100 == 0) or i % 500 == 0) and rank == 0:
            print("iter {} IoUf {:.2f}, IoUb {:.2f}, IoUf0 {:.2f}, IoUb0 {:.2f}".format(i, IoUf, IoUb, IoUf0, IoUb0))
    if rank == 0:
        print("Epoch {}: The mIoU {:.2f}, loss {:.2f}, mIoU0 {:.2f}".format(
            epoch + 1, train_Ious.mean(), train_losses.mean(), train_Ious0.mean()))
    return train_Ious, train_losses

"""Variant heads on the extractor's features, on HIP kernels
(csrc/heads.hip) behind the C ABI:

  CosCls(in_dim, n_classes, cls_type)   src/model/pspnet.py:290-313  (cosine classifier)
  parse_param_coscls(cls_type)          src/model/pspnet.py:318-324
  get_classifier(args, num_classes)     src/model/pspnet.py:326-334  ('cos' / 'cosN')
  get_corr(q, k)                        src/model/model_util.py:101-109  (MMN correlation)

CosCls keeps the reference's parameter names and shapes (``cls.weight`` [n, C, 1, 1], or
``cls.weight_g`` / ``cls.weight_v`` under WeightNorm, ``cls.bias``, ``scale_factor``), so a
reference state_dict loads as is.  Its forward and the backward to its own parameters run on
the device; the frozen extractor receives no gradient (no caller backpropagates into it).
"""
from __future__ import annotations

import math

import torch

from . import _lib
from .transformer import as_tokens


def parse_param_coscls(cls_type: str):
    """pspnet.py:318-324: (WeightNormR, weight_norm, bias, temp) from a 4-letter code."""
    wn_r = {"r": True, "0": False, "o": False}
    wn = {"n": True, "0": False, "o": False}
    bias = {"b": True, "0": False, "o": False}
    temp = {"t": True, "0": False, "o": False}
    return wn_r[cls_type[0]], wn[cls_type[1]], bias[cls_type[2]], temp[cls_type[3]]


class _Cls(torch.nn.Module):
    """Parameter holder with nn.Conv2d(in_dim, n, 1)'s names (and WeightNorm's, dim=0)."""

    def __init__(self, in_dim: int, n: int, bias: bool, weight_norm_r: bool, device):
        super().__init__()
        bound = 1.0 / math.sqrt(in_dim)   # nn.Conv2d default init (kaiming_uniform, a=sqrt(5))
        w = torch.empty(n, in_dim, 1, 1, device=device).uniform_(-bound, bound)
        if weight_norm_r:   # WeightNorm.apply(cls, 'weight', dim=0): g = ||v|| per output channel
            self.weight_g = torch.nn.Parameter(w.flatten(1).norm(dim=1).view(n, 1, 1, 1))
            self.weight_v = torch.nn.Parameter(w)
        else:
            self.weight = torch.nn.Parameter(w)
        self.bias = torch.nn.Parameter(torch.empty(n, device=device).uniform_(-bound, bound)) if bias else None


class _CosFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, g, bias, scale, mode):
        B, P, C = x.shape
        n = weight.shape[0]
        out = torch.empty((B, n, P), device=x.device, dtype=torch.float32)
        _lib.check(_lib.lib().cwt_cos_classify(_lib.ctx(x.device.index), _lib.ptr(x), B, P, C, n, _lib.ptr(weight),
                                               _lib.ptr(g), _lib.ptr(bias), _lib.ptr(scale), mode, _lib.ptr(out),
                                               _lib.stream_ptr(x.device)), "cwt_cos_classify")
        ctx.save_for_backward(x, weight, g, bias, scale)
        ctx.mode = mode
        return out

    @staticmethod
    def backward(ctx, dout):
        x, weight, g, bias, scale = ctx.saved_tensors
        B, P, C = x.shape
        n = weight.shape[0]
        dout = dout.contiguous()
        dw = torch.empty_like(weight)
        dg = torch.empty_like(g) if g is not None else None
        db = torch.empty_like(bias) if bias is not None else None
        ds = torch.empty_like(scale)
        _lib.check(_lib.lib().cwt_cos_classify_bwd(_lib.ctx(x.device.index), _lib.ptr(x), B, P, C, n, _lib.ptr(weight),
                                                   _lib.ptr(g), _lib.ptr(bias), _lib.ptr(scale), ctx.mode,
                                                   _lib.ptr(dout), _lib.ptr(dw), _lib.ptr(dg), _lib.ptr(db),
                                                   _lib.ptr(ds), _lib.stream_ptr(x.device)), "cwt_cos_classify_bwd")
        return None, dw, dg, db, ds.reshape(scale.shape), None


class CosCls(torch.nn.Module):
    """pspnet.py:290-313: scores = scale * (W . x / max(||x||, 1e-5) + b) per pixel."""

    def __init__(self, in_dim: int = 512, n_classes: int = 2, cls_type: str = "0000", device=None):
        super().__init__()
        if in_dim != 512:
            raise NotImplementedError("the cosine head kernels take 512-channel features (bottleneck_dim)")
        if not 1 <= n_classes <= 64:
            raise NotImplementedError("n_classes must be in [1, 64]")
        self.WeightNormR, self.weight_norm, self.bias, self.temp = parse_param_coscls(cls_type)
        dev = torch.device("cuda", device if device is not None else torch.cuda.current_device()) \
            if torch.cuda.is_available() else torch.device("cpu")
        self.cls = _Cls(in_dim, n_classes, self.bias, self.WeightNormR, dev)
        if self.temp:
            self.scale_factor = torch.nn.Parameter(torch.tensor(2.0, device=dev))
        else:
            self.scale_factor = 2.0
            self.register_buffer("_scale", torch.tensor([2.0], device=dev), persistent=False)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        _lib.require(x, "x")
        B, C, h, w = x.shape
        tok = as_tokens(x).permute(0, 2, 3, 1).reshape(B, h * w, C)   # the [B, hw, C] token map (a view)
        mode = (1 if self.WeightNormR else 0) | (2 if self.weight_norm else 0)
        if self.WeightNormR:
            weight, g = self.cls.weight_v, self.cls.weight_g
        else:
            weight, g = self.cls.weight, None
        scale = self.scale_factor if self.temp else self._scale
        out = _CosFn.apply(tok, weight, g, self.cls.bias, scale, mode)
        return out.view(B, -1, h, w)

    def reset_parameters(self):
        n, C = (self.cls.weight_v if self.WeightNormR else self.cls.weight).shape[:2]
        fresh = _Cls(C, n, self.bias, self.WeightNormR, self.scale_factor.device if self.temp else self._scale.device)
        with torch.no_grad():
            for (_, p), (_, q) in zip(self.cls.named_parameters(), fresh.named_parameters()):
                p.copy_(q)


def get_classifier(args, num_classes=None):
    """pspnet.py:326-334 for dist 'cos' / 'cosN' (the CWT drivers build their 1x1 dot-product
    classifier themselves: the inner loop, episode.inner_adapt)."""
    get = args.get if isinstance(args, dict) else (lambda k, d=None: getattr(args, k, d))
    if num_classes is None:
        num_classes = get("num_classes_tr")
    dist = get("dist", "dot")
    if dist in ("cos", "cosN"):
        return CosCls(in_dim=get("bottleneck_dim", 512), n_classes=num_classes, cls_type=get("cls_type", "0000"))
    raise NotImplementedError(f"dist {dist!r}: only the cosine heads are built here")


class _CorrFn(torch.autograd.Function):
    """get_corr under autograd: the backward is cwt_corr_backward (normalize's Jacobian around
    two f32-MFMA GEMMs, d_sim . k_hat and d_sim^T . q_hat)."""

    @staticmethod
    def forward(ctx, qt, kt):
        ctx.save_for_backward(qt, kt)
        return _corr_tokens(qt, kt)

    @staticmethod
    def backward(ctx, d_sim):
        qt, kt = ctx.saved_tensors
        bs, ch, h, w = qt.shape
        Pq, Pk = h * w, kt.shape[2] * kt.shape[3]
        dq = torch.empty_like(qt) if ctx.needs_input_grad[0] else None
        dk = torch.empty_like(kt) if ctx.needs_input_grad[1] else None
        if dq is None and dk is None:
            return None, None
        d = d_sim.contiguous()
        _lib.check(_lib.lib().cwt_corr_backward(_lib.ctx(qt.device.index), _lib.ptr(qt), _lib.ptr(kt), bs, Pq, Pk, ch,
                                                _lib.ptr(d), _lib.ptr(dq), _lib.ptr(dk), 0, 0,
                                                _lib.stream_ptr(qt.device)), "cwt_corr_backward")
        return dq, dk


def _corr_tokens(qt: torch.Tensor, kt: torch.Tensor) -> torch.Tensor:
    bs, ch, h, w = qt.shape
    Pq, Pk = h * w, kt.shape[2] * kt.shape[3]
    sim = torch.empty((bs, Pq, Pk), device=qt.device, dtype=torch.float32)
    _lib.check(_lib.lib().cwt_corr(_lib.ctx(qt.device.index), _lib.ptr(qt), _lib.ptr(kt), bs, Pq, Pk, ch, _lib.ptr(sim),
                                   _lib.stream_ptr(qt.device)), "cwt_corr")
    return sim


def get_corr(q: torch.Tensor, k: torch.Tensor) -> torch.Tensor:
    """model_util.py:101-109: q, k [bs, ch, h, w] -> sim [bs, h*w, h*w] (q tokens x k tokens),
    cosine similarity of every pair (F.normalize eps 1e-12), exact fp32 on the matrix cores.
    Differentiable (cwt_corr_backward) when either input requires grad."""
    _lib.require(q, "q")
    _lib.require(k, "k")
    bs, ch, h, w = q.shape
    if k.shape[0] != bs or k.shape[1] != ch:
        raise ValueError("q and k must share batch and channels")
    qt, kt = as_tokens(q), as_tokens(k)
    if torch.is_grad_enabled() and (qt.requires_grad or kt.requires_grad):
        return _CorrFn.apply(qt, kt)
    return _corr_tokens(qt, kt)

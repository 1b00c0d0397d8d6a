"""Drop-in for the reference's Classifier Weight Transformer (src/model/transformer.py:33-83).

``MultiHeadAttentionOne(n_head, d_model, d_k, d_v, dropout)`` keeps the reference
constructor, ``forward(q, k, v) -> [B, 2, d_model]`` signature and state_dict keys
(``w_qkvs.weight``, ``layer_norm.{weight,bias}``, ``fc.{weight,bias}``).  The forward and
the parameter backward run as HIP kernels (libcwt.so, cwt_attention_fwd/bwd) in the
re-associated form described in cwt_attn.hip / DESIGN.md.

All parameters live in ONE flat fp32 device buffer (``self.flat``); the named tensors are
views of it.  That makes the 8-GPU gradient all-reduce one RCCL call on one bucket and the
outer SGD step one kernel.

Differences from the reference, by design: k and v must be the same tensor
(the only way the CWT drivers call it, test.py:197 / train.py:257).  In training mode the two
dropouts run as in the reference (``self.attention.dropout`` p=0.1 on the attention
probabilities, ``self.dropout`` on the fc output; set their ``.p`` to 0 exactly as the
reference would), with masks from the kernels' counter-based generator (a fresh seed per
forward, util.dropout_seed: the host RNG stream that draws W0 is left untouched, as the
reference's CUDA-generator dropouts leave it) instead of torch's Philox stream.
"""
from __future__ import annotations

import math
from collections import OrderedDict

import numpy as np
import torch

from . import _lib
from .util import dropout_seed


def _layout(heads: int, C: int):
    names = [("w_qkvs.weight", (heads * C, C)), ("layer_norm.weight", (C,)), ("layer_norm.bias", (C,)),
             ("fc.weight", (C, heads * C)), ("fc.bias", (C,))]
    out, off = [], 0
    for n, shp in names:
        k = int(np.prod(shp))
        out.append((n, shp, off, k))
        off += k
    return out, off


def as_tokens(k: torch.Tensor) -> torch.Tensor:
    """[B,C,h,w] (any memory format) -> NHWC-contiguous [B,h,w,C] storage, returned as [B,C,h,w]
    channels_last so its data_ptr is the token-major [B, hw, C] map the kernels read."""
    if k.dim() == 3:  # [B, hw, C] tokens already
        return k.contiguous()
    return k.contiguous(memory_format=torch.channels_last)


class _CWTFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, f, flat, mod, drop):
        out, saved = mod._fwd(q, f, need_saved=True, drop=drop)
        ctx.mod, ctx.drop = mod, drop
        ctx.save_for_backward(q, f, flat)
        ctx.saved_buf = saved
        return out

    @staticmethod
    def backward(ctx, d_out):
        q, f, flat = ctx.saved_tensors
        g = torch.zeros_like(flat)
        ctx.mod._bwd(q, f, ctx.saved_buf, d_out.contiguous(), g, drop=ctx.drop)
        return None, None, g, None, None


class _Attention(torch.nn.Module):
    """Holder mirroring the reference's ScaledDotProductAttention attributes (transformer.py:12-19):
    ``temperature`` and ``dropout`` (nn.Dropout(0.1), applied in training mode)."""

    def __init__(self, temperature: float, attn_dropout: float = 0.1):
        super().__init__()
        self.temperature = temperature
        self.dropout = torch.nn.Dropout(attn_dropout)


class MultiHeadAttentionOne(torch.nn.Module):
    """transformer.py:33-83 (shared projection, d_k = d_v = d_model per head)."""
    _uid = 0

    def __init__(self, n_head: int, d_model: int, d_k: int, d_v: int, dropout: float = 0.1, device=None):
        super().__init__()
        if not (d_model == d_k == d_v == 512):
            raise NotImplementedError("the CWT path uses d_model = d_k = d_v = 512 (test.py:57)")
        if n_head not in (1, 2, 4):
            raise NotImplementedError("n_head must be 1, 2 or 4 (heads 1 in the yaml, 4 in scripts/*.sh)")
        self.n_head, self.d_model = n_head, d_model
        self.attention = _Attention(temperature=float(np.power(d_k, 0.5)))  # transformer.py:47
        self.dropout = torch.nn.Dropout(dropout)                              # transformer.py:52
        self._layout, total = _layout(n_head, d_model)
        MultiHeadAttentionOne._uid += 1
        self._uid = MultiHeadAttentionOne._uid   # with flat._version: the identity of the folded weights
        dev = torch.device("cuda", device if device is not None else torch.cuda.current_device()) \
            if torch.cuda.is_available() else torch.device("cpu")
        self.flat = torch.nn.Parameter(torch.zeros(total, dtype=torch.float32, device=dev))
        self._init_reference_like()

    # -- parameters -----------------------------------------------------------------------
    def _init_reference_like(self):
        """transformer.py:45,51 init: w_qkvs ~ N(0, sqrt(2/(d_model+d_k))), fc xavier_normal,
        LayerNorm (1, 0), fc.bias U(+-1/sqrt(fan_in)) (nn.Linear default)."""
        C, H = self.d_model, self.n_head
        with torch.no_grad():
            self.view("w_qkvs.weight").normal_(0, math.sqrt(2.0 / (2 * C)))
            self.view("layer_norm.weight").fill_(1.0)
            self.view("layer_norm.bias").zero_()
            self.view("fc.weight").normal_(0, math.sqrt(2.0 / (H * C + C)))
            b = 1.0 / math.sqrt(H * C)
            self.view("fc.bias").uniform_(-b, b)

    def view(self, name: str, t: torch.Tensor | None = None) -> torch.Tensor:
        t = self.flat if t is None else t
        for n, shp, off, k in self._layout:
            if n == name:
                return t.data[off:off + k].view(shp) if t is self.flat else t[off:off + k].view(shp)
        raise KeyError(name)

    def state_dict(self, *a, **k):
        return OrderedDict((n, self.flat.data[off:off + kk].view(shp).clone()) for n, shp, off, kk in self._layout)

    def load_state_dict(self, sd, strict: bool = True):
        for n, shp, off, k in self._layout:
            if n not in sd:
                if strict:
                    raise KeyError(n)
                continue
            v = sd[n]
            v = torch.as_tensor(np.asarray(v)) if not isinstance(v, torch.Tensor) else v
            if tuple(v.shape) != tuple(shp):
                raise ValueError(f"{n}: {tuple(v.shape)} != {shp}")
            with torch.no_grad():
                self.flat.data[off:off + k].copy_(v.reshape(-1).to(self.flat.device, torch.float32))
        torch.autograd.graph.increment_version(self.flat)   # writes through .data do not bump it
        return self

    def named_views(self):
        # detach() (not .data) shares flat's version counter: an in-place write through a view
        # bumps params_version(), so the folded inference weights cannot go stale
        flat = self.flat.detach()
        return [(n, flat[off:off + k].view(shp)) for n, shp, off, k in self._layout]

    # -- kernels --------------------------------------------------------------------------
    def _ptrs(self, t: torch.Tensor):
        return [_lib.ptr(self.view(n, t)) for n in ("w_qkvs.weight", "fc.weight", "fc.bias", "layer_norm.weight",
                                                    "layer_norm.bias")]

    def _check(self, q, f):
        _lib.require(q, "q")
        _lib.require(f, "k")
        if q.dim() != 3 or q.shape[1] != 2 or q.shape[2] != self.d_model:
            raise ValueError(f"q must be [B,2,{self.d_model}], got {tuple(q.shape)}")
        B = q.shape[0]
        if f.dim() == 4:
            if f.shape[0] != B or f.shape[1] != self.d_model:
                raise ValueError(f"k must be [B,{self.d_model},h,w], got {tuple(f.shape)}")
            hw = f.shape[2] * f.shape[3]
        else:
            hw = f.shape[1]
        return B, hw

    @property
    def dropout_p(self) -> float:
        return float(self.dropout.p)

    def _drop(self):
        """(attention p, output p, seed) in training mode with a dropout on, else None."""
        pa, po = float(self.attention.dropout.p), float(self.dropout.p)
        if not self.training or (pa == 0.0 and po == 0.0):
            return None
        seed = dropout_seed()   # leaves the host RNG stream (W0 draws) as the reference's
        return pa, po, seed

    def _fwd(self, q, f, need_saved: bool, drop=None):
        q = q.contiguous()
        B, hw = self._check(q, f)
        out = torch.empty((B, 2, self.d_model), device=q.device, dtype=torch.float32)
        saved = None
        if need_saved:
            n = _lib.lib().cwt_attention_saved_floats(B, hw, self.d_model, self.n_head)
            saved = torch.empty(n, device=q.device, dtype=torch.float32)
        w, fw, fb, lw, lb = self._ptrs(self.flat)
        pa, po, seed = drop if drop is not None else (0.0, 0.0, 0)
        _lib.check(_lib.lib().cwt_attention_fwd_train(_lib.ctx(q.device.index), _lib.ptr(q), _lib.ptr(f), B, hw,
                                                      self.d_model, self.n_head, w, fw, fb, lw, lb, _lib.ptr(out),
                                                      _lib.ptr(saved), pa, po, seed, _lib.stream_ptr(q.device)),
                   "cwt_attention_fwd_train")
        return out, saved

    def _bwd(self, q, f, saved, d_out, grad_flat, drop=None):
        B, hw = self._check(q, f)
        w, fw, fb, lw, lb = self._ptrs(self.flat)
        gw, gfw, gfb, glw, glb = self._ptrs(grad_flat)
        pa, po, seed = drop if drop is not None else (0.0, 0.0, 0)
        _lib.check(_lib.lib().cwt_attention_bwd_train(_lib.ctx(q.device.index), _lib.ptr(q), _lib.ptr(f), B, hw,
                                                      self.d_model, self.n_head, w, fw, fb, lw, lb, _lib.ptr(saved),
                                                      _lib.ptr(d_out), gw, gfw, gfb, glw, glb, pa, po, seed,
                                                      _lib.stream_ptr(q.device)), "cwt_attention_bwd_train")

    # -- reference API --------------------------------------------------------------------
    def forward(self, q, k, v, query_input=False):
        """transformer.py:54: q [B,2,512]; k = v = normalised query features [B,512,h,w]."""
        if k is not v and k.data_ptr() != v.data_ptr():
            raise NotImplementedError("CWT kernels attend with k == v (test.py:197, train.py:257)")
        f = as_tokens(k)
        drop = self._drop()
        if torch.is_grad_enabled() and self.flat.requires_grad:
            return _CWTFunction.apply(q, f, self.flat, self, drop)
        out, _ = self._fwd(q, f, need_saved=False, drop=drop)
        return out

    def infer(self, q, k):
        """Eval-mode forward whatever the module's mode (the inference engine's call)."""
        out, _ = self._fwd(q, as_tokens(k), need_saved=False)
        return out

    def params_version(self) -> int:
        """Identity of the current parameter values for libcwt's folded-weight cache: this module's
        id and flat's in-place version counter (bumped by load_state_dict, the optimisers and any
        in-place op on flat; code writing through flat.data must call
        torch.autograd.graph.increment_version(flat))."""
        return (self._uid << 40) | (int(self.flat._version) & ((1 << 40) - 1))

    def infer_raw(self, q, f, with_logits0: bool = True):
        """The inference episode's normalize + baseline logits + eval-mode CWT (test.py:190-197) over
        the RAW query features in one pass (cwt_attention_infer, 4 heads): returns (W' [B,2,512],
        inv_norm [B,hw] with F.normalize(f) = f * inv_norm, pred_q0 = W . f [B,2,h,w] or None)."""
        if self.n_head != 4:
            raise NotImplementedError("the fused inference tail needs 4 heads (scripts/*.sh); use infer()")
        q = q.contiguous()
        B, hw = self._check(q, f)
        ft = as_tokens(f)
        out = torch.empty((B, 2, self.d_model), device=q.device, dtype=torch.float32)
        inv = torch.empty((B, hw), device=q.device, dtype=torch.float32)
        lg0 = torch.empty((B, 2) + tuple(f.shape[2:]), device=q.device, dtype=torch.float32) if with_logits0 else None
        w, fw, fb, lw, lb = self._ptrs(self.flat)
        _lib.check(_lib.lib().cwt_attention_infer(_lib.ctx(q.device.index), _lib.ptr(q), _lib.ptr(ft), B, hw,
                                                  self.d_model, self.n_head, w, fw, fb, lw, lb, self.params_version(),
                                                  _lib.ptr(out), _lib.ptr(inv), _lib.ptr(lg0),
                                                  _lib.stream_ptr(q.device)), "cwt_attention_infer")
        return out, inv, lg0

    # explicit training API (no autograd graph; used by the episode drivers)
    def forward_train(self, q, f):
        f = as_tokens(f)
        drop = self._drop()
        out, saved = self._fwd(q, f, need_saved=True, drop=drop)
        return out, (q.contiguous(), f, saved, drop)

    def backward_into(self, state, d_out, grad_flat=None):
        q, f, saved, drop = state
        if grad_flat is None:
            if self.flat.grad is None:
                self.flat.grad = torch.zeros_like(self.flat)
            grad_flat = self.flat.grad
        self._bwd(q, f, saved, d_out.contiguous(), grad_flat, drop=drop)
        return grad_flat

"""DeTr, the transformer head of the train_trans / train_tp_trans variants,
on HIP kernels (csrc/detr.hip, the f32-MFMA GEMM of csrc/heads.hip, MatchNet of csrc/match.hip)
behind the C ABI:

  SinePositionalEncoding(num_feats, ...)          src/model/positional_encoding.py:7-74
  MSDeformAttn(d_model, n_levels, n_heads, ...)   src/model/ops/modules/ms_deform_attn.py:30-117
                                                  (+ ms_deform_attn_core_pytorch, functions/
                                                  ms_deform_attn_func.py:41-61)
  DeformAtt(embed_dims, n_heads, n_points, ...)   src/model/detr.py:78-151
  DeTr(args, sf_att, cs_att, reduce_dim)          src/model/detr.py:13-75

The modules keep the reference's parameter names (``adjust_feature.0.weight``,
``cross_trans.NeighConsensus.conv.*``, ``self_trans.level_embed``, ``self_trans.self_trans.
{sampling_offsets,attention_weights,value_proj,output_proj}.{weight,bias}``) and its
initialisation, so a reference state_dict loads as is.  Built: one feature level (DeformAtt's
n_levels = 1, the only one DeTr constructs), 2-D reference points, no padding masks (DeTr is
called with padding_mask=None, train_trans.py:146,284), dropout off (eval).

The reference's DeTr.compute_feat (detr.py:49-61) indexes ``fq_lst[int(l) - 2]`` and concatenates
the entries, which does not match what this repo's reference PSPNet.get_feat_list returns (a dict
{2, 3, 4: [feature]}, pspnet.py:272-287): as written it cannot run against that extractor.  Here
``rmid`` names the layers as in_fea_dim_lookup does ('l34' = layer3 + layer4, 1024 + 2048
channels, detr.py:10), and fq_lst / fs_lst may be that dict (of features or one-element lists) or
a list indexed by layer - 2.

Training (round 4): under autograd every op of the head has its device
backward -- cwt_linear_backward (adjust_feature's segments, the four MSDeformAttn projections),
cwt_deform_attn_backward (softmax over the points, bilinear sampling: values, offsets, logits),
cwt_norm_blend_backward, the position embedding's identity gradient, and MatchNet's
(match.py) -- so DeTr trains as train_trans.py:100 runs it.

Parity is unpinned: the reference cannot be run here and holds no fixtures for this
head; tests/test_gpu_detr.py checks it against oracle/detr_oracle.py (float64, torch's own
grid_sample for the sampling).
"""
from __future__ import annotations

import math

import torch

from . import _lib
from .match import MatchNet
from .transformer import as_tokens

IN_FEA_DIM = {"l3": 1024, "l4": 2048, "l34": 1024 + 2048, "l23": 512 + 1024}


def _get(args, k, default=None):
    if isinstance(args, dict):
        return args.get(k, default)
    return getattr(args, k, default)


def linear(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None = None, relu: bool = False,
           out: torch.Tensor | None = None, accumulate: bool = False) -> torch.Tensor:
    """x [P, K] (contiguous tokens), weight [N, K] (or [N, K, 1, 1]) -> [P, N] (cwt_linear)."""
    _lib.require(x, "x")
    P, K = x.shape
    w = weight.detach().reshape(weight.shape[0], -1).contiguous()
    N = w.shape[0]
    if w.shape[1] != K:
        raise ValueError(f"linear: weight has {w.shape[1]} input features, x has {K}")
    if out is None:
        if accumulate:
            raise ValueError("linear: accumulate needs out")
        out = torch.empty((P, N), device=x.device, dtype=torch.float32)
    b = bias.detach().contiguous() if bias is not None else None
    _lib.check(_lib.lib().cwt_linear(_lib.ctx(x.device.index), _lib.ptr(x), P, K, _lib.ptr(w),
                                     _lib.ptr(b) if b is not None else None, N, int(relu), int(accumulate),
                                     _lib.ptr(out), _lib.stream_ptr(x.device)), "cwt_linear")
    return out


def _needs_grad(*ts) -> bool:
    return torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in ts)


class _LinearFn(torch.autograd.Function):
    """linear under autograd; the backward is cwt_linear_backward (ReLU mask from the output)."""

    @staticmethod
    def forward(ctx, x, weight, bias, relu):
        out = linear(x, weight, bias, relu)
        ctx.save_for_backward(x, weight, out if relu else None)
        ctx.has_bias = bias is not None
        return out

    @staticmethod
    def backward(ctx, d):
        x, weight, out = ctx.saved_tensors
        w = weight.detach().reshape(weight.shape[0], -1).contiguous()
        N, K = w.shape
        P = x.shape[0]
        d = d.contiguous()
        f = dict(device=x.device, dtype=torch.float32)
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        dw = torch.empty((N, K), **f) if ctx.needs_input_grad[1] else None
        db = torch.empty(N, **f) if (ctx.has_bias and ctx.needs_input_grad[2]) else None
        _lib.check(_lib.lib().cwt_linear_backward(_lib.ctx(x.device.index), _lib.ptr(x), P, K, _lib.ptr(w), N,
                                                  _lib.ptr(out), _lib.ptr(d), _lib.ptr(dx), _lib.ptr(dw), K,
                                                  _lib.ptr(db), _lib.stream_ptr(x.device)), "cwt_linear_backward")
        return dx, (dw.reshape(weight.shape) if dw is not None else None), db, None


def linear_t(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None = None, relu: bool = False):
    """linear, differentiable when x or the parameters require grad."""
    if _needs_grad(x, weight, bias):
        return _LinearFn.apply(x, weight, bias, relu)
    return linear(x, weight, bias, relu)


class _NormBlendFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, at, bt, wt):
        ctx.save_for_backward(at, bt)
        ctx.wt = float(wt)
        return _norm_blend_tokens(at, bt, wt)

    @staticmethod
    def backward(ctx, d):
        at, bt = ctx.saved_tensors
        B, C, h, w = at.shape
        dt = as_tokens(d)
        da = torch.empty_like(at) if ctx.needs_input_grad[0] else None
        db = torch.empty_like(bt) if ctx.needs_input_grad[1] else None
        _lib.check(_lib.lib().cwt_norm_blend_backward(_lib.ctx(at.device.index), _lib.ptr(at), _lib.ptr(bt), B * h * w,
                                                      C, ctx.wt, _lib.ptr(dt), _lib.ptr(da), _lib.ptr(db),
                                                      _lib.stream_ptr(at.device)), "cwt_norm_blend_backward")
        return da, db, None


def _norm_blend_tokens(at, bt, wt):
    B, C, h, w = at.shape
    out = torch.empty((B, C, h, w), device=at.device, dtype=torch.float32, memory_format=torch.channels_last)
    _lib.check(_lib.lib().cwt_norm_blend(_lib.ctx(at.device.index), _lib.ptr(at), _lib.ptr(bt), B * h * w, C, float(wt),
                                         _lib.ptr(out), _lib.stream_ptr(at.device)), "cwt_norm_blend")
    return out


def norm_blend(a: torch.Tensor, b: torch.Tensor, wt: float) -> torch.Tensor:
    """F.normalize(a, dim=1) + F.normalize(b, dim=1) * wt for [B, C, h, w] maps (detr.py:41,45);
    returns a channels_last [B, C, h, w] map (differentiable: cwt_norm_blend_backward)."""
    at, bt = as_tokens(a), as_tokens(b)
    if _needs_grad(at, bt):
        return _NormBlendFn.apply(at, bt, wt)
    return _norm_blend_tokens(at, bt, wt)


class SinePositionalEncoding(torch.nn.Module):
    """positional_encoding.py:7-74.  ``add_to(x)`` = x + pos for the mask DeformAtt builds without a
    padding mask (a zero long tensor, detr.py:135), on the device."""

    def __init__(self, num_feats: int, temperature: int = 10000, normalize: bool = False, scale=2 * math.pi,
                 eps: float = 1e-6):
        super().__init__()
        if normalize and not isinstance(scale, (float, int)):
            raise TypeError("when normalize is set, scale should be provided and in float or int type")
        self.num_feats, self.temperature, self.normalize, self.scale, self.eps = (num_feats, temperature, normalize,
                                                                                  scale, eps)

    def add_to(self, x: torch.Tensor) -> torch.Tensor:
        """x [B, C, h, w] with C = 2 num_feats -> x + pos (channels_last); the gradient with respect
        to x is the identity (pos is a constant of the shape)."""
        xt = as_tokens(x)
        B, C, h, w = xt.shape
        if C != 2 * self.num_feats:
            raise ValueError(f"expected {2 * self.num_feats} channels, got {C}")
        if _needs_grad(xt):
            return _AddPosFn.apply(xt, self)
        return self._add(xt)

    def _add(self, xt: torch.Tensor) -> torch.Tensor:
        B, C, h, w = xt.shape
        out = torch.empty_like(xt)
        _lib.check(_lib.lib().cwt_sine_pos_add(_lib.ctx(xt.device.index), _lib.ptr(xt), B, h, w, C,
                                               float(self.temperature), int(self.normalize), float(self.scale),
                                               float(self.eps), _lib.ptr(out), _lib.stream_ptr(xt.device)),
                   "cwt_sine_pos_add")
        return out


class _AddPosFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, xt, mod):
        return mod._add(xt)

    @staticmethod
    def backward(ctx, d):
        return d, None


def _deform_core(value, offs, logits, N, H, W, M, P, D):
    core = torch.empty((N * H * W, M * D), device=value.device, dtype=torch.float32)
    _lib.check(_lib.lib().cwt_deform_attn(_lib.ctx(value.device.index), _lib.ptr(value), _lib.ptr(offs),
                                          _lib.ptr(logits), N, H, W, M, P, D, _lib.ptr(core),
                                          _lib.stream_ptr(value.device)), "cwt_deform_attn")
    return core


class _DeformCoreFn(torch.autograd.Function):
    """The deformable-attention core under autograd (cwt_deform_attn / cwt_deform_attn_backward)."""

    @staticmethod
    def forward(ctx, value, offs, logits, N, H, W, M, P, D):
        core = _deform_core(value, offs, logits, N, H, W, M, P, D)
        ctx.save_for_backward(value, offs, logits)
        ctx.meta = (N, H, W, M, P, D)
        return core

    @staticmethod
    def backward(ctx, d):
        value, offs, logits = ctx.saved_tensors
        N, H, W, M, P, D = ctx.meta
        d = d.contiguous()
        dv, do, dl = torch.empty_like(value), torch.empty_like(offs), torch.empty_like(logits)
        _lib.check(_lib.lib().cwt_deform_attn_backward(_lib.ctx(value.device.index), _lib.ptr(value), _lib.ptr(offs),
                                                       _lib.ptr(logits), N, H, W, M, P, D, _lib.ptr(d), _lib.ptr(dv),
                                                       _lib.ptr(do), _lib.ptr(dl), _lib.stream_ptr(value.device)),
                   "cwt_deform_attn_backward")
        return dv, do, dl, None, None, None, None, None, None


class MSDeformAttn(torch.nn.Module):
    """ms_deform_attn.py:30-117 (parameters and initialisation as the reference); forward over one
    level with 2-D reference points on the device."""

    def __init__(self, d_model: int = 256, n_levels: int = 4, n_heads: int = 8, n_points: int = 4, device=None):
        super().__init__()
        if d_model % n_heads != 0:
            raise ValueError(f"d_model must be divisible by n_heads, but got {d_model} and {n_heads}")
        self.im2col_step = 64
        self.d_model, self.n_levels, self.n_heads, self.n_points = d_model, n_levels, n_heads, n_points
        self.sampling_offsets = torch.nn.Linear(d_model, n_heads * n_levels * n_points * 2, device=device)
        self.attention_weights = torch.nn.Linear(d_model, n_heads * n_levels * n_points, device=device)
        self.value_proj = torch.nn.Linear(d_model, d_model, device=device)
        self.output_proj = torch.nn.Linear(d_model, d_model, device=device)
        self._reset_parameters()

    def _reset_parameters(self):
        """ms_deform_attn.py:61-75 (parameter initialisation, not a compute path)."""
        with torch.no_grad():
            self.sampling_offsets.weight.zero_()
            thetas = torch.arange(self.n_heads, dtype=torch.float32) * (2.0 * math.pi / self.n_heads)
            grid = torch.stack([thetas.cos(), thetas.sin()], -1)
            grid = (grid / grid.abs().max(-1, keepdim=True)[0]).view(self.n_heads, 1, 1, 2).repeat(
                1, self.n_levels, self.n_points, 1)
            for i in range(self.n_points):
                grid[:, :, i, :] *= i + 1
            self.sampling_offsets.bias.copy_(grid.view(-1))
            self.attention_weights.weight.zero_()
            self.attention_weights.bias.zero_()
            torch.nn.init.xavier_uniform_(self.value_proj.weight)
            self.value_proj.bias.zero_()
            torch.nn.init.xavier_uniform_(self.output_proj.weight)
            self.output_proj.bias.zero_()

    def forward(self, query, reference_points, input_flatten, input_spatial_shapes, input_level_start_index=None,
                input_padding_mask=None):
        """query / input_flatten [N, H*W, C]; reference_points [N, H*W, 1, 2] must be DeformAtt's
        grid of pixel centres (the only form built); input_spatial_shapes [[H, W]]."""
        if input_padding_mask is not None:
            raise NotImplementedError("MSDeformAttn: input_padding_mask is not built (DeTr passes None)")
        shapes = [tuple(int(v) for v in s) for s in torch.as_tensor(input_spatial_shapes).reshape(-1, 2).tolist()]
        if len(shapes) != 1 or self.n_levels != 1:
            raise NotImplementedError("MSDeformAttn: one feature level only (DeformAtt n_levels = 1)")
        H, W = shapes[0]
        if reference_points is not None and reference_points.shape[-1] != 2:
            raise NotImplementedError("MSDeformAttn: 2-D reference points only")
        N, Lq, C = query.shape
        if Lq != H * W or input_flatten.shape[1] != H * W:
            raise ValueError("MSDeformAttn: queries must be the H*W pixel centres of the single level")
        q = query.reshape(N * Lq, C).contiguous()
        v_in = input_flatten.reshape(N * Lq, C).contiguous()
        value = linear_t(v_in, self.value_proj.weight, self.value_proj.bias)
        offs = linear_t(q, self.sampling_offsets.weight, self.sampling_offsets.bias)
        logits = linear_t(q, self.attention_weights.weight, self.attention_weights.bias)
        M, P = self.n_heads, self.n_points
        if _needs_grad(value, offs, logits):
            core = _DeformCoreFn.apply(value, offs, logits, N, H, W, M, P, C // M)
        else:
            core = _deform_core(value, offs, logits, N, H, W, M, P, C // M)
        return linear_t(core, self.output_proj.weight, self.output_proj.bias).reshape(N, Lq, C)


class DeformAtt(torch.nn.Module):
    """detr.py:78-151 (n_levels = 1): self-attention of the query map with deformable sampling,
    the query tokens carrying the sine position embedding."""

    def __init__(self, embed_dims: int = 512, n_heads: int = 8, n_points: int = 9, n_levels: int = 1, device=None):
        super().__init__()
        if n_levels != 1:
            raise NotImplementedError("DeformAtt: one level (the DeTr configuration)")
        self.num_levels = n_levels
        self.level_embed = torch.nn.Parameter(torch.rand(n_levels, embed_dims, device=device))  # unused at 1 level
        self.positional_encoding = SinePositionalEncoding(embed_dims // 2, normalize=True)
        self.self_trans = MSDeformAttn(d_model=embed_dims, n_levels=n_levels, n_heads=n_heads, n_points=n_points,
                                       device=device)

    def forward(self, fq_fea, f_q, padding_mask=None):
        """fq_fea [B, C, h, w] (the queries' key features), f_q [B, C, h, w] (sampled values)
        -> sa_fq [B, C, h, w] (channels_last)."""
        if padding_mask is not None:
            raise NotImplementedError("DeformAtt: padding masks are not built (DeTr passes None)")
        if isinstance(fq_fea, (list, tuple)):
            if len(fq_fea) != 1:
                raise NotImplementedError("DeformAtt: one level")
            fq_fea = fq_fea[0]
        B, C, h, w = fq_fea.shape
        q = self.positional_encoding.add_to(fq_fea)                     # q_flatten + pos_embed_flatten
        qt = q.permute(0, 2, 3, 1).reshape(B, h * w, C)                 # storage order: no copy
        vt = as_tokens(f_q).permute(0, 2, 3, 1).reshape(B, h * w, C)
        out = self.self_trans(qt, None, vt, [[h, w]])
        return out.reshape(B, h, w, C).permute(0, 3, 1, 2)


class _AdjustFn(torch.autograd.Function):
    """adjust_feature (detr.py:22,58-59) under autograd: d x_l = g . W_l and the weight gradient's
    column segment l = g^T . x_l, with g the output gradient through the ReLU."""

    @staticmethod
    def forward(ctx, mod, weight, *feats):
        out = mod._adjust(list(feats))
        ctx.mod = mod
        ctx.save_for_backward(out, *feats)
        return out

    @staticmethod
    def backward(ctx, d):
        out, *feats = ctx.saved_tensors
        mod = ctx.mod
        B, N, h, w = out.shape
        P = B * h * w
        dt = as_tokens(d).permute(0, 2, 3, 1).reshape(P, N)
        o2 = out.permute(0, 2, 3, 1).reshape(P, N)
        segs = mod._weight_segments([f.shape[1] for f in feats])
        Ktot = sum(f.shape[1] for f in feats)
        dev = out.device
        dW = torch.empty((N, Ktot), device=dev, dtype=torch.float32) if ctx.needs_input_grad[1] else None
        grads, off = [], 0
        for i, (f, wseg) in enumerate(zip(feats, segs)):
            K = f.shape[1]
            ft = f.permute(0, 2, 3, 1).reshape(P, K)
            dx = torch.empty_like(f) if ctx.needs_input_grad[2 + i] else None
            dxt = dx.permute(0, 2, 3, 1).reshape(P, K) if dx is not None else None
            _lib.check(_lib.lib().cwt_linear_backward(
                _lib.ctx(dev.index), _lib.ptr(ft), P, K, _lib.ptr(wseg), N, _lib.ptr(o2), _lib.ptr(dt), _lib.ptr(dxt),
                _lib.ptr(dW[:, off:]) if dW is not None else None, Ktot, None, _lib.stream_ptr(dev)),
                "cwt_linear_backward")
            grads.append(dx)
            off += K
        return (None, dW.reshape(mod.adjust_feature[0].weight.shape) if dW is not None else None, *grads)


class DeTr(torch.nn.Module):
    """detr.py:13-75: adjust_feature (1x1 conv, no bias, ReLU) on the concatenated layer features,
    then the cross attention (MatchNet over the adjusted query / support features, values f_s)
    and / or the deformable self attention, each blended into f_q as normalize(f_q) +
    normalize(att) * att_wt.  Returns (f_q, sa_fq or None, ca_fq or None)."""

    def __init__(self, args, sf_att: bool = False, cs_att: bool = True, reduce_dim: int = 512, device=None):
        super().__init__()
        self.args, self.reduce_dim, self.sf_att, self.cs_att = args, reduce_dim, sf_att, cs_att
        rmid = str(_get(args, "rmid"))
        if rmid not in IN_FEA_DIM:
            raise NotImplementedError(f"DeTr: rmid {rmid!r} (built: {sorted(IN_FEA_DIM)})")
        self.rmid = rmid
        self.layers_used = [int(c) for c in rmid[1:]]
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        in_fea_dim = IN_FEA_DIM[rmid]
        self.adjust_feature = torch.nn.Sequential(
            torch.nn.Conv2d(in_fea_dim, reduce_dim, kernel_size=1, padding=0, bias=False, device=dev),
            torch.nn.ReLU(inplace=True))
        if _get(args, "drop", False) not in (False, None, 0):
            raise NotImplementedError("DeTr: the adjust_feature Dropout2d (args.drop) is training-only")
        if cs_att:
            self.cross_trans = MatchNet(temp=float(_get(args, "temp", 20.0)), cv_type="red", sce=False,
                                        sym_mode=True, device=dev)
        if sf_att:
            self.self_trans = DeformAtt(embed_dims=reduce_dim, n_levels=1, n_heads=8, n_points=9, device=dev)
        self.att_wt = float(_get(args, "att_wt", 0.2))
        self._wsplit, self._wkey = None, None

    def _weight_segments(self, dims):
        """adjust_feature's weight split per input layer ([reduce_dim][C_l] each, contiguous)."""
        w = self.adjust_feature[0].weight
        key = (w.data_ptr(), w._version, tuple(dims))
        if self._wsplit is None or key != self._wkey:
            with torch.no_grad():
                w2 = w.detach().reshape(self.reduce_dim, -1)
                segs, o = [], 0
                for d in dims:
                    segs.append(w2[:, o:o + d].contiguous())
                    o += d
            self._wsplit, self._wkey = segs, key
        return self._wsplit

    def _layer(self, lst, lid):
        if isinstance(lst, dict):
            f = lst[lid]
        else:
            f = lst[lid - 2]
        return f[0] if isinstance(f, (list, tuple)) else f

    def _adjust(self, feats):
        """relu(sum_l x_l . W_l^T) over the layer segments (the concatenation never materialised)."""
        B, _, h, w = feats[0].shape
        segs = self._weight_segments([f.shape[1] for f in feats])
        out = torch.empty((B, self.reduce_dim, h, w), device=feats[0].device, dtype=torch.float32,
                          memory_format=torch.channels_last)
        o2 = out.permute(0, 2, 3, 1).reshape(B * h * w, self.reduce_dim)
        for i, (f, wseg) in enumerate(zip(feats, segs)):
            ft = as_tokens(f).permute(0, 2, 3, 1).reshape(B * h * w, f.shape[1])
            last = i == len(feats) - 1
            linear(ft, wseg, None, relu=last, out=o2, accumulate=i > 0)
        return out

    def compute_feat(self, fq_lst, fs_lst):
        """detr.py:49-61: relu(conv1x1(cat(layer features))) for the query and the support maps,
        the concatenation never materialised (one product per layer segment, accumulated);
        differentiable (cwt_linear_backward per segment) under autograd."""
        outs = []
        weight = self.adjust_feature[0].weight
        for lst in (fq_lst, fs_lst):
            feats = [as_tokens(self._layer(lst, lid)) for lid in self.layers_used]
            if _needs_grad(weight, *feats):
                outs.append(_AdjustFn.apply(self, weight, *feats))
            else:
                outs.append(self._adjust(feats))
        return outs[0], outs[1]

    def forward(self, fq_lst, fs_lst, f_q, f_s, padding_mask=None, s_padding_mask=None):
        if padding_mask is not None or s_padding_mask is not None:
            raise NotImplementedError("DeTr: padding masks are not built (train_trans.py passes None)")
        fq_fea, fs_fea = self.compute_feat(fq_lst, fs_lst)
        sa_fq = ca_fq = None
        if self.cs_att:
            ca_fq = self.cross_trans(fq_fea, fs_fea, f_s, ig_mask=None, ret_corr=False)
            f_q = norm_blend(f_q, ca_fq, self.att_wt)
        if self.sf_att:
            sa_fq = self.self_trans(fq_fea, f_q, padding_mask=padding_mask)
            f_q = norm_blend(f_q, sa_fq, self.att_wt)
        return f_q, sa_fq, ca_fq

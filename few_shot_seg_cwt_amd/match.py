"""MatchNet, the 4-D matching head of the MMN / MatchNet variants, on
HIP kernels (csrc/match.hip) behind the C ABI:

  MutualMatching(corr4d)                      src/model/match.py:21-53
  NeighConsensus(kernel_sizes, channels, ...)  src/model/match.py:56-85  (CenterPivotConv4d layers,
                                               src/model/conv4d.py:11-62, or Conv4d layers,
                                               conv4d.py:64-138)
  MatchNet(temp, cv_type, in_channel, ...)     src/model/match.py:88-163 (forward, corr_forward,
                                               run_match_model)
  WeightAverage(c_in, args)                    src/model/msm/msm_func.py:50-104
  MMN(args, agg, wa, red_dim)                  src/model/mmn.py:11-71 (forward)

Training (round 4): under autograd (grad enabled and a parameter or input
requiring grad) MatchNet.corr_forward / forward ('red' layers), get_corr, WeightAverage and the
MMN head (agg 'cat' or 'sum', red_dim) run their backward on the device --
cwt_match_corr_backward (softmax readout, both MutualMatchings with torch.max's single-index
gradient routing, the CenterPivotConv4d layers' input / weight / bias gradients over both
symmetric branches), cwt_corr_backward, cwt_weight_average_backward, cwt_mmn_blend_backward
(csrc/match_bwd.hip) -- so the MMN trainers (train_cca.py:101-196, train_aug.py:102) and DeTr's
cross attention (train_trans.py:100) can train this head.  Round 5: MatchNet.forward's backward
with ig_mask and the cycle mask (train_tp_match.py:188, train_match.py:164 use_cyc; the mask's
train-mode Dropout(0.1) drawn on the device), cwt_match_readout_backward, and the spatial context
encoder's weight / bias gradients (train_match.py:104 sce=args.sce).

The modules keep the reference's parameter names (``NeighConsensus.conv.{0,2,4}.conv{1,2}.
{weight,bias}``), so a reference state_dict loads as is.  Built: the default head of every MMN /
MatchNet script -- CenterPivotConv4d ('red'), kernel sizes [3, 3, 3], channels [10, 10, 1],
in_channel 1 or 2, symmetric or not -- and the MMN head of the mmn configs (rmid 'l34', all_lr
'l', agg 'cat', wa True, red_dim False), forward only (inference), with MatchNet.forward's ig_mask and (round 3) its
cycle-consistency mask (cyc; training mode since round 5), and NeighConsensus over full Conv4d layers ('cv4',
fp32 VALU), the spatial context encoder (sce, spatial_context.py), and MMN's agg 'sum' and red_dim.
Not built: forward_mmn (its MSBlock) and the MMN trainers' backward.

Parity is unpinned: the reference cannot be run here and holds no fixtures for
this head; tests/test_gpu_match.py checks it against oracle/match_oracle.py, a float64
restatement of the same modules.
"""
from __future__ import annotations

import ctypes as C
import math

import torch
import torch.nn.functional as F

from . import _lib
from .heads import get_corr
from .transformer import as_tokens
from .util import dropout_seed


def MutualMatching(corr4d: torch.Tensor) -> torch.Tensor:
    """match.py:21-53: corr4d [B, C, ha, wa, hb, wb] -> same shape, each channel scaled by its
    ratios to the max over the query positions and over the support positions."""
    _lib.require(corr4d, "corr4d")
    B, C, ha, wa, hb, wb = corr4d.shape
    NA, NB = ha * wa, hb * wb
    x = corr4d.reshape(B, C, NA, NB).permute(0, 2, 3, 1).contiguous()   # channels last
    y = torch.empty_like(x)
    _lib.check(_lib.lib().cwt_mutual_matching(_lib.ctx(x.device.index), _lib.ptr(x), B, NA, NB, C, _lib.ptr(y),
                                              _lib.stream_ptr(x.device)), "cwt_mutual_matching")
    return y.permute(0, 3, 1, 2).reshape(B, C, ha, wa, hb, wb)


class CenterPivotConv4d(torch.nn.Module):
    """conv4d.py:11-62 parameter holder (conv1 over the first position pair, conv2 over the
    second), stride 1, kernel 3, padding 1; the layer runs inside NeighConsensus's fused path."""

    def __init__(self, in_channels: int, out_channels: int, kernel_size=(3,) * 4, padding=(1,) * 4,
                 stride=(1,) * 4, bias: bool = True, device=None):
        super().__init__()
        if tuple(kernel_size) != (3,) * 4 or tuple(padding) != (1,) * 4 or tuple(stride) != (1,) * 4 or not bias:
            raise NotImplementedError("CenterPivotConv4d: kernel 3, padding 1, stride 1, bias only")
        self.conv1 = torch.nn.Conv2d(in_channels, out_channels, 3, padding=1, bias=True, device=device)
        self.conv2 = torch.nn.Conv2d(in_channels, out_channels, 3, padding=1, bias=True, device=device)


class Conv4d(torch.nn.Module):
    """conv4d.py:101-138 parameter holder: ``weight`` in the reference's pre-permuted layout
    [k0][co][ci][k1][k2][k3] (Conv4d permutes it in its constructor, so a reference state_dict
    holds that layout), ``bias`` [co]; _ConvNd's default initialisation on [co][ci][3][3][3][3].
    Kernel 3, padding 1, stride 1; the layer runs inside NeighConsensus's device path."""

    def __init__(self, in_channels: int, out_channels: int, kernel_size=(3,) * 4, padding=(1,) * 4, bias: bool = True,
                 pre_permuted_filters: bool = True, device=None):
        super().__init__()
        if tuple(kernel_size) != (3,) * 4 or tuple(padding) != (1,) * 4 or not bias or not pre_permuted_filters:
            raise NotImplementedError("Conv4d: kernel 3, padding 1, bias, pre-permuted filters only")
        w = torch.empty(out_channels, in_channels, 3, 3, 3, 3)
        torch.nn.init.kaiming_uniform_(w, a=math.sqrt(5))
        bound = 1.0 / math.sqrt(in_channels * 81)
        self.weight = torch.nn.Parameter(w.permute(2, 0, 1, 3, 4, 5).contiguous().to(device))
        self.bias = torch.nn.Parameter(torch.empty(out_channels).uniform_(-bound, bound).to(device))
        self.pre_permuted_filters = True


class NeighConsensus(torch.nn.Module):
    """match.py:56-85 with the default geometry: three 4-D conv + ReLU layers, channels
    in_channel -> 10 -> 10 -> 1, symmetric mode conv(x) + conv(x^T)^T.  ``conv`` defaults to
    'cv4' (full Conv4d) as the reference signature does (match.py:57); MatchNet passes its
    config's cv_type ('red' = CenterPivotConv4d in every reference config)."""

    def __init__(self, kernel_sizes=(3, 3, 3), channels=(10, 10, 1), symmetric_mode: bool = True, conv: str = "cv4",
                 in_channel: int = 1, device=None):
        super().__init__()
        if conv not in ("red", "cv4"):
            raise ValueError(f"NeighConsensus: conv must be 'red' or 'cv4' (match.py:15), got {conv!r}")
        self.conv_type = conv
        if tuple(kernel_sizes) != (3, 3, 3) or tuple(channels) != (10, 10, 1) or in_channel not in (1, 2):
            raise NotImplementedError("NeighConsensus: kernel sizes [3,3,3], channels [10,10,1], in_channel 1 or 2")
        self.symmetric_mode = symmetric_mode
        self.kernel_sizes = list(kernel_sizes)
        self.channels = list(channels)
        self.in_channel = in_channel
        mods = []
        ch_in = in_channel
        for ch_out in channels:
            layer = Conv4d(ch_in, ch_out, device=device) if conv == "cv4" else CenterPivotConv4d(ch_in, ch_out,
                                                                                                  device=device)
            mods += [layer, torch.nn.ReLU(inplace=True)]
            ch_in = ch_out
        self.conv = torch.nn.Sequential(*mods)
        self._packed, self._packed_key = None, None

    def param_list(self):
        """The layers' parameters in cwt_match_corr_forward's order."""
        ps = []
        for i in (0, 2, 4):
            layer = self.conv[i]
            if self.conv_type == "cv4":
                ps += [layer.weight, layer.bias]
            else:
                ps += [layer.conv1.weight, layer.conv1.bias, layer.conv2.weight, layer.conv2.bias]
        return ps

    def packed(self) -> torch.Tensor:
        """The layers' parameters in cwt_match_corr_forward's order (cached per parameter version)."""
        ps = []
        for i in (0, 2, 4):
            layer = self.conv[i]
            if self.conv_type == "cv4":
                ps += [layer.weight, layer.bias]
            else:
                ps += [layer.conv1.weight, layer.conv1.bias, layer.conv2.weight, layer.conv2.bias]
        key = tuple((p.data_ptr(), p._version) for p in ps)
        if self._packed is None or key != self._packed_key:
            with torch.no_grad():
                self._packed = torch.cat([p.detach().reshape(-1).float() for p in ps]).contiguous()
            self._packed_key = key
        return self._packed


class SpatialContextEncoder(torch.nn.Module):
    """src/model/base/spatial_context.py:68-110: x [B, C, h, w] -> relu(conv1x1(cat(x,
    featureL2Norm(generate_spatial_descriptor(x, k))))) [B, hidden, h, w].  The descriptor on
    the device (cwt_sce_descriptor), the 1x1 conv as two accumulated f32-MFMA GEMMs over the
    concatenation's two segments (detr.linear), the descriptor segment padded to a multiple of 4
    columns with zero weights.  Keeps the reference's ``embeddingFea.0.{weight,bias}``."""

    def __init__(self, kernel_size: int = 25, input_dim: int = 25 * 25 + 2048, hidden_dim: int = 2048, device=None):
        super().__init__()
        self.kernel_size = kernel_size
        self.embeddingFea = torch.nn.Sequential(torch.nn.Conv2d(input_dim, hidden_dim, 1, padding=0, device=device),
                                                torch.nn.ReLU(inplace=True))
        self._wsplit, self._wkey = None, None

    def _weights(self, C: int, ldg: int):
        conv = self.embeddingFea[0]
        key = (conv.weight.data_ptr(), conv.weight._version, C, ldg)
        if self._wsplit is None or key != self._wkey:
            with torch.no_grad():
                W = conv.weight.detach().reshape(conv.weight.shape[0], -1).float()
                k2 = self.kernel_size ** 2
                if W.shape[1] != C + k2:
                    raise ValueError(f"SpatialContextEncoder: input_dim {W.shape[1]} != C + k^2 = {C + k2}")
                wg = torch.zeros((W.shape[0], ldg), device=W.device, dtype=torch.float32)
                wg[:, :k2] = W[:, C:]
                self._wsplit = (W[:, :C].contiguous(), wg.contiguous())
            self._wkey = key
        return self._wsplit

    def _descriptor(self, xt: torch.Tensor, ldg: int) -> torch.Tensor:
        B, C, h, w = xt.shape
        g = torch.empty((B * h * w, ldg), device=xt.device, dtype=torch.float32)
        _lib.check(_lib.lib().cwt_sce_descriptor(_lib.ctx(xt.device.index), _lib.ptr(xt), B, h, w, C, self.kernel_size,
                                                 ldg, _lib.ptr(g), _lib.stream_ptr(xt.device)), "cwt_sce_descriptor")
        return g

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        from .detr import linear
        conv = self.embeddingFea[0]
        if torch.is_grad_enabled() and x.requires_grad:
            # the reference writes the descriptor into a leaf Variable created with x's requires_grad
            # (spatial_context.py:32-53): torch refuses that in-place write, so the encoder has no
            # gradient path into x there either
            raise RuntimeError("SpatialContextEncoder: x requiring grad (the reference's generate_spatial_descriptor "
                               "cannot run on it)")
        xt = as_tokens(x)
        if _needs_grad(conv.weight, conv.bias):   # train_match.py with sce: the embedding trains
            return _SceFn.apply(xt, conv.weight, conv.bias, self)
        with torch.no_grad():
            B, C, h, w = xt.shape
            ldg = (self.kernel_size ** 2 + 3) & ~3
            g = self._descriptor(xt, ldg)
            wx, wg = self._weights(C, ldg)
            tok = xt.permute(0, 2, 3, 1).reshape(B * h * w, C)   # a view of the NHWC storage
            out = linear(tok, wx)
            linear(g, wg, conv.bias, relu=True, out=out, accumulate=True)
            return out.reshape(B, h, w, -1).permute(0, 3, 1, 2)


class _SceFn(torch.autograd.Function):
    """SpatialContextEncoder under autograd (the 1x1 conv's weight and bias train; the input and
    its descriptor carry no gradient, as in the reference): out = relu([x | g] W^T + b); backward
    by cwt_linear_backward over the two segments of the concatenation, the ReLU mask from out."""

    @staticmethod
    def forward(ctx, xt, weight, bias, enc):
        from .detr import linear
        B, C, h, w = xt.shape
        ldg = (enc.kernel_size ** 2 + 3) & ~3
        g = enc._descriptor(xt, ldg)
        wx, wg = enc._weights(C, ldg)
        tok = xt.permute(0, 2, 3, 1).reshape(B * h * w, C)
        out = linear(tok, wx)
        linear(g, wg, bias, relu=True, out=out, accumulate=True)
        ctx.save_for_backward(tok, g, wx, wg, out)
        ctx.meta = (weight.shape, enc.kernel_size ** 2, bias is not None)
        return out.reshape(B, h, w, -1).permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, d):
        tok, g, wx, wg, out = ctx.saved_tensors
        wshape, k2, has_b = ctx.meta
        P, C = tok.shape
        N, ldg = wg.shape
        dt = d.permute(0, 2, 3, 1).reshape(P, N).contiguous()
        dev = tok.device
        dwx = torch.empty((N, C), device=dev, dtype=torch.float32)
        dwg = torch.empty((N, ldg), device=dev, dtype=torch.float32)
        db = torch.empty(N, device=dev, dtype=torch.float32) if has_b else None
        L, cx, st = _lib.lib(), _lib.ctx(dev.index), _lib.stream_ptr(dev)
        _lib.check(L.cwt_linear_backward(cx, _lib.ptr(tok), P, C, _lib.ptr(wx), N, _lib.ptr(out), _lib.ptr(dt), None,
                                         _lib.ptr(dwx), C, None, st), "cwt_linear_backward")
        _lib.check(L.cwt_linear_backward(cx, _lib.ptr(g), P, ldg, _lib.ptr(wg), N, _lib.ptr(out), _lib.ptr(dt), None,
                                         _lib.ptr(dwg), ldg, _lib.ptr(db), st), "cwt_linear_backward")
        dw = torch.cat([dwx, dwg[:, :k2]], 1).reshape(wshape)
        return None, dw, db, None


class _MatchCorrFn(torch.autograd.Function):
    """MatchNet.corr_forward ('red' layers) under autograd: cwt_match_corr_forward_train keeps the
    activations, cwt_match_corr_backward runs the whole chain's backward on the device."""

    @staticmethod
    def forward(ctx, corr, vt, symmetric, temp, h, w, *params):
        # corr [B, L, hw, hw] contiguous; vt [B, Cv, h, w] token-contiguous (channels_last) or None
        B, L = corr.shape[0], corr.shape[1]
        hw, dev = h * w, corr.device
        with torch.no_grad():
            packed = torch.cat([p.detach().reshape(-1).float() for p in params]).contiguous()
        n = C.c_int64()
        _lib.check(_lib.lib().cwt_match_corr_saved_floats(B, L, h, w, int(symmetric), int(vt is not None), C.byref(n)),
                   "cwt_match_corr_saved_floats")
        saved = torch.empty(n.value, device=dev, dtype=torch.float32)
        corr2d = torch.empty((B, hw, hw), device=dev, dtype=torch.float32)
        Cv = vt.shape[1] if vt is not None else 0
        wv = torch.empty((B, h, w, Cv), device=dev, dtype=torch.float32) if vt is not None else None
        _lib.check(_lib.lib().cwt_match_corr_forward_train(
            _lib.ctx(dev.index), _lib.ptr(corr), B, L, h, w, _lib.ptr(packed), int(symmetric), float(temp),
            _lib.ptr(vt), Cv, _lib.ptr(corr2d), _lib.ptr(wv), _lib.ptr(saved), _lib.stream_ptr(dev)),
            "cwt_match_corr_forward_train")
        ctx.save_for_backward(corr, vt if vt is not None else corr.new_empty(0), packed, saved)
        ctx.meta = (h, w, int(symmetric), float(temp), vt is not None)
        ctx.shapes = [p.shape for p in params]
        return corr2d, (wv.permute(0, 3, 1, 2) if wv is not None else corr.new_empty(0))

    @staticmethod
    def backward(ctx, g_corr2d, g_wv):
        corr, vt, packed, saved = ctx.saved_tensors
        h, w, sym, temp, has_v = ctx.meta
        B, L = corr.shape[0], corr.shape[1]
        dev = corr.device
        gw = g_wv.permute(0, 2, 3, 1).contiguous() if (has_v and g_wv is not None and g_wv.numel()) else None
        Cv = vt.shape[1] if has_v else 0
        d_corr = torch.empty_like(corr) if ctx.needs_input_grad[0] else None
        d_v = (torch.empty((B, h, w, Cv), device=dev, dtype=torch.float32)
               if (has_v and gw is not None and ctx.needs_input_grad[1]) else None)
        d_params = torch.empty_like(packed)
        gc = g_corr2d.contiguous() if g_corr2d is not None else None
        _lib.check(_lib.lib().cwt_match_corr_backward(
            _lib.ctx(dev.index), _lib.ptr(corr), B, L, h, w, _lib.ptr(packed), sym, temp,
            _lib.ptr(vt) if has_v else None, Cv, _lib.ptr(saved), _lib.ptr(gc), _lib.ptr(gw), _lib.ptr(d_corr),
            _lib.ptr(d_params), _lib.ptr(d_v), _lib.stream_ptr(dev)), "cwt_match_corr_backward")
        sizes = [math.prod(s) for s in ctx.shapes]
        grads = [g.reshape(s) for g, s in zip(torch.split(d_params, sizes), ctx.shapes)]
        return (d_corr, d_v.permute(0, 3, 1, 2) if d_v is not None else None, None, None, None, None, *grads)


def _needs_grad(*ts) -> bool:
    return torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in ts)


class _MatchMaskedFn(torch.autograd.Function):
    """MatchNet.forward with the support masks (match.py:103-130: ig_mask and, with cyc, the cycle
    mask) under autograd ('red' layers).  Forward: cwt_match_corr_forward_train (the chain,
    activations kept) -> cwt_match_masks_train on a copy of corr2d -> cwt_match_readout.  Backward:
    cwt_match_readout_backward (softmax readout, then the ig-masked columns zeroed: the reference
    overwrote them with a constant) -> cwt_match_corr_backward through both MutualMatchings and the
    NeighConsensus layers.  The cycle mask is constant under autograd (argmax indices; its train-mode
    Dropout(0.1) draws one scale per support position, stream 5 of the counter-based draw)."""

    @staticmethod
    def forward(ctx, corr, vt, ig, sm, symmetric, temp, h, w, drop_p, seed, *params):
        B, L = corr.shape[0], corr.shape[1]
        hw, dev = h * w, corr.device
        Lb, cx, st = _lib.lib(), _lib.ctx(dev.index), _lib.stream_ptr(dev)
        with torch.no_grad():
            packed = torch.cat([p.detach().reshape(-1).float() for p in params]).contiguous()
        n = C.c_int64()
        _lib.check(Lb.cwt_match_corr_saved_floats(B, L, h, w, int(symmetric), 0, C.byref(n)),
                   "cwt_match_corr_saved_floats")
        saved = torch.empty(n.value, device=dev, dtype=torch.float32)
        corr2d = torch.empty((B, hw, hw), device=dev, dtype=torch.float32)
        _lib.check(Lb.cwt_match_corr_forward_train(cx, _lib.ptr(corr), B, L, h, w, _lib.ptr(packed), int(symmetric),
                                                   float(temp), None, 0, _lib.ptr(corr2d), None, _lib.ptr(saved), st),
                   "cwt_match_corr_forward_train")
        inc = torch.empty((B, hw), device=dev, dtype=torch.float32) if sm is not None else None
        _lib.check(Lb.cwt_match_masks_train(cx, _lib.ptr(corr2d), B, hw, hw, _lib.ptr(ig) if ig is not None else None,
                                            _lib.ptr(sm) if sm is not None else None,
                                            _lib.ptr(inc) if inc is not None else None, float(drop_p), int(seed), st),
                   "cwt_match_masks_train")
        Cv = vt.shape[1]
        wv = torch.empty((B, h, w, Cv), device=dev, dtype=torch.float32)
        _lib.check(Lb.cwt_match_readout(cx, _lib.ptr(corr2d), B, hw, hw, float(temp), _lib.ptr(vt), Cv, _lib.ptr(wv), st),
                   "cwt_match_readout")
        ctx.save_for_backward(corr, vt, packed, saved, corr2d, ig if ig is not None else corr.new_empty(0))
        ctx.meta = (h, w, int(symmetric), float(temp), ig is not None)
        ctx.shapes = [p.shape for p in params]
        if inc is None:
            inc = corr.new_empty(0)
        ctx.mark_non_differentiable(inc)
        return wv.permute(0, 3, 1, 2), corr2d, inc

    @staticmethod
    def backward(ctx, g_wv, g_corr2d, g_inc):
        corr, vt, packed, saved, corr2d, ig = ctx.saved_tensors
        h, w, sym, temp, has_ig = ctx.meta
        B, L = corr.shape[0], corr.shape[1]
        hw, dev = h * w, corr.device
        Lb, cx, st = _lib.lib(), _lib.ctx(dev.index), _lib.stream_ptr(dev)
        d2 = g_corr2d.contiguous().clone() if g_corr2d is not None else torch.zeros((B, hw, hw), device=dev)
        gw = g_wv.permute(0, 2, 3, 1).contiguous() if g_wv is not None else None
        Cv = vt.shape[1]
        d_v = (torch.empty((B, h, w, Cv), device=dev, dtype=torch.float32)
               if (gw is not None and ctx.needs_input_grad[1]) else None)
        if gw is not None or has_ig:
            _lib.check(Lb.cwt_match_readout_backward(cx, _lib.ptr(corr2d), B, hw, hw, temp, _lib.ptr(vt), Cv,
                                                     _lib.ptr(gw), _lib.ptr(ig) if has_ig else None, _lib.ptr(d2),
                                                     _lib.ptr(d_v), st), "cwt_match_readout_backward")
        d_corr = torch.empty_like(corr) if ctx.needs_input_grad[0] else None
        d_params = torch.empty_like(packed)
        _lib.check(Lb.cwt_match_corr_backward(cx, _lib.ptr(corr), B, L, h, w, _lib.ptr(packed), sym, temp, None, 0,
                                              _lib.ptr(saved), _lib.ptr(d2), None, _lib.ptr(d_corr),
                                              _lib.ptr(d_params), None, st), "cwt_match_corr_backward")
        sizes = [math.prod(s) for s in ctx.shapes]
        grads = [g.reshape(s) for g, s in zip(torch.split(d_params, sizes), ctx.shapes)]
        return (d_corr, d_v.permute(0, 3, 1, 2) if d_v is not None else None, None, None, None, None, None, None,
                None, None, *grads)


class MatchNet(torch.nn.Module):
    """match.py:88-163.  forward(fq_fea, fs_fea, v) and corr_forward(corr4d, v, ret_attn) on the
    device; v is the support feature map [B, Cv, h, w] (returned weighted_v has its shape)."""

    def __init__(self, temp: float = 3.0, cv_type: str = "red", in_channel: int = 1, sce: bool = False,
                 cyc: bool = False, sym_mode: bool = True, cv_kernels=(3, 3, 3), cv_channels=(10, 10, 1),
                 device=None):
        super().__init__()
        self.temp = temp
        self.sce, self.cyc = sce, cyc
        self.in_channel = in_channel
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        if sce:   # match.py:95-97
            self.SpatialContextEncoder = SpatialContextEncoder(kernel_size=25, input_dim=25 * 25 + 2048, hidden_dim=2048,
                                                               device=dev)
        self.NeighConsensus = NeighConsensus(kernel_sizes=cv_kernels, channels=cv_channels, symmetric_mode=sym_mode,
                                             conv=cv_type, in_channel=in_channel, device=dev)

    def _run(self, corr: torch.Tensor, h: int, w: int, v: torch.Tensor | None):
        """corr [B, L, hw, hw] contiguous -> (corr2d [B, hw, hw], weighted_v tokens or None)."""
        _lib.require(corr, "corr")
        B, L = corr.shape[0], corr.shape[1]
        if L != self.in_channel:
            raise ValueError("input corr channel inconsistent with in_channel of NCNet")
        hw = h * w
        nc = self.NeighConsensus
        # the backward is built for CenterPivotConv4d ('red') layers, the layers every config trains;
        # 'cv4' runs the inference kernels and its outputs carry no gradient
        if nc.conv_type == "red" and _needs_grad(corr, v, *nc.param_list()):
            vt = as_tokens(v if v.dim() == 4 else v.reshape(v.shape[0], v.shape[1], h, w)) if v is not None else None
            corr2d, wv = _MatchCorrFn.apply(corr.contiguous(), vt, nc.symmetric_mode, float(self.temp), h, w,
                                            *nc.param_list())
            return corr2d, (wv if v is not None else None)
        params = nc.packed()
        corr2d = torch.empty((B, hw, hw), device=corr.device, dtype=torch.float32)
        wv, vt, Cv = None, None, 0
        if v is not None:
            vt = as_tokens(v if v.dim() == 4 else v.reshape(v.shape[0], v.shape[1], h, w))
            Cv = vt.shape[1]
            wv = torch.empty((B, h, w, Cv), device=corr.device, dtype=torch.float32)
        entry = "cwt_match_corr_forward_cv4" if self.NeighConsensus.conv_type == "cv4" else "cwt_match_corr_forward"
        _lib.check(getattr(_lib.lib(), entry)(
            _lib.ctx(corr.device.index), _lib.ptr(corr), B, L, h, w, _lib.ptr(params),
            1 if self.NeighConsensus.symmetric_mode else 0, float(self.temp),
            _lib.ptr(vt) if vt is not None else None, Cv, _lib.ptr(corr2d), _lib.ptr(wv) if wv is not None else None,
            _lib.stream_ptr(corr.device)), entry)
        return corr2d, (wv.permute(0, 3, 1, 2) if wv is not None else None)

    def run_match_model(self, corr4d: torch.Tensor) -> torch.Tensor:
        """match.py:159-163: corr4d [B, L, h, w, h, w] -> [B, 1, h, w, h, w]."""
        B, L, h, w = corr4d.shape[:4]
        corr2d, _ = self._run(corr4d.reshape(B, L, h * w, h * w).contiguous(), h, w, None)
        return corr2d.reshape(B, 1, h, w, h, w)

    def corr_forward(self, corr4d: torch.Tensor, v: torch.Tensor, ret_attn: bool = False):
        """match.py:142-157 (returns weighted_v [B, Cv, h, w]; with ret_attn (corr2d, weighted_v))."""
        B, ch, h, w = corr4d.shape[:4]
        assert ch == self.in_channel, "input corr channel inconsistent with in_channel of NCNet"
        corr2d, wv = self._run(corr4d.reshape(B, ch, h * w, h * w).contiguous(), h, w, v)
        return (corr2d, wv) if ret_attn else wv

    def forward(self, fq_fea, fs_fea, v, s_mask=None, ig_mask=None, ret_corr=False, use_cyc=False, ret_cyc=False):
        """match.py:103-140: normalised features (-> the spatial context encoder with ``sce``) ->
        get_corr -> run_match_model ->
        the ig mask and, with ``cyc`` and ``use_cyc``, the cycle-consistency mask (run_cyc,
        match.py:165-182; cwt_match_masks) -> softmax(temp * corr2d) -> v . attn^T
        (cwt_match_readout).  Returns as the reference: weighted_v, plus corr2d [B, h, w, h, w]
        with ret_corr, plus the inconsistent mask [B, 1, h*w] with ret_cyc."""
        B, ch, h, w = fq_fea.shape
        hw = h * w
        if self.sce:   # match.py:108-113: F.normalize, then the encoder on both maps
            from .detr import norm_blend
            fq_fea = self.SpatialContextEncoder(norm_blend(fq_fea, fq_fea, 0.0))   # normalize(a) + normalize(a) * 0
            fs_fea = self.SpatialContextEncoder(norm_blend(fs_fea, fs_fea, 0.0))
        corr = get_corr(fq_fea, fs_fea)   # normalises both (the reference's F.normalize first is the same map)
        cyc_on = bool(self.cyc and use_cyc)
        if ig_mask is None and not cyc_on:
            if ret_cyc:   # the reference reads an unbound inconsistent_mask here
                raise UnboundLocalError("ret_cyc needs the cycle mask (cyc=True and use_cyc=True)")
            corr2d, wv = self._run(corr.reshape(B, 1, hw, hw), h, w, v)
            return (wv, corr2d.reshape(B, h, w, h, w)) if ret_corr else wv
        if cyc_on and s_mask is None:   # run_cyc returns None and the reference fails on it
            raise ValueError("the cycle mask needs s_mask")
        # train mode: run_cyc's ass_drop = nn.Dropout(0.1) on the mask (match.py:97,181), one counter
        # draw per call.  The reference's nn.Dropout on a CUDA tensor draws from the CUDA generator and
        # never moves the host RNG stream (the W0 draws), so the seed comes from util.dropout_seed
        drop_p = 0.1 if (cyc_on and self.training) else 0.0
        seed = dropout_seed() if drop_p > 0 else 0
        dev = corr.device
        ig = None
        if ig_mask is not None:
            if ig_mask.numel() != B * hw:
                raise ValueError("ig_mask must hold B * h * w entries (ig_mask.view(B, -1, h*w))")
            ig = ig_mask.reshape(B, hw).to(device=dev, dtype=torch.uint8).contiguous()
        sm, inc = None, None
        if cyc_on:
            if s_mask.numel() != B * hw:
                raise ValueError("s_mask must hold B * h * w entries (s_mask.view(B, n_s))")
            sm = s_mask.reshape(B, hw).to(device=dev, dtype=torch.int64).contiguous()
        nc = self.NeighConsensus
        vt = as_tokens(v if v.dim() == 4 else v.reshape(v.shape[0], v.shape[1], h, w))
        if nc.conv_type == "red" and _needs_grad(corr, vt, *nc.param_list()):
            wv, corr2d, inc = _MatchMaskedFn.apply(corr.reshape(B, 1, hw, hw).contiguous(), vt, ig, sm,
                                                   nc.symmetric_mode, float(self.temp), h, w, drop_p, seed,
                                                   *nc.param_list())
            out = [wv]
            if ret_corr:
                out.append(corr2d.reshape(B, h, w, h, w))
            if ret_cyc:
                if sm is None:
                    raise UnboundLocalError("ret_cyc needs the cycle mask (cyc=True and use_cyc=True)")
                out.append(inc.unsqueeze(1))
            return out[0] if len(out) == 1 else tuple(out)
        corr2d, _ = self._run(corr.reshape(B, 1, hw, hw), h, w, None)
        if cyc_on:
            inc = torch.empty((B, hw), device=dev, dtype=torch.float32)
        _lib.check(_lib.lib().cwt_match_masks_train(
            _lib.ctx(dev.index), _lib.ptr(corr2d), B, hw, hw, _lib.ptr(ig) if ig is not None else None,
            _lib.ptr(sm) if sm is not None else None, _lib.ptr(inc) if inc is not None else None, float(drop_p), seed,
            _lib.stream_ptr(dev)), "cwt_match_masks_train")
        Cv = vt.shape[-1] if vt.dim() == 3 else vt.shape[1]
        wv = torch.empty((B, h, w, Cv), device=dev, dtype=torch.float32)
        _lib.check(_lib.lib().cwt_match_readout(
            _lib.ctx(dev.index), _lib.ptr(corr2d), B, hw, hw, float(self.temp), _lib.ptr(vt), Cv, _lib.ptr(wv),
            _lib.stream_ptr(dev)), "cwt_match_readout")
        wv = wv.permute(0, 3, 1, 2)
        out = [wv]
        if ret_corr:
            out.append(corr2d.reshape(B, h, w, h, w))
        if ret_cyc:
            if inc is None:
                raise UnboundLocalError("ret_cyc needs the cycle mask (cyc=True and use_cyc=True)")
            out.append(inc.unsqueeze(1))
        return out[0] if len(out) == 1 else tuple(out)


def init_match_params(mod: torch.nn.Module, seed: int = 0) -> None:
    """Deterministic parameters for tests / benchmarks (nn.Conv2d's default init bounds)."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for name, p in mod.named_parameters():
            fan_in = p.shape[1] * p.shape[2] * p.shape[3] if p.dim() == 4 else (p.shape[2] * 81 if p.dim() == 6 else 100)
            bound = 1.0 / math.sqrt(fan_in)
            p.copy_((torch.rand(p.shape, generator=g, dtype=torch.float32) * 2 - 1) * bound)


class WeightAverage(torch.nn.Module):
    """msm_func.py:50-104 (R = 3): x + conv_back(softmax-weighted g over the 3x3 replicate-padded
    neighbourhood, weights = cosine similarity of phi(neighbour) and theta(x)).  Parameter names
    conv_theta / conv_phi / conv_g / conv_back as the reference."""

    def __init__(self, c_in: int, args=None, R: int = 3, device=None):
        super().__init__()
        if R != 3:
            raise NotImplementedError("WeightAverage: R = 3 only")
        for k in ("att_drop", "proj_drop"):
            p = (args.get(k, 0.0) if isinstance(args, dict) else getattr(args, k, 0.0)) if args is not None else 0.0
            if p:
                raise NotImplementedError("WeightAverage: att_drop / proj_drop are identities here (eval)")
        c_out = c_in // 2
        self.c_in, self.c_out, self.R = c_in, c_out, R
        self.conv_theta = torch.nn.Conv2d(c_in, c_out, 1, device=device)
        self.conv_phi = torch.nn.Conv2d(c_in, c_out, 1, device=device)
        self.conv_g = torch.nn.Conv2d(c_in, c_out, 1, device=device)
        self.conv_back = torch.nn.Conv2d(c_out, c_in, 1, device=device)
        self._w, self._key = None, None

    def _weights(self):
        ps = [self.conv_theta.weight, self.conv_phi.weight, self.conv_g.weight, self.conv_back.weight]
        key = tuple((p.data_ptr(), p._version) for p in ps)
        if self._w is None or key != self._key:
            with torch.no_grad():
                tpg = torch.cat([p.detach().reshape(self.c_out, self.c_in) for p in ps[:3]]).contiguous()
                back = ps[3].detach().reshape(self.c_in, self.c_out).contiguous()
            self._w, self._key = (tpg, back), key
        return self._w

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        _lib.require(x, "x")
        N, C, h, w = x.shape
        if C != self.c_in:
            raise ValueError(f"expected {self.c_in} channels, got {C}")
        xt = as_tokens(x)
        ps = [self.conv_theta.weight, self.conv_theta.bias, self.conv_phi.weight, self.conv_phi.bias,
              self.conv_g.weight, self.conv_g.bias, self.conv_back.weight, self.conv_back.bias]
        if _needs_grad(xt, *ps):
            return _WeightAverageFn.apply(xt, *ps)
        tpg, back = self._weights()
        out = torch.empty((N, C, h, w), device=x.device, dtype=torch.float32, memory_format=torch.channels_last)
        _lib.check(_lib.lib().cwt_weight_average(
            _lib.ctx(x.device.index), _lib.ptr(xt), N, h, w, C, _lib.ptr(tpg), _lib.ptr(self.conv_theta.bias),
            _lib.ptr(self.conv_phi.bias), _lib.ptr(self.conv_g.bias), _lib.ptr(back), _lib.ptr(self.conv_back.bias),
            _lib.ptr(out), _lib.stream_ptr(x.device)), "cwt_weight_average")
        return out


class _WeightAverageFn(torch.autograd.Function):
    """WeightAverage under autograd: cwt_weight_average_train keeps theta | phi | g and the
    weighted average, cwt_weight_average_backward forms every gradient on the device."""

    @staticmethod
    def forward(ctx, xt, wt, bt, wp, bp, wg, bg, wb, bb):
        N, Cc, h, w = xt.shape
        co = Cc // 2
        dev = xt.device
        with torch.no_grad():
            tpg_w = torch.cat([p.detach().reshape(co, Cc) for p in (wt, wp, wg)]).contiguous()
            back = wb.detach().reshape(Cc, co).contiguous()
        out = torch.empty((N, Cc, h, w), device=dev, dtype=torch.float32, memory_format=torch.channels_last)
        tpg = torch.empty((N * h * w, 3 * co), device=dev, dtype=torch.float32)
        wavg = torch.empty((N * h * w, co), device=dev, dtype=torch.float32)
        _lib.check(_lib.lib().cwt_weight_average_train(
            _lib.ctx(dev.index), _lib.ptr(xt), N, h, w, Cc, _lib.ptr(tpg_w), _lib.ptr(bt), _lib.ptr(bp), _lib.ptr(bg),
            _lib.ptr(back), _lib.ptr(bb), _lib.ptr(out), _lib.ptr(tpg), _lib.ptr(wavg), _lib.stream_ptr(dev)),
            "cwt_weight_average_train")
        ctx.save_for_backward(xt, tpg_w, bt, bp, bg, back, tpg, wavg)
        return out

    @staticmethod
    def backward(ctx, d_out):
        xt, tpg_w, bt, bp, bg, back, tpg, wavg = ctx.saved_tensors
        N, Cc, h, w = xt.shape
        co = Cc // 2
        dev = xt.device
        d = as_tokens(d_out)
        dx = torch.empty_like(xt) if ctx.needs_input_grad[0] else None
        f = dict(device=dev, dtype=torch.float32)
        d_wtpg, d_bt, d_bp, d_bg = torch.empty((3 * co, Cc), **f), torch.empty(co, **f), torch.empty(co, **f), \
            torch.empty(co, **f)
        d_wb, d_bb = torch.empty((Cc, co), **f), torch.empty(Cc, **f)
        _lib.check(_lib.lib().cwt_weight_average_backward(
            _lib.ctx(dev.index), _lib.ptr(xt), N, h, w, Cc, _lib.ptr(tpg_w), _lib.ptr(bt), _lib.ptr(bp), _lib.ptr(bg),
            _lib.ptr(back), _lib.ptr(tpg), _lib.ptr(wavg), _lib.ptr(d), _lib.ptr(dx), _lib.ptr(d_wtpg), _lib.ptr(d_bt),
            _lib.ptr(d_bp), _lib.ptr(d_bg), _lib.ptr(d_wb), _lib.ptr(d_bb), _lib.stream_ptr(dev)),
            "cwt_weight_average_backward")
        wshape = (co, Cc, 1, 1)
        return (dx, d_wtpg[:co].reshape(wshape), d_bt, d_wtpg[co:2 * co].reshape(wshape), d_bp,
                d_wtpg[2 * co:].reshape(wshape), d_bg, d_wb.reshape(Cc, co, 1, 1), d_bb)


class _MMNCorrFn(torch.autograd.Function):
    """MMN's stacked correlations (mmn.py:44-58, agg 'cat') under autograd: corr4d[b, l] =
    get_corr(fq_l[b or 0], fs_l[b]); the backward is cwt_corr_backward per (b, l), a query feature
    shared by the B support rows (fq expanded, mmn.py:50) accumulating its B gradients in order."""

    @staticmethod
    def forward(ctx, B, L, agg_sum, *feats):
        h, w = feats[0].shape[2], feats[0].shape[3]
        P = h * w
        dev = feats[0].device
        corr4d = torch.empty((B, L, P, P), device=dev, dtype=torch.float32)
        for li in range(L):
            q, k = feats[2 * li], feats[2 * li + 1]
            for b in range(B):
                qb = q[:1] if q.shape[0] == 1 else q[b:b + 1]
                _lib.check(_lib.lib().cwt_corr(_lib.ctx(dev.index), _lib.ptr(qb), _lib.ptr(k[b:b + 1]), 1, P, P,
                                               q.shape[1], _lib.ptr(corr4d[b, li]), _lib.stream_ptr(dev)), "cwt_corr")
        ctx.save_for_backward(*feats)
        ctx.BL = (B, L, agg_sum)
        if agg_sum:   # mmn.py:62-63: the layers' correlations summed into one channel
            summed = torch.empty((B, 1, P, P), device=dev, dtype=torch.float32)
            _lib.check(_lib.lib().cwt_channel_sum(_lib.ctx(dev.index), _lib.ptr(corr4d), B, L, P * P, _lib.ptr(summed),
                                                  _lib.stream_ptr(dev)), "cwt_channel_sum")
            return summed
        return corr4d

    @staticmethod
    def backward(ctx, g):
        feats = ctx.saved_tensors
        B, L, agg_sum = ctx.BL
        g = g.contiguous()   # agg 'sum': every layer's correlation receives the summed channel's gradient
        h, w = feats[0].shape[2], feats[0].shape[3]
        P = h * w
        dev = feats[0].device
        grads = []
        for li in range(L):
            q, k = feats[2 * li], feats[2 * li + 1]
            nq, nk = ctx.needs_input_grad[3 + 2 * li], ctx.needs_input_grad[4 + 2 * li]
            dq = torch.empty_like(q) if nq else None
            dk = torch.empty_like(k) if nk else None
            if nq or nk:
                for b in range(B):
                    shared = q.shape[0] == 1
                    qi = 0 if shared else b
                    _lib.check(_lib.lib().cwt_corr_backward(
                        _lib.ctx(dev.index), _lib.ptr(q[qi:qi + 1]), _lib.ptr(k[b:b + 1]), 1, P, P, q.shape[1],
                        _lib.ptr(g[b, 0 if agg_sum else li]), _lib.ptr(dq[qi:qi + 1]) if nq else None,
                        _lib.ptr(dk[b:b + 1]) if nk else None, int(shared and b > 0), 0, _lib.stream_ptr(dev)),
                        "cwt_corr_backward")
            grads += [dq, dk]
        return (None, None, None, *grads)


class _MMNBlendFn(torch.autograd.Function):
    """mmn.py:65-67 under autograd (cwt_mmn_blend / cwt_mmn_blend_backward)."""

    @staticmethod
    def forward(ctx, fqt, att_t, att_wt):
        B = att_t.shape[0]
        dev = fqt.device
        att_fq = torch.empty(fqt.shape, device=dev, dtype=torch.float32, memory_format=torch.channels_last)
        fq = torch.empty_like(att_fq)
        _lib.check(_lib.lib().cwt_mmn_blend(_lib.ctx(dev.index), _lib.ptr(fqt), _lib.ptr(att_t), B, fqt.numel(),
                                            float(att_wt), _lib.ptr(att_fq), _lib.ptr(fq), _lib.stream_ptr(dev)),
                   "cwt_mmn_blend")
        ctx.meta = (B, float(att_wt), tuple(att_t.shape))
        return fq, att_fq

    @staticmethod
    def backward(ctx, d_fq, d_att_fq):
        B, att_wt, ashape = ctx.meta
        dfq = as_tokens(d_fq) if d_fq is not None else None
        dm = as_tokens(d_att_fq) if d_att_fq is not None else None
        ref = dfq if dfq is not None else dm
        dev = ref.device
        d_att = torch.empty(ashape, device=dev, dtype=torch.float32, memory_format=torch.channels_last)
        d_in = torch.empty_like(ref) if (ctx.needs_input_grad[0] and dfq is not None) else None
        _lib.check(_lib.lib().cwt_mmn_blend_backward(_lib.ctx(dev.index), _lib.ptr(dfq), _lib.ptr(dm), B, ref.numel(),
                                                     att_wt, _lib.ptr(d_att), _lib.ptr(d_in), _lib.stream_ptr(dev)),
                   "cwt_mmn_blend_backward")
        return d_in, d_att, None


def _get(args, k, default=None):
    if isinstance(args, dict):
        return args.get(k, default)
    return getattr(args, k, default)


class MMN(torch.nn.Module):
    """mmn.py:11-71: per-layer WeightAverage, the 4-D correlation of every (query, support)
    layer feature pair stacked as channels, MatchNet.corr_forward over it with v = f_s, and the
    blend fq = f_q * (1 - att_wt) + mean_shots(att_fq) * att_wt."""

    def __init__(self, args, agg: str = "cat", wa: bool = False, red_dim=False, device=None):
        super().__init__()
        if agg not in ("cat", "sum"):
            raise ValueError(f"MMN: agg must be 'cat' or 'sum', got {agg!r}")
        self.args, self.agg, self.wa, self.red_dim = args, agg, wa, red_dim
        rmid = str(_get(args, "rmid"))
        self.bid_lst = [int(c) for c in rmid[1:]]
        layers = int(_get(args, "layers", 50))
        self.nbottlenecks = [3, 4, 6, 3] if layers == 50 else [3, 4, 23, 3]
        self.feature_channels = [256, 512, 1024, 2048]
        all_lr = str(_get(args, "all_lr", "l"))
        if any(str(i) in all_lr for i in self.bid_lst):
            raise NotImplementedError("MMN: every-bottleneck features (all_lr naming a layer) are not built")
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        if wa or red_dim:   # mmn.py:26-33: the wa_ modules exist whenever red_dim does
            for bid in self.bid_lst:
                c_in = self.feature_channels[bid - 1]
                if isinstance(red_dim, int) and not isinstance(red_dim, bool) and red_dim:
                    setattr(self, "rd_" + str(bid),
                            torch.nn.Sequential(torch.nn.Conv2d(c_in, red_dim, 1, bias=False, device=dev),
                                                torch.nn.ReLU(inplace=True)))
                    c_in = red_dim
                setattr(self, "wa_" + str(bid), WeightAverage(c_in, args, device=dev))
        match_ch = 1 if agg == "sum" else len(self.bid_lst)
        self.att_wt = float(_get(args, "att_wt", 0.2))
        self.corr_net = MatchNet(temp=float(_get(args, "temp", 20.0)), cv_type=str(_get(args, "conv4d", "red")),
                                 sce=False, cyc=False, sym_mode=True, in_channel=match_ch, device=dev)

    def _reduce(self, idx: int, x: torch.Tensor) -> torch.Tensor:
        """rd_<layer>: 1x1 conv (no bias) + ReLU on the f32-MFMA GEMM (differentiable: linear_t)."""
        from .detr import linear_t
        conv = getattr(self, "rd_" + str(idx))[0]
        xt = as_tokens(x)
        N, C, h, w = xt.shape
        y = linear_t(xt.permute(0, 2, 3, 1).reshape(N * h * w, C), conv.weight, None, relu=True)
        return y.reshape(N, h, w, -1).permute(0, 3, 1, 2)

    def _forward_train(self, fq_lst, fs_lst, f_q, f_s, ret_attn: bool):
        """forward under autograd: red_dim's 1x1 conv + ReLU, WeightAverage, the stacked (or, agg
        'sum', summed) correlations, corr_forward and the blend as differentiable device ops."""
        B, ch, h, w = f_s.shape
        L = len(self.bid_lst)
        feats = []
        for idx in self.bid_lst[::-1]:
            fq_fea, fs_fea = fq_lst[idx][0], fs_lst[idx][0]
            if self.red_dim:
                fq_fea, fs_fea = self._reduce(idx, fq_fea), self._reduce(idx, fs_fea)
            if self.wa:
                m = getattr(self, "wa_" + str(idx))
                fq_fea, fs_fea = m(fq_fea), m(fs_fea)
            feats += [as_tokens(fq_fea), as_tokens(fs_fea)]
        corr4d = _MMNCorrFn.apply(B, L, self.agg == "sum", *feats)
        attn, att = self.corr_net._run(corr4d, h, w, f_s)
        fq, att_fq = _MMNBlendFn.apply(as_tokens(f_q), as_tokens(att), self.att_wt)
        return (attn, fq, att_fq) if ret_attn else (fq, att_fq)

    def forward(self, fq_lst, fs_lst, f_q, f_s, ret_attn: bool = False):
        """mmn.py:42-71: fq_lst / fs_lst {layer: [feature]} (extract_features with rmid),
        f_q [1, C, h, w], f_s [B, C, h, w] -> (fq, att_fq) [or (attn, fq, att_fq)].  Under
        autograd (a parameter or an input requiring grad) the backward runs on the device."""
        feats_in = [t for lst in (fq_lst, fs_lst) for idx in self.bid_lst for t in lst[idx][:1]]
        if _needs_grad(f_q, f_s, *feats_in, *self.parameters()):
            return self._forward_train(fq_lst, fs_lst, f_q, f_s, ret_attn)
        B, ch, h, w = f_s.shape
        P = h * w
        L = len(self.bid_lst)
        corr4d = torch.empty((B, L, P, P), device=f_s.device, dtype=torch.float32)
        for li, idx in enumerate(self.bid_lst[::-1]):
            fq_fea, fs_fea = fq_lst[idx][0], fs_lst[idx][0]
            if self.red_dim:   # rd_<layer>: 1x1 conv (no bias) + ReLU on the device GEMM
                fq_fea, fs_fea = self._reduce(idx, fq_fea), self._reduce(idx, fs_fea)
            if self.wa:
                m = getattr(self, "wa_" + str(idx))
                fq_fea, fs_fea = m(fq_fea), m(fs_fea)   # the query once: its B expanded copies are equal
            for b in range(B):
                qt, kt = as_tokens(fq_fea[:1] if fq_fea.shape[0] == 1 else fq_fea[b:b + 1]), as_tokens(fs_fea[b:b + 1])
                C = qt.shape[1]
                _lib.check(_lib.lib().cwt_corr(_lib.ctx(f_s.device.index), _lib.ptr(qt), _lib.ptr(kt), 1, P, P, C,
                                               _lib.ptr(corr4d[b, li]), _lib.stream_ptr(f_s.device)), "cwt_corr")
        if self.agg == "sum":   # mmn.py:62-63
            summed = torch.empty((B, 1, P, P), device=f_s.device, dtype=torch.float32)
            _lib.check(_lib.lib().cwt_channel_sum(_lib.ctx(f_s.device.index), _lib.ptr(corr4d), B, L, P * P,
                                                  _lib.ptr(summed), _lib.stream_ptr(f_s.device)), "cwt_channel_sum")
            corr4d = summed
        attn, att = self.corr_net._run(corr4d, h, w, f_s)   # att [B, Cv, h, w] (channels_last)
        att_t = as_tokens(att)
        fqt = as_tokens(f_q)
        att_fq = torch.empty((1, ch, h, w), device=f_s.device, dtype=torch.float32, memory_format=torch.channels_last)
        fq = torch.empty_like(att_fq)
        _lib.check(_lib.lib().cwt_mmn_blend(_lib.ctx(f_s.device.index), _lib.ptr(fqt), _lib.ptr(att_t), B, P * ch,
                                            self.att_wt, _lib.ptr(att_fq), _lib.ptr(fq), _lib.stream_ptr(f_s.device)),
                   "cwt_mmn_blend")
        if ret_attn:
            return attn, fq, att_fq
        return fq, att_fq

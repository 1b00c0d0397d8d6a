"""ORACLE — test infrastructure only.  CPU restatement of the reference's DeTr head
(src/model/detr.py:13-151) in float64 torch: SinePositionalEncoding, MSDeformAttn's single-level
forward with ms_deform_attn_core_pytorch, DeformAtt and DeTr.forward.

Only ``tests/`` may import this module, and only as the checker.  The product path
(``few_shot_seg_cwt_amd.detr``) never imports it.

Parity unpinned: the reference cannot be run in this container and holds no
fixtures for this head, so this restatement is checked by its own construction (each function
cites the reference file:line it restates; the sampling goes through torch's own F.grid_sample
exactly as ms_deform_attn_core_pytorch calls it) and by tests/test_detr_oracle.py (the sampling
against an explicit per-point bilinear loop, the position embedding against its closed form).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from oracle import match_oracle as MO


def sine_pos_embed(mask: torch.Tensor, num_feats: int, temperature: float = 10000, normalize: bool = False,
                   scale: float = 2 * math.pi, eps: float = 1e-6, dtype=torch.float64) -> torch.Tensor:
    """positional_encoding.py:44-74 for mask [bs, h, w] -> [bs, 2 num_feats, h, w]; ``~mask`` as
    torch evaluates it for the mask's dtype (a long zero mask gives -1: detr.py:135)."""
    not_mask = ~mask
    y_embed = not_mask.cumsum(1, dtype=dtype)
    x_embed = not_mask.cumsum(2, dtype=dtype)
    if normalize:
        y_embed = y_embed / (y_embed[:, -1:, :] + eps) * scale
        x_embed = x_embed / (x_embed[:, :, -1:] + eps) * scale
    dim_t = torch.arange(num_feats, dtype=dtype)
    dim_t = temperature ** (2 * (dim_t // 2) / num_feats)
    pos_x = x_embed[:, :, :, None] / dim_t
    pos_y = y_embed[:, :, :, None] / dim_t
    pos_x = torch.stack((pos_x[:, :, :, 0::2].sin(), pos_x[:, :, :, 1::2].cos()), dim=4).flatten(3)
    pos_y = torch.stack((pos_y[:, :, :, 0::2].sin(), pos_y[:, :, :, 1::2].cos()), dim=4).flatten(3)
    return torch.cat((pos_y, pos_x), dim=3).permute(0, 3, 1, 2)


def reference_points(H: int, W: int, dtype=torch.float64) -> torch.Tensor:
    """DeformAtt.get_reference_points (detr.py:98-110) for one level: [1, H*W, 1, 2] (x, y)."""
    ref_y, ref_x = torch.meshgrid(torch.linspace(0.5, H - 0.5, H, dtype=dtype),
                                  torch.linspace(0.5, W - 0.5, W, dtype=dtype), indexing="ij")
    ref = torch.stack((ref_x.reshape(-1)[None] / W, ref_y.reshape(-1)[None] / H), -1)
    return ref[:, :, None, :]


def deform_core(value, H, W, sampling_locations, attention_weights):
    """ms_deform_attn_func.py:41-61 for one level: value [N, S, M, D], sampling_locations
    [N, Lq, M, 1, P, 2], attention_weights [N, Lq, M, 1, P] -> [N, Lq, M*D]."""
    N_, S_, M_, D_ = value.shape
    _, Lq_, _, L_, P_, _ = sampling_locations.shape
    grids = 2 * sampling_locations - 1
    v = value.flatten(2).transpose(1, 2).reshape(N_ * M_, D_, H, W)
    g = grids[:, :, :, 0].transpose(1, 2).flatten(0, 1)
    sv = F.grid_sample(v, g, mode="bilinear", padding_mode="zeros", align_corners=False)   # [N*M, D, Lq, P]
    aw = attention_weights.transpose(1, 2).reshape(N_ * M_, 1, Lq_, L_ * P_)
    out = (sv * aw).sum(-1).view(N_, M_ * D_, Lq_)
    return out.transpose(1, 2).contiguous()


def ms_deform_attn(query, input_flatten, H, W, p, n_heads: int, n_points: int):
    """ms_deform_attn.py:84-117 (one level, 2-D reference points of DeformAtt, no padding mask);
    p = dict of the module's Linear weights / biases (value_proj, sampling_offsets,
    attention_weights, output_proj)."""
    N, Lq, C = query.shape
    value = F.linear(input_flatten, p["value_proj.weight"], p["value_proj.bias"]).view(N, Lq, n_heads, C // n_heads)
    offs = F.linear(query, p["sampling_offsets.weight"], p["sampling_offsets.bias"]).view(N, Lq, n_heads, 1,
                                                                                          n_points, 2)
    aw = F.linear(query, p["attention_weights.weight"], p["attention_weights.bias"]).view(N, Lq, n_heads, n_points)
    aw = F.softmax(aw, -1).view(N, Lq, n_heads, 1, n_points)
    ref = reference_points(H, W, query.dtype)
    normalizer = torch.tensor([[W, H]], dtype=query.dtype)
    loc = ref[:, :, None, :, None, :] + offs / normalizer[None, None, None, :, None, :]
    out = deform_core(value, H, W, loc, aw)
    return F.linear(out, p["output_proj.weight"], p["output_proj.bias"])


def deform_att(fq_fea, f_q, p, n_heads: int = 8, n_points: int = 9):
    """DeformAtt.forward (detr.py:87-96) at one level, padding_mask None."""
    B, C, h, w = fq_fea.shape
    mask = torch.zeros((B, h, w)).long()
    pos = sine_pos_embed(mask, C // 2, normalize=True, dtype=fq_fea.dtype)
    q = (fq_fea + pos).flatten(2).permute(0, 2, 1)
    v = f_q.flatten(2).permute(0, 2, 1)
    out = ms_deform_attn(q, v, h, w, p, n_heads, n_points)
    return out.permute(0, 2, 1).reshape(B, C, h, w)


def match_forward(fq_fea, fs_fea, v, layers, temp: float):
    """MatchNet.forward (match.py:103-140) without sce / ig_mask / cyc."""
    B, ch, h, w = fq_fea.shape
    a = F.normalize(fq_fea, dim=1).reshape(B, ch, h * w)
    b = F.normalize(fs_fea, dim=1).reshape(B, ch, h * w)
    corr = torch.bmm(a.transpose(1, 2), b).reshape(B, 1, h, w, h, w)
    _, wv = MO.corr_forward(corr, v, layers, temp, True)
    return wv


def detr_forward(fq_feats, fs_feats, f_q, f_s, w_adjust, match_layers, deform_p, temp: float, att_wt: float,
                 cs_att: bool = True, sf_att: bool = False):
    """DeTr.forward (detr.py:36-47): fq_feats / fs_feats the per-layer features in rmid order,
    w_adjust [reduce_dim, sum C_l, 1, 1]."""
    fq_fea = torch.relu(F.conv2d(torch.cat(fq_feats, 1), w_adjust))
    fs_fea = torch.relu(F.conv2d(torch.cat(fs_feats, 1), w_adjust))
    sa = ca = None
    if cs_att:
        ca = match_forward(fq_fea, fs_fea, f_s, match_layers, temp)
        f_q = F.normalize(f_q, p=2, dim=1) + F.normalize(ca, p=2, dim=1) * att_wt
    if sf_att:
        sa = deform_att(fq_fea, f_q, deform_p)
        f_q = F.normalize(f_q, p=2, dim=1) + F.normalize(sa, p=2, dim=1) * att_wt
    return f_q, sa, ca

"""ORACLE — test infrastructure only.  CPU restatement of the reference's MatchNet head
(the 4-D matching head of the MMN / MatchNet variants).

Only ``tests/`` may import this module, and only as the checker.  The product path
(``few_shot_seg_cwt_amd.match``) never imports it.

Parity unpinned: the reference cannot be run in this container and holds no
fixtures for this head, so this restatement is checked only by its own construction (each
function cites the reference file:line whose algorithm it restates, written independently of
it) and by tests/test_match_oracle.py's algebraic identities (symmetric-mode transpose
equivariance, the separable CenterPivotConv4d against a dense 4-D convolution with the
cross-shaped kernel).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def mutual_matching(x: torch.Tensor, eps: float = 1e-5) -> torch.Tensor:
    """match.py:21-53: x [B, C, ha, wa, hb, wb]; per channel, the ratio of each score to the
    maximum over the query positions (for its support position) and to the maximum over the
    support positions (for its query position): x * ((x / maxA) * (x / maxB))."""
    B, C, ha, wa, hb, wb = x.shape
    m = x.reshape(B, C, ha * wa, hb * wb)
    max_over_q = m.amax(dim=2, keepdim=True)   # for every support position
    max_over_s = m.amax(dim=3, keepdim=True)   # for every query position
    r_s = m / (max_over_q + eps)
    r_q = m / (max_over_s + eps)
    return (m * (r_q * r_s)).reshape(B, C, ha, wa, hb, wb)


def center_pivot_conv4d(x: torch.Tensor, w1, b1, w2, b2) -> torch.Tensor:
    """conv4d.py:40-62 at stride 1, kernel 3, padding 1: a 2-D conv (w1, b1) over the first
    position pair for every fixed second pair, plus one (w2, b2) over the second pair for every
    fixed first pair."""
    B, C, ha, wa, hb, wb = x.shape
    O = w1.shape[0]
    # over (ha, wa): fold (hb, wb) into the batch
    xa = x.permute(0, 4, 5, 1, 2, 3).reshape(B * hb * wb, C, ha, wa)
    ya = F.conv2d(xa, w1, b1, padding=1).reshape(B, hb, wb, O, ha, wa).permute(0, 3, 4, 5, 1, 2)
    # over (hb, wb): fold (ha, wa) into the batch
    xb = x.permute(0, 2, 3, 1, 4, 5).reshape(B * ha * wa, C, hb, wb)
    yb = F.conv2d(xb, w2, b2, padding=1).reshape(B, ha, wa, O, hb, wb).permute(0, 3, 1, 2, 4, 5)
    return ya + yb


def conv4d(x: torch.Tensor, w_perm, b) -> torch.Tensor:
    """conv4d.py:64-98 (conv_4d) at kernel 3: w_perm is the pre-permuted filter [k0][co][ci][k1]
    [k2][k3]; for each first-dimension slice i, conv3d of the zero-padded input slices i-1, i,
    i+1 with the matching filter slices (the bias once, with the centre slice)."""
    B, C, h, w, d, t = x.shape
    xs = x.permute(2, 0, 1, 3, 4, 5)
    pad = w_perm.shape[0] // 2
    Z = torch.zeros((pad, B, C, w, d, t), dtype=x.dtype)
    xp = torch.cat((Z, xs, Z), 0)
    out = []
    for i in range(h):
        o = F.conv3d(xp[i + pad], w_perm[pad], bias=b, stride=1, padding=pad)
        for p_ in range(1, pad + 1):
            o = o + F.conv3d(xp[i + pad - p_], w_perm[pad - p_], bias=None, stride=1, padding=pad)
            o = o + F.conv3d(xp[i + pad + p_], w_perm[pad + p_], bias=None, stride=1, padding=pad)
        out.append(o)
    return torch.stack(out, 0).permute(1, 2, 0, 3, 4, 5)


def neigh_consensus_cv4(x: torch.Tensor, layers, symmetric: bool = True) -> torch.Tensor:
    """match.py:56-85 with conv='cv4': layers = [(w_perm, b)] * 3, each Conv4d then ReLU."""
    def stack(z):
        for (wp, b) in layers:
            z = torch.relu(conv4d(z, wp, b))
        return z
    y = stack(x)
    if symmetric:
        y = y + stack(x.permute(0, 1, 4, 5, 2, 3)).permute(0, 1, 4, 5, 2, 3)
    return y


def neigh_consensus(x: torch.Tensor, layers, symmetric: bool = True) -> torch.Tensor:
    """match.py:56-85: layers = [(w1, b1, w2, b2)] * 3, each CenterPivotConv4d then ReLU;
    symmetric mode adds the stack applied to the pair-swapped tensor, swapped back."""
    def stack(z):
        for (w1, b1, w2, b2) in layers:
            z = torch.relu(center_pivot_conv4d(z, w1, b1, w2, b2))
        return z
    y = stack(x)
    if symmetric:
        y = y + stack(x.permute(0, 1, 4, 5, 2, 3)).permute(0, 1, 4, 5, 2, 3)
    return y


def run_match_model(corr4d: torch.Tensor, layers, symmetric: bool = True) -> torch.Tensor:
    """match.py:159-163 (layers of 2 tensors: Conv4d 'cv4'; of 4: CenterPivotConv4d 'red')."""
    nc = neigh_consensus_cv4 if len(layers[0]) == 2 else neigh_consensus
    return mutual_matching(nc(mutual_matching(corr4d), layers, symmetric))


def corr_forward(corr4d: torch.Tensor, v: torch.Tensor, layers, temp: float, symmetric: bool = True):
    """match.py:142-157: corr4d [B, L, h, w, h, w], v [B, Cv, h, w] ->
    (corr2d [B, hw, hw], weighted_v [B, Cv, h, w])."""
    B, L, h, w = corr4d.shape[:4]
    corr2d = run_match_model(corr4d, layers, symmetric).reshape(B, h * w, h * w)
    attn = torch.softmax(corr2d * temp, dim=-1)
    wv = torch.bmm(v.reshape(B, v.shape[1], h * w), attn.transpose(1, 2)).reshape(B, v.shape[1], h, w)
    return corr2d, wv


def spatial_descriptor(x: torch.Tensor, k: int) -> torch.Tensor:
    """spatial_context.py:13-56 (generate_spatial_descriptor): x [B, C, h, w] -> [B, k*k, h, w],
    the dot product of each pixel's feature with every position of its zero-padded k x k
    window (row-major window order)."""
    B, C, h, w = x.shape
    pad = k // 2
    patches = F.unfold(x, k, padding=pad).reshape(B, C, k * k, h * w)
    return (patches * x.reshape(B, C, 1, h * w)).sum(1).reshape(B, k * k, h, w)


def spatial_context_encoder(x: torch.Tensor, k: int, weight, bias) -> torch.Tensor:
    """spatial_context.py:59-110: featureL2Norm (eps 1e-6 inside the root), cat, 1x1 conv, ReLU."""
    g = spatial_descriptor(x, k)
    g = g / torch.pow(torch.sum(g * g, 1) + 1e-6, 0.5).unsqueeze(1)
    return torch.relu(F.conv2d(torch.cat([x, g], 1), weight, bias))


def support_masks(corr2d: torch.Tensor, ig_mask=None, s_mask=None):
    """match.py:117-126 with run_cyc (match.py:165-182) in eval mode (Dropout identity):
    corr2d [B, N_q, N_s] -> (masked corr2d, inconsistent [B, N_s] or None).  Not in place."""
    B, nq, ns = corr2d.shape
    c = corr2d.clone()
    if ig_mask is not None:
        m = ig_mask.reshape(B, 1, ns).expand(c.shape)
        c[m == True] = 0.0001   # noqa: E712  (the reference's spelling)
    inc = None
    if s_mask is not None:
        sm = s_mask.reshape(B, ns)
        k2q = c.max(1)[1]
        q2k = c.max(2)[1]
        re_map_idx = torch.gather(q2k, 1, k2q)
        re_map_mask = torch.gather(sm, 1, re_map_idx)
        inc = (~(sm == re_map_mask)).to(c.dtype)
        c = c + inc.unsqueeze(1) * (-1000.0)
    return c, inc


def layers_from_state(sd, prefix: str = "NeighConsensus.conv.", dtype=torch.float64):
    out = []
    for i in (0, 2, 4):
        p = f"{prefix}{i}."
        if p + "weight" in sd:   # Conv4d ('cv4')
            out.append((sd[p + "weight"].to(dtype), sd[p + "bias"].to(dtype)))
            continue
        out.append(tuple(sd[p + n].to(dtype) for n in ("conv1.weight", "conv1.bias", "conv2.weight", "conv2.bias")))
    return out


def weight_average(x: torch.Tensor, p) -> torch.Tensor:
    """msm_func.py:50-104 (R = 3, dropouts off): p = (w_theta, b_theta, w_phi, b_phi, w_g, b_g,
    w_back, b_back) as nn.Conv2d 1x1 weights / biases."""
    wt, bt, wp, bp, wg, bg, wb, bb = p
    B, C, h, w = x.shape
    xp = F.pad(x, (1, 1, 1, 1), mode="replicate")
    theta = F.conv2d(x, wt, bt)
    cos, gs = [], []
    for dy in range(3):
        for dx in range(3):
            nb = xp[:, :, dy:dy + h, dx:dx + w]      # the neighbour at offset (dy - 1, dx - 1)
            cos.append(F.cosine_similarity(F.conv2d(nb, wp, bp), theta, dim=1))
            gs.append(F.conv2d(nb, wg, bg))
    sm = torch.softmax(torch.stack(cos, 1), dim=1)            # [B, 9, h, w]
    wavg = sum(sm[:, r:r + 1] * gs[r] for r in range(9))
    return x + F.conv2d(wavg, wb, bb)


def feat_list(x: torch.Tensor, sd, layers: int = 50):
    """get_feat_list (pspnet.py:272-287) with all_lr 'l': {2, 3, 4: the layer's last block output}."""
    from oracle.cwt_oracle import RESNET_BLOCKS, bottleneck, stem
    x = stem(x, sd)
    out = {}
    for li, nblk in enumerate(RESNET_BLOCKS[layers], start=1):
        for b in range(nblk):
            x = bottleneck(x, sd, li, b)
        if li >= 2:
            out[li] = x
    return out


def mmn_forward(fq_lst, fs_lst, f_q, f_s, bid_lst, wa_params, layers, temp: float, att_wt: float,
                agg: str = "cat", rd_weights=None):
    """mmn.py:42-71: fq_lst / fs_lst {layer: feature}, wa_params {layer: weight_average params}
    or None, rd_weights {layer: rd_<layer>.0.weight} (red_dim) or None, agg 'cat' or 'sum' ->
    (fq, att_fq)."""
    B, ch, h, w = f_s.shape
    corrs = []
    for idx in bid_lst[::-1]:
        fq, fs = fq_lst[idx].expand(B, -1, -1, -1), fs_lst[idx]
        if rd_weights is not None:
            fq, fs = torch.relu(F.conv2d(fq, rd_weights[idx])), torch.relu(F.conv2d(fs, rd_weights[idx]))
        if wa_params is not None:
            fq, fs = weight_average(fq, wa_params[idx]), weight_average(fs, wa_params[idx])
        bq = F.normalize(fq.reshape(B, fq.shape[1], h * w), dim=1)
        bs = F.normalize(fs.reshape(B, fs.shape[1], h * w), dim=1)
        corrs.append(torch.bmm(bq.transpose(1, 2), bs).reshape(B, 1, h, w, h, w))
    corr4d = torch.cat(corrs, 1)
    if agg == "sum":
        corr4d = torch.sum(corr4d, dim=1, keepdim=True)
    _, att = corr_forward(corr4d, f_s, layers, temp, True)
    att = att.mean(dim=0, keepdim=True)
    return f_q * (1 - att_wt) + att * att_wt, att


def wa_params_from_state(sd, prefix: str, dtype=torch.float64):
    return tuple(sd[prefix + n].to(dtype) for n in ("conv_theta.weight", "conv_theta.bias", "conv_phi.weight",
                                                     "conv_phi.bias", "conv_g.weight", "conv_g.bias",
                                                     "conv_back.weight", "conv_back.bias"))

"""CPU checks of oracle/detr_oracle.py (the DeTr restatement the GPU tests compare against; parity
unpinned): the deformable sampling (F.grid_sample as ms_deform_attn_func.py:41-61
calls it) against an explicit per-point bilinear loop with zero padding and align_corners=False,
the sine position embedding against its closed form for DeformAtt's long zero mask, and the
reference points against the pixel centres."""
import math

import torch

from oracle import detr_oracle as D


def test_reference_points_are_pixel_centres():
    H, W = 3, 5
    ref = D.reference_points(H, W)[0, :, 0]
    for i in range(H):
        for j in range(W):
            assert torch.allclose(ref[i * W + j], torch.tensor([(j + 0.5) / W, (i + 0.5) / H], dtype=torch.float64))


def test_sine_pos_long_mask_closed_form():
    """detr.py:135 builds the mask as zeros().long(), so ~mask = -1: the embeddings are -(i+1)
    over -(H) + eps, i.e. (i + 1) / (H - eps) * 2 pi."""
    B, h, w, nf = 1, 4, 6, 8
    pos = D.sine_pos_embed(torch.zeros((B, h, w)).long(), nf, normalize=True)
    for c in range(2 * nf):
        k = c % nf
        dt = 10000 ** (2 * (k // 2) / nf)
        for i in range(h):
            for j in range(w):
                e = (-(i + 1)) / (-h + 1e-6) * 2 * math.pi if c < nf else (-(j + 1)) / (-w + 1e-6) * 2 * math.pi
                ref = math.sin(e / dt) if k % 2 == 0 else math.cos(e / dt)
                assert abs(float(pos[0, c, i, j]) - ref) < 1e-12


def _bilinear_zero(img, x, y):
    """img [D, H, W]; pixel-space (x, y) (align_corners False source index); zero outside."""
    D_, H, W = img.shape
    x0, y0 = math.floor(x), math.floor(y)
    out = torch.zeros(D_, dtype=img.dtype)
    for yy, wy in ((y0, y0 + 1 - y), (y0 + 1, y - y0)):
        for xx, wx in ((x0, x0 + 1 - x), (x0 + 1, x - x0)):
            if 0 <= yy < H and 0 <= xx < W:
                out += img[:, yy, xx] * (wx * wy)
    return out


def test_deform_core_matches_explicit_bilinear():
    g = torch.Generator().manual_seed(3)
    N, H, W, M, Dh, P = 1, 5, 7, 2, 3, 4
    value = torch.rand(N, H * W, M, Dh, generator=g, dtype=torch.float64)
    ref = D.reference_points(H, W)
    offs = (torch.rand(N, H * W, M, 1, P, 2, generator=g, dtype=torch.float64) - 0.5) * 6   # some fall outside
    loc = ref[:, :, None, :, None, :] + offs / torch.tensor([[W, H]], dtype=torch.float64)[None, None, None, :, None, :]
    aw = torch.softmax(torch.rand(N, H * W, M, P, generator=g, dtype=torch.float64), -1).view(N, H * W, M, 1, P)
    out = D.deform_core(value, H, W, loc, aw)
    for q in range(H * W):
        for m in range(M):
            img = value[0, :, m, :].T.reshape(Dh, H, W)
            acc = torch.zeros(Dh, dtype=torch.float64)
            for p in range(P):
                lx, ly = float(loc[0, q, m, 0, p, 0]), float(loc[0, q, m, 0, p, 1])
                acc += _bilinear_zero(img, lx * W - 0.5, ly * H - 0.5) * float(aw[0, q, m, 0, p])
            assert torch.allclose(out[0, q, m * Dh:(m + 1) * Dh], acc, atol=1e-12)


def test_detr_parameter_names_and_init_follow_the_reference():
    """DeTr / DeformAtt / MSDeformAttn keep the reference's state_dict keys (detr.py:13-110,
    ms_deform_attn.py:54-59) and MSDeformAttn's initialisation (ms_deform_attn.py:61-75); host
    only (parameters on the CPU, no forward)."""
    from few_shot_seg_cwt_amd.detr import DeTr, MSDeformAttn
    cpu = torch.device("cpu")
    net = DeTr(dict(rmid="l34", temp=20.0, att_wt=0.2), sf_att=True, cs_att=True, reduce_dim=512, device=cpu)
    keys = set(net.state_dict().keys())
    want = {"adjust_feature.0.weight", "self_trans.level_embed"}
    for i in (0, 2, 4):
        for c in ("conv1", "conv2"):
            want |= {f"cross_trans.NeighConsensus.conv.{i}.{c}.weight", f"cross_trans.NeighConsensus.conv.{i}.{c}.bias"}
    for m in ("sampling_offsets", "attention_weights", "value_proj", "output_proj"):
        want |= {f"self_trans.self_trans.{m}.weight", f"self_trans.self_trans.{m}.bias"}
    assert keys == want, sorted(keys ^ want)
    assert tuple(net.adjust_feature[0].weight.shape) == (512, 3072, 1, 1)
    m = MSDeformAttn(d_model=512, n_levels=1, n_heads=8, n_points=9, device=cpu)
    assert torch.count_nonzero(m.sampling_offsets.weight) == 0 and torch.count_nonzero(m.attention_weights.weight) == 0
    b = m.sampling_offsets.bias.view(8, 1, 9, 2)
    for h in range(8):
        th = h * 2 * math.pi / 8
        d = torch.tensor([math.cos(th), math.sin(th)])
        d = d / d.abs().max()
        for p in range(9):
            assert torch.allclose(b[h, 0, p], d * (p + 1), atol=1e-6)

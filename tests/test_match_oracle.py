"""CPU checks of oracle/match_oracle.py (the MatchNet restatement; parity unpinned: no
reference fixture exists for this head).  The restatement is checked against
independent formulations of the same maps: MutualMatching element by element, the separable
CenterPivotConv4d against a dense 4-D correlation with its cross-shaped 3^4 kernel, and the
symmetric NeighConsensus's equivariance under swapping the two position pairs."""
import torch

from oracle import match_oracle as M


def _layers(L, seed):
    g = torch.Generator().manual_seed(seed)
    out, ci = [], L
    for co in (10, 10, 1):
        mk = lambda *s: (torch.rand(*s, generator=g, dtype=torch.float64) * 2 - 1) * 0.3  # noqa: E731
        out.append((mk(co, ci, 3, 3), mk(co), mk(co, ci, 3, 3), mk(co)))
        ci = co
    return out


def test_mutual_matching_elementwise():
    g = torch.Generator().manual_seed(1)
    x = torch.rand(2, 2, 3, 4, 4, 3, generator=g, dtype=torch.float64)
    y = M.mutual_matching(x)
    B, C = 2, 2
    m = x.reshape(B, C, 12, 12)
    for b in range(B):
        for c in range(C):
            for i in range(12):
                for j in range(12):
                    v = m[b, c, i, j]
                    ref = v * ((v / (m[b, c, i, :].max() + 1e-5)) * (v / (m[b, c, :, j].max() + 1e-5)))
                    assert torch.allclose(y.reshape(B, C, 12, 12)[b, c, i, j], ref, rtol=1e-14, atol=0)


def test_center_pivot_equals_dense_cross_kernel():
    g = torch.Generator().manual_seed(2)
    B, C, O, ha, wa, hb, wb = 1, 2, 3, 4, 5, 5, 3
    x = torch.rand(B, C, ha, wa, hb, wb, generator=g, dtype=torch.float64)
    w1, w2 = torch.rand(O, C, 3, 3, generator=g, dtype=torch.float64), torch.rand(O, C, 3, 3, generator=g, dtype=torch.float64)
    b1, b2 = torch.rand(O, generator=g, dtype=torch.float64), torch.rand(O, generator=g, dtype=torch.float64)
    y = M.center_pivot_conv4d(x, w1, b1, w2, b2)
    xp = torch.nn.functional.pad(x, (1, 1, 1, 1, 1, 1, 1, 1))
    ref = torch.zeros(B, O, ha, wa, hb, wb, dtype=torch.float64) + (b1 + b2).view(1, O, 1, 1, 1, 1)
    for t1 in range(3):
        for t2 in range(3):
            for t3 in range(3):
                for t4 in range(3):
                    k = torch.zeros(O, C, dtype=torch.float64)
                    if (t3, t4) == (1, 1):
                        k = k + w1[:, :, t1, t2]
                    if (t1, t2) == (1, 1):
                        k = k + w2[:, :, t3, t4]
                    if not k.abs().sum():
                        continue
                    sl = xp[:, :, t1:t1 + ha, t2:t2 + wa, t3:t3 + hb, t4:t4 + wb]
                    ref = ref + torch.einsum("oc,bcijkl->boijkl", k, sl)
    assert torch.allclose(y, ref, rtol=1e-12, atol=1e-12)


def test_symmetric_consensus_is_swap_equivariant():
    g = torch.Generator().manual_seed(3)
    x = torch.rand(1, 2, 5, 4, 5, 4, generator=g, dtype=torch.float64)
    layers = _layers(2, 4)
    y = M.neigh_consensus(x, layers, symmetric=True)
    ys = M.neigh_consensus(x.permute(0, 1, 4, 5, 2, 3), layers, symmetric=True).permute(0, 1, 4, 5, 2, 3)
    assert torch.allclose(y, ys, rtol=1e-12, atol=1e-12)


def test_support_masks_against_loops():
    """oracle support_masks (match.py:117-126, run_cyc 165-182, eval mode) against explicit
    loops: the ig columns set to 1e-4, k2q / q2k first-index argmaxes, the -1000 offsets."""
    from oracle import match_oracle as M
    g = torch.Generator().manual_seed(4)
    B, n = 2, 12
    c = torch.rand(B, n, n, generator=g, dtype=torch.float64)
    ig = torch.rand(B, n, generator=g) < 0.25
    sm = (torch.rand(B, n, generator=g) < 0.5).long()
    out, inc = M.support_masks(c, ig, sm)
    for b in range(B):
        cm = [[1e-4 if bool(ig[b, j]) else float(c[b, i, j]) for j in range(n)] for i in range(n)]
        for j in range(n):
            col = [cm[i][j] for i in range(n)]
            k2q = col.index(max(col))
            q2k = cm[k2q].index(max(cm[k2q]))
            bad = int(sm[b, j]) != int(sm[b, q2k])
            assert float(inc[b, j]) == (1.0 if bad else 0.0)
            for i in range(n):
                assert float(out[b, i, j]) == cm[i][j] + (-1000.0 if bad else 0.0)


def test_conv4d_against_direct_sum_and_swap():
    """oracle conv4d (conv_4d's per-slice conv3d sum, conv4d.py:64-98, pre-permuted filter)
    against the direct 4-D cross-correlation with zero padding; and the identity the device's
    symmetric branch uses: conv(x^T)^T = conv(x) with the filter's position pairs exchanged."""
    from oracle import match_oracle as M
    g = torch.Generator().manual_seed(8)
    B, C, O = 1, 2, 3
    sh = (3, 4, 3, 2)
    x = torch.rand(B, C, *sh, generator=g, dtype=torch.float64)
    w = torch.rand(O, C, 3, 3, 3, 3, generator=g, dtype=torch.float64) - 0.5
    b = torch.rand(O, generator=g, dtype=torch.float64)
    wp = w.permute(2, 0, 1, 3, 4, 5).contiguous()
    y = M.conv4d(x, wp, b)
    xpad = torch.nn.functional.pad(x, (1, 1, 1, 1, 1, 1, 1, 1))
    ref = torch.zeros(B, O, *sh, dtype=torch.float64)
    for i in range(sh[0]):
        for j in range(sh[1]):
            for k in range(sh[2]):
                for l in range(sh[3]):
                    patch = xpad[0, :, i:i + 3, j:j + 3, k:k + 3, l:l + 3]
                    ref[0, :, i, j, k, l] = (w * patch[None]).sum(dim=(1, 2, 3, 4, 5)) + b
    assert torch.allclose(y, ref, atol=1e-12)
    xs = torch.rand(B, C, 3, 4, 3, 4, generator=g, dtype=torch.float64)
    lhs = M.conv4d(xs.permute(0, 1, 4, 5, 2, 3), wp, b).permute(0, 1, 4, 5, 2, 3)
    w_sw = w.permute(0, 1, 4, 5, 2, 3)   # filter taps (u0, u1, u2, u3) <- (u2, u3, u0, u1)
    rhs = M.conv4d(xs, w_sw.permute(2, 0, 1, 3, 4, 5).contiguous(), b)
    assert torch.allclose(lhs, rhs, atol=1e-12)


def test_spatial_descriptor_against_loops():
    """oracle spatial_descriptor (unfold form) against generate_spatial_descriptor's per-pixel
    window loop (spatial_context.py:13-56) on a small map."""
    from oracle import match_oracle as M
    g = torch.Generator().manual_seed(6)
    B, C, h, w, k = 2, 5, 6, 7, 5
    x = torch.rand(B, C, h, w, generator=g, dtype=torch.float64)
    d = M.spatial_descriptor(x, k)
    pad = k // 2
    xp = torch.nn.functional.pad(x, (pad, pad, pad, pad))
    for hi in range(h):
        for wj in range(w):
            q = x[:, :, hi, wj]
            patch = xp[:, :, hi:hi + k, wj:wj + k].reshape(B, C, k * k)
            ref = torch.bmm(q.unsqueeze(1), patch).squeeze(1)
            assert torch.allclose(d[:, :, hi, wj], ref, atol=1e-12)

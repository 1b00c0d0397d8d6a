// Classifier Weight Transformer: MultiHeadAttentionOne (reference transformer.py:33-83,
// ScaledDotProductAttention transformer.py:12-30), eval forward and parameter backward.
//
// The reference projects all hw query-feature tokens through the shared w_qkvs (2 x
// hw x 512 x 512H MACs: 15.1 GFLOP at hw=3600, H=4) although only 2 queries attend.
// Re-associating the two products keeps every token in the 512-dim input space:
//   a_hi  = W_h q_i                       (W_h = w_qkvs rows h*C..h*C+C-1)
//   r_hi  = W_h^T a_hi / sqrt(C)          => score_hip = r_hi . f_p = (W_h q_i).(W_h f_p)/sqrt(C)
//   P_hi  = softmax_p(score_hi)
//   g_hi  = sum_p P_hip f_p               => out_hi = W_h g_hi = sum_p P_hip (W_h f_p)
//   y_i   = fc(concat_h out_hi) + q_i ;  out_i = LayerNorm(y_i)
// which is the same function with 59 MFLOP of token work instead of 15.1 GFLOP, and reads
// the 7.4 MB token map exactly once (flash-decoding style chunk partials + a combine).
#include "common.h"
#include "kernels.h"

namespace cwt {

// out[v*ovs + j] = alpha * sum_k A[j][k] * X[v*xvs + (j/rows_per_group)*xgs + k] (+bias[j]) (+res[v*rvs+j])
// One wave per output row; lanes split K (KPL floats per lane, K = 64*KPL).
template <int KPL>
__global__ __launch_bounds__(256) void rowdot_kernel(const float* __restrict__ A, int R, const float* __restrict__ X,
                                                     int nv, long xvs, long xgs, int rows_per_group,
                                                     const float* __restrict__ bias, const float* __restrict__ res,
                                                     long rvs, float* __restrict__ out, long ovs, float alpha,
                                                     float* __restrict__ zero, long zero_n) {
  // zero: a buffer the NEXT launch accumulates into, cleared here instead of by a memset launch
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (zero && gid < zero_n) zero[gid] = 0.f;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  constexpr int K = 64 * KPL;
  float a[KPL];
  const float* ar = A + (long)row * K + lane * 4;
#pragma unroll
  for (int c = 0; c < KPL / 4; ++c) {
    f32x4 u = *(const f32x4*)(ar + c * 256);
    a[4 * c] = u[0]; a[4 * c + 1] = u[1]; a[4 * c + 2] = u[2]; a[4 * c + 3] = u[3];
  }
  const long gofs = (long)(row / rows_per_group) * xgs;
  for (int v = 0; v < nv; ++v) {
    const float* xr = X + v * xvs + gofs + lane * 4;
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < KPL / 4; ++c) {
      f32x4 u = *(const f32x4*)(xr + c * 256);
      s = fmaf(a[4 * c], u[0], s);
      s = fmaf(a[4 * c + 1], u[1], s);
      s = fmaf(a[4 * c + 2], u[2], s);
      s = fmaf(a[4 * c + 3], u[3], s);
    }
    s = wave_sum(s);
    if (lane == 0) {
      float o = alpha * s;
      if (bias) o += bias[row];
      if (res) o += res[v * rvs + row];
      out[v * ovs + row] = o;
    }
  }
}

int launch_rowdot(const float* A, int R, int K, const float* X, int nv, long xvs, long xgs, int rows_per_group,
                  const float* bias, const float* res, long rvs, float* out, long ovs, float alpha, hipStream_t st,
                  float* zero = nullptr, long zero_n = 0) {
  dim3 grid(cdiv(R, 4)), block(256);
  if (zero && zero_n > (long)grid.x * 256) return fail(CWT_EARG, "rowdot: buffer to clear exceeds the grid");
  if (K == 512)
    hipLaunchKernelGGL((rowdot_kernel<8>), grid, block, 0, st, A, R, X, nv, xvs, xgs, rows_per_group, bias, res,
                       rvs, out, ovs, alpha, zero, zero_n);
  else if (K == 1024)
    hipLaunchKernelGGL((rowdot_kernel<16>), grid, block, 0, st, A, R, X, nv, xvs, xgs, rows_per_group, bias, res,
                       rvs, out, ovs, alpha, zero, zero_n);
  else if (K == 2048)
    hipLaunchKernelGGL((rowdot_kernel<32>), grid, block, 0, st, A, R, X, nv, xvs, xgs, rows_per_group, bias, res,
                       rvs, out, ovs, alpha, zero, zero_n);
  else if (K == 4096)
    hipLaunchKernelGGL((rowdot_kernel<64>), grid, block, 0, st, A, R, X, nv, xvs, xgs, rows_per_group, bias, res,
                       rvs, out, ovs, alpha, zero, zero_n);
  else
    return fail(CWT_EARG, "rowdot: unsupported K");
  CWT_LAUNCH_CHECK();
  return 0;
}

// out[g][v][k] += alpha * sum_{d in chunk} A[g*Dg + d][k] * X[v*xvs + g*Dg + d]
// (transposed GEMV per group g).  Block = (k block of 256, group, d chunk of 16); the
// chunk's 16 rows are loaded before any FMA (16 loads in flight per lane).
constexpr int COLDOT_D = 16;
__global__ __launch_bounds__(64) void coldot_kernel(const float* __restrict__ A, int K, int Dg,
                                                    const float* __restrict__ X, int nv, long xvs,
                                                    float* __restrict__ out, float alpha) {
  const int k = blockIdx.x * 256 + threadIdx.x * 4;
  const int g = blockIdx.y;
  const int d0 = blockIdx.z * COLDOT_D;
  if (k >= K) return;
  const int dn = min(COLDOT_D, Dg - d0);
  f32x4 av[COLDOT_D];
#pragma unroll
  for (int d = 0; d < COLDOT_D; ++d) av[d] = *(const f32x4*)(A + ((long)g * Dg + d0 + min(d, dn - 1)) * K + k);
  f32x4 acc[8];
#pragma unroll
  for (int v = 0; v < 8; ++v) acc[v] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int d = 0; d < COLDOT_D; ++d) {
    if (d >= dn) break;
    const long row = (long)g * Dg + d0 + d;
#pragma unroll
    for (int v = 0; v < 8; ++v)
      if (v < nv) acc[v] += X[v * xvs + row] * av[d];
  }
#pragma unroll
  for (int v = 0; v < 8; ++v)
    if (v < nv) {
      float* o = out + ((long)g * nv + v) * K + k;
#pragma unroll
      for (int q = 0; q < 4; ++q) atomicAdd(o + q, alpha * acc[v][q]);
    }
}

int launch_coldot(const float* A, int G, int Dg, int K, const float* X, int nv, long xvs, float* out, float alpha,
                  hipStream_t st) {
  if (nv > 8) return fail(CWT_EARG, "coldot: at most 8 vectors");
  dim3 grid(cdiv(K, 256), G, cdiv(Dg, COLDOT_D));
  hipLaunchKernelGGL(coldot_kernel, grid, dim3(64), 0, st, A, K, Dg, X, nv, xvs, out, alpha);
  CWT_LAUNCH_CHECK();
  return 0;
}

// ---- attention over the token map: chunk partials (max, sum-exp, exp-weighted token sums) ----
constexpr int ATT_TPW = 8;                 // tokens per wave
constexpr int ATT_TPB = 4 * ATT_TPW;       // tokens per workgroup

// r: [H][nv][C] scores queries (already / sqrt(C)), row rho = h*2 + i of batch b is r[h][b*2+i].
// f: [B][hw][C].  part_g: [B][nchunk][NR][C]; part_ml: [B][nchunk][NR][2].
// Optionally stores the raw scores for the backward pass: scores [B][NR][hw].
// Training-mode attention dropout (transformer.py:17,28: dropout AFTER the softmax): token p of
// row rho enters g with weight m = dropout_scale(p_drop, seed, 1, (b*NR + rho)*hw + p); the
// softmax denominator l is unaffected.
template <int NR>
__global__ __launch_bounds__(256) void attn_partial_kernel(const float* __restrict__ r, const float* __restrict__ f,
                                                           int hw, int nv, float* __restrict__ part_g,
                                                           float* __restrict__ part_ml, float* __restrict__ scores,
                                                           float p_drop, unsigned long long seed) {
  constexpr int C = 512;
  __shared__ float rs[NR][C];
  __shared__ float wml[4][NR][2];
  __shared__ float wg[4][NR][C];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int chunk = blockIdx.x, b = blockIdx.y, nchunk = gridDim.x;
  for (int i = t; i < NR * C; i += 256) {
    const int rho = i / C, k = i % C;
    const int h = rho >> 1, qi = rho & 1;
    rs[rho][k] = r[((long)h * nv + b * 2 + qi) * C + k];
  }
  __syncthreads();
  const int tok0 = chunk * ATT_TPB + wv * ATT_TPW;
  float fv[ATT_TPW][8];
#pragma unroll
  for (int tt = 0; tt < ATT_TPW; ++tt) {
    const int p = tok0 + tt;
    if (p < hw) {
      const float* src = f + ((long)b * hw + p) * C + lane * 8;
      f32x4 u = *(const f32x4*)src, v = *(const f32x4*)(src + 4);
      fv[tt][0] = u[0]; fv[tt][1] = u[1]; fv[tt][2] = u[2]; fv[tt][3] = u[3];
      fv[tt][4] = v[0]; fv[tt][5] = v[1]; fv[tt][6] = v[2]; fv[tt][7] = v[3];
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) fv[tt][q] = 0.f;
    }
  }
  float s[ATT_TPW][NR];
#pragma unroll
  for (int rho = 0; rho < NR; ++rho) {
    float rv[8];
    f32x4 u = *(const f32x4*)&rs[rho][lane * 8], v = *(const f32x4*)&rs[rho][lane * 8 + 4];
    rv[0] = u[0]; rv[1] = u[1]; rv[2] = u[2]; rv[3] = u[3]; rv[4] = v[0]; rv[5] = v[1]; rv[6] = v[2]; rv[7] = v[3];
#pragma unroll
    for (int tt = 0; tt < ATT_TPW; ++tt) {
      float d = 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q) d = fmaf(rv[q], fv[tt][q], d);
      s[tt][rho] = wave_sum_dpp(d);
    }
  }
  if (scores && lane < ATT_TPW) {
#pragma unroll
    for (int tt = 0; tt < ATT_TPW; ++tt)
      if (tt == lane && tok0 + tt < hw) {
#pragma unroll
        for (int rho = 0; rho < NR; ++rho) scores[((long)b * NR + rho) * hw + tok0 + tt] = s[tt][rho];
      }
  }
#pragma unroll
  for (int rho = 0; rho < NR; ++rho) {
    float m = -INFINITY;
#pragma unroll
    for (int tt = 0; tt < ATT_TPW; ++tt)
      if (tok0 + tt < hw) m = fmaxf(m, s[tt][rho]);
    float l = 0.f;
    float g[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) g[q] = 0.f;
#pragma unroll
    for (int tt = 0; tt < ATT_TPW; ++tt) {
      const float e = (tok0 + tt < hw) ? __expf(s[tt][rho] - m) : 0.f;
      l += e;
      const float em = p_drop > 0.f ? e * dropout_scale(p_drop, seed, 1, ((long)b * NR + rho) * hw + tok0 + tt) : e;
#pragma unroll
      for (int q = 0; q < 8; ++q) g[q] = fmaf(em, fv[tt][q], g[q]);
    }
    if (lane == 0) {
      wml[wv][rho][0] = m;
      wml[wv][rho][1] = l;
    }
    *(f32x4*)&wg[wv][rho][lane * 8] = f32x4{g[0], g[1], g[2], g[3]};
    *(f32x4*)&wg[wv][rho][lane * 8 + 4] = f32x4{g[4], g[5], g[6], g[7]};
  }
  __syncthreads();
  // combine the 4 waves
  for (int i = t; i < NR * C; i += 256) {
    const int rho = i / C, k = i % C;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < 4; ++w) M = fmaxf(M, wml[w][rho][0]);
    float G = 0.f, L = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float sc = (wml[w][rho][0] == -INFINITY) ? 0.f : __expf(wml[w][rho][0] - M);
      G = fmaf(sc, wg[w][rho][k], G);
      L = fmaf(sc, wml[w][rho][1], L);
    }
    part_g[(((long)b * nchunk + chunk) * NR + rho) * C + k] = G;
    if (k == 0) {
      part_ml[(((long)b * nchunk + chunk) * NR + rho) * 2] = M;
      part_ml[(((long)b * nchunk + chunk) * NR + rho) * 2 + 1] = L;
    }
  }
}

// g[h][b*2+i][k] = sum_c e^{m_c-M} part_g_c / sum_c e^{m_c-M} l_c; also stores (M, L) per row.
// Block = (64 channels, row rho, batch b); its 4 waves take every 4th chunk, then combine in LDS.
template <int NR>
__global__ __launch_bounds__(256) void attn_combine_kernel(const float* __restrict__ part_g,
                                                           const float* __restrict__ part_ml, int nchunk, int nv,
                                                           float* __restrict__ g, float* __restrict__ ml_out) {
  constexpr int C = 512;
  __shared__ float sm[4], sg[4][64], sl[4];
  const int t = threadIdx.x, kk = t & 63, cg = t >> 6;
  const int k = blockIdx.x * 64 + kk;
  const int rho = blockIdx.y, b = blockIdx.z;
  const float* ml = part_ml + ((long)b * nchunk * NR + rho) * 2;
  // 8 chunks per round in flight (unconditional loads at clamped chunk indices)
  float M = -INFINITY;
  for (int c0 = cg; c0 < nchunk; c0 += 32) {
    float mv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) mv[u] = ml[(long)min(c0 + 4 * u, nchunk - 1) * NR * 2];
#pragma unroll
    for (int u = 0; u < 8; ++u) M = fmaxf(M, mv[u]);  // clamped duplicates do not change a max
  }
  if (kk == 0) sm[cg] = M;
  __syncthreads();
  M = fmaxf(fmaxf(sm[0], sm[1]), fmaxf(sm[2], sm[3]));
  float G = 0.f, L = 0.f;
  const float* pg = part_g + ((long)b * nchunk * NR + rho) * C + k;
  for (int c0 = cg; c0 < nchunk; c0 += 32) {
    float mc[8], lc[8], gc[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const long c = min(c0 + 4 * u, nchunk - 1);
      mc[u] = ml[c * NR * 2];
      lc[u] = ml[c * NR * 2 + 1];
      gc[u] = pg[c * NR * C];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (c0 + 4 * u >= nchunk) break;
      const float sc = (mc[u] == -INFINITY) ? 0.f : __expf(mc[u] - M);
      G = fmaf(sc, gc[u], G);
      L = fmaf(sc, lc[u], L);
    }
  }
  sg[cg][kk] = G;
  if (kk == 0) sl[cg] = L;
  __syncthreads();
  if (cg == 0) {
    const float Gs = (sg[0][kk] + sg[1][kk]) + (sg[2][kk] + sg[3][kk]);
    const float Ls = (sl[0] + sl[1]) + (sl[2] + sl[3]);
    const int h = rho >> 1, qi = rho & 1;
    g[((long)h * nv + b * 2 + qi) * C + k] = Gs / Ls;
    if (ml_out && k == 0) {
      ml_out[((long)b * NR + rho) * 2] = M;
      ml_out[((long)b * NR + rho) * 2 + 1] = Ls;
    }
  }
}

// Training-mode output dropout (transformer.py:52,80): y = dropout(fc(o)) + q, in place on y =
// fc(o) (stream 2, index v*C + k).
__global__ void dropout_residual_kernel(float* __restrict__ y, const float* __restrict__ q, int n, float p,
                                        unsigned long long seed) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = y[i] * dropout_scale(p, seed, 2, i) + q[i];
}

// LayerNorm over C=512 per row (nn.LayerNorm(512), eps 1e-5, biased variance).
__global__ void layernorm_kernel(const float* __restrict__ y, const float* __restrict__ w,
                                 const float* __restrict__ bb, float* __restrict__ out, float* __restrict__ stats,
                                 float eps) {
  constexpr int C = 512;
  const int v = blockIdx.x, lane = threadIdx.x;
  const float* yr = y + (long)v * C;
  float x[8];
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    x[q] = yr[lane + 64 * q];
    s += x[q];
  }
  const float mean = wave_sum(s) / (float)C;
  float ss = 0.f;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const float d = x[q] - mean;
    ss = fmaf(d, d, ss);
  }
  const float var = wave_sum(ss) / (float)C;
  const float rstd = 1.0f / sqrtf(var + eps);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int k = lane + 64 * q;
    out[(long)v * C + k] = (x[q] - mean) * rstd * w[k] + bb[k];
  }
  if (stats && lane == 0) {
    stats[v * 2] = mean;
    stats[v * 2 + 1] = rstd;
  }
}

// ---------------------------------------------------------------------------------------
// Saved-tensor layout for the backward pass (floats), nv = 2B, NR = 2H:
//   qp[nv][H*C] | r[H][nv][C] | g[H][nv][C] | o[nv][H*C] | y[nv][C] | ln[nv][2] |
//   ml[B][NR][2] | scores[B][NR][hw]
// ---------------------------------------------------------------------------------------
struct SavedLayout {
  long qp, r, g, o, y, ln, ml, sc, total;
};
static SavedLayout saved_layout(int B, int hw, int C, int H) {
  SavedLayout L;
  const long nv = 2L * B, NR = 2L * H;
  long off = 0;
  L.qp = off; off += nv * H * C;
  L.r = off; off += (long)H * nv * C;
  L.g = off; off += (long)H * nv * C;
  L.o = off; off += nv * H * C;
  L.y = off; off += nv * C;
  L.ln = off; off += nv * 2;
  L.ml = off; off += (long)B * NR * 2;
  L.sc = off; off += (long)B * NR * hw;
  L.total = off;
  return L;
}
size_t attention_saved_floats(int B, int hw, int C, int H) { return (size_t)saved_layout(B, hw, C, H).total; }

size_t attention_ws_floats(int B, int hw, int C, int H) {
  const int nchunk = cdiv(hw, ATT_TPB);
  return (size_t)saved_layout(B, hw, C, H).total + (size_t)B * nchunk * 2 * H * (C + 2);
}

int attention_fwd(const float* q, const float* f, int B, int hw, int C, int H, const float* w_qkvs,
                  const float* fc_w, const float* fc_b, const float* ln_w, const float* ln_b, float* out,
                  float* saved, float* ws, hipStream_t st, float p_attn, float p_out, unsigned long long seed) {
  if (C != 512) return fail(CWT_EARG, "attention: C must be 512");
  if (!(H == 1 || H == 2 || H == 4)) return fail(CWT_EARG, "attention: heads must be 1, 2 or 4");
  const int nv = 2 * B;
  const int NR = 2 * H;
  SavedLayout L = saved_layout(B, hw, C, H);
  float* sv = saved ? saved : ws;  // scratch holds the same layout when no backward is needed
  float* part = ws + L.total;
  const int nchunk = cdiv(hw, ATT_TPB);
  float* part_g = part;
  float* part_ml = part + (long)B * nchunk * NR * C;
  const float inv_t = 1.0f / sqrtf((float)C);
  int rc;
  // 1. qp[v][j] = w_qkvs[j] . q[v]
  if ((rc = launch_rowdot(w_qkvs, H * C, C, q, nv, C, 0, H * C, nullptr, nullptr, 0, sv + L.qp, (long)H * C, 1.f,
                          st, sv + L.r, (long)H * nv * C)))
    return rc;
  // 2. r[h][v][k] = sum_d w_qkvs[h*C+d][k] qp[v][h*C+d] / sqrt(C)  (r cleared by step 1's launch)
  if ((rc = launch_coldot(w_qkvs, H, C, C, sv + L.qp, nv, (long)H * C, sv + L.r, inv_t, st))) return rc;
  // 3. chunk partials over the token map
  dim3 g3(nchunk, B);
  float* sc_out = saved ? sv + L.sc : nullptr;
  if (H == 1)
    hipLaunchKernelGGL((attn_partial_kernel<2>), g3, dim3(256), 0, st, sv + L.r, f, hw, nv, part_g, part_ml, sc_out,
                       p_attn, seed);
  else if (H == 2)
    hipLaunchKernelGGL((attn_partial_kernel<4>), g3, dim3(256), 0, st, sv + L.r, f, hw, nv, part_g, part_ml, sc_out,
                       p_attn, seed);
  else
    hipLaunchKernelGGL((attn_partial_kernel<8>), g3, dim3(256), 0, st, sv + L.r, f, hw, nv, part_g, part_ml, sc_out,
                       p_attn, seed);
  CWT_LAUNCH_CHECK();
  // 4. combine -> g[h][v][C]
  dim3 g4(C / 64, NR, B);
  if (H == 1)
    hipLaunchKernelGGL((attn_combine_kernel<2>), g4, dim3(256), 0, st, part_g, part_ml, nchunk, nv, sv + L.g, sv + L.ml);
  else if (H == 2)
    hipLaunchKernelGGL((attn_combine_kernel<4>), g4, dim3(256), 0, st, part_g, part_ml, nchunk, nv, sv + L.g, sv + L.ml);
  else
    hipLaunchKernelGGL((attn_combine_kernel<8>), g4, dim3(256), 0, st, part_g, part_ml, nchunk, nv, sv + L.g, sv + L.ml);
  CWT_LAUNCH_CHECK();
  // 5. o[v][h*C+d] = w_qkvs[h*C+d] . g[h][v]
  if ((rc = launch_rowdot(w_qkvs, H * C, C, sv + L.g, nv, C, (long)nv * C, C, nullptr, nullptr, 0, sv + L.o,
                          (long)H * C, 1.f, st)))
    return rc;
  // 6. y[v][d] = fc_w[d] . o[v] + fc_b[d] + q[v][d]   (with output dropout on the fc term)
  if ((rc = launch_rowdot(fc_w, C, H * C, sv + L.o, nv, (long)H * C, 0, C, fc_b, p_out > 0.f ? nullptr : q, C,
                          sv + L.y, C, 1.f, st)))
    return rc;
  if (p_out > 0.f) {
    hipLaunchKernelGGL(dropout_residual_kernel, dim3(cdiv(nv * C, 256)), dim3(256), 0, st, sv + L.y, q, nv * C, p_out,
                       seed);
    CWT_LAUNCH_CHECK();
  }
  // 7. LayerNorm
  hipLaunchKernelGGL(layernorm_kernel, dim3(nv), dim3(64), 0, st, sv + L.y, ln_w, ln_b, out, sv + L.ln, 1e-5f);
  CWT_LAUNCH_CHECK();
  return 0;
}


// ---------------------------------------------------------------------------------------
// Backward (train.py:264 loss_q.backward through the CWT; q and f carry no gradient).
// With a_hi = W_h q_i, r_hi = W_h^T a_hi / tau, s = r.f, P = softmax(s), g = P.f, o = W_h g:
//   dy   = LayerNorm'(d_out)               dln_w += d_out*xhat, dln_b += d_out
//   dfc_b += dy ; dfc_w += dy o^T ;  do = fc_w^T dy
//   dg_h = W_h^T do_h
//   dr_h = sum_p P_p (dg_h.f_p - dg_h.g_h) f_p            (one pass over the token map)
//   da_h = W_h dr_h / tau
//   dW_h += do_h g_h^T + a_h dr_h^T / tau + da_h q^T        (rank-3nv update per head)
// ---------------------------------------------------------------------------------------

// One workgroup of 512 threads (thread = channel k) handles every row v.
// dy is the gradient w.r.t. the fc output: the LayerNorm input gradient times the output-dropout
// mask (p_out > 0; regenerated from the forward's seed).
__global__ __launch_bounds__(512) void ln_bwd_kernel(const float* __restrict__ d_out, const float* __restrict__ y,
                                                     const float* __restrict__ stats, const float* __restrict__ w,
                                                     int nv, float* __restrict__ dy, float* __restrict__ g_w,
                                                     float* __restrict__ g_b, float* __restrict__ g_fc_b, float p_out,
                                                     unsigned long long seed) {
  constexpr int C = 512;
  __shared__ float red[2][8];
  const int k = threadIdx.x, lane = k & 63, wv = k >> 6;
  float gw = 0.f, gb = 0.f, gfb = 0.f;
  for (int v = 0; v < nv; ++v) {
    const float mean = stats[v * 2], rstd = stats[v * 2 + 1];
    const float xh = (y[(long)v * C + k] - mean) * rstd;
    const float go = d_out[(long)v * C + k];
    gw = fmaf(go, xh, gw);
    gb += go;
    const float dxh = go * w[k];
    float s1 = wave_sum(dxh), s2 = wave_sum(dxh * xh);
    if (lane == 0) {
      red[0][wv] = s1;
      red[1][wv] = s2;
    }
    __syncthreads();
    float m1 = 0.f, m2 = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      m1 += red[0][i];
      m2 += red[1][i];
    }
    __syncthreads();
    m1 /= (float)C;
    m2 /= (float)C;
    float d = rstd * (dxh - m1 - xh * m2);
    if (p_out > 0.f) d *= dropout_scale(p_out, seed, 2, (unsigned long long)v * C + k);
    dy[(long)v * C + k] = d;
    gfb += d;
  }
  g_w[k] += gw;
  g_b[k] += gb;
  g_fc_b[k] += gfb;
}

struct OuterTerm {
  const float* u;  // u[v*u_vs + j]
  long u_vs;
  const float* V;  // V[v*V_vs + g*V_gs + k]
  long V_vs, V_gs;
  float alpha;
};

// G[j][k] += sum_t alpha_t sum_v u_t[v][j] * V_t[v][group(j)][k]; thread per (j, 4 k's)
__global__ void outer_acc_kernel(float* __restrict__ G, int R, int K, int rows_per_group, int nv, OuterTerm t0,
                                 OuterTerm t1, OuterTerm t2, int nterms) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int k4n = K >> 2;
  if (idx >= (long)R * k4n) return;
  const int j = (int)(idx / k4n);
  const int k = (int)(idx - (long)j * k4n) * 4;
  const int g = j / rows_per_group;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const OuterTerm ts[3] = {t0, t1, t2};
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    if (t >= nterms) break;
    f32x4 a = {0.f, 0.f, 0.f, 0.f};
    for (int v = 0; v < nv; ++v) {
      const float u = ts[t].u[v * ts[t].u_vs + j];
      const f32x4 vv = *(const f32x4*)(ts[t].V + v * ts[t].V_vs + g * ts[t].V_gs + k);
      a += u * vv;
    }
    acc += ts[t].alpha * a;
  }
  *(f32x4*)(G + (long)j * K + k) += acc;
}

static int launch_outer(float* G, int R, int K, int rows_per_group, int nv, OuterTerm t0, OuterTerm t1, OuterTerm t2,
                        int nterms, hipStream_t st) {
  const long total = (long)R * (K / 4);
  hipLaunchKernelGGL(outer_acc_kernel, dim3(cdiv(total, 256)), dim3(256), 0, st, G, R, K, rows_per_group, nv, t0, t1,
                     t2, nterms);
  CWT_LAUNCH_CHECK();
  return 0;
}

// dr[h][b*2+i][k] += sum_p P_p (dg.f_p - dg.g) f_p over the workgroup's tokens
// With attention dropout (g = sum_p m_p P_p f_p): ds_p = P_p (m_p dg.f_p - dg.g).
template <int NR>
__global__ __launch_bounds__(256) void attn_bwd_kernel(const float* __restrict__ dg, const float* __restrict__ g,
                                                       const float* __restrict__ f, const float* __restrict__ scores,
                                                       const float* __restrict__ ml, int hw, int nv,
                                                       float* __restrict__ dr, float p_drop, unsigned long long seed) {
  constexpr int C = 512;
  __shared__ float dgs[NR][C];
  __shared__ float dgg[NR];
  __shared__ float wred[4][NR][C];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int chunk = blockIdx.x, b = blockIdx.y;
  for (int i = t; i < NR * C; i += 256) {
    const int rho = i / C, k = i % C;
    dgs[rho][k] = dg[((long)(rho >> 1) * nv + b * 2 + (rho & 1)) * C + k];
  }
  // dg . g per row (one wave per row, redundantly per workgroup: 8 x 512 MACs)
  for (int rho = wv; rho < NR; rho += 4) {
    const float* gr = g + ((long)(rho >> 1) * nv + b * 2 + (rho & 1)) * C;
    const float* dr_ = dg + ((long)(rho >> 1) * nv + b * 2 + (rho & 1)) * C;
    float s = 0.f;
    for (int k = lane; k < C; k += 64) s = fmaf(dr_[k], gr[k], s);
    s = wave_sum(s);
    if (lane == 0) dgg[rho] = s;
  }
  __syncthreads();
  const int tok0 = chunk * ATT_TPB + wv * ATT_TPW;
  float fv[ATT_TPW][8];
#pragma unroll
  for (int tt = 0; tt < ATT_TPW; ++tt) {
    const int p = tok0 + tt;
    if (p < hw) {
      const float* src = f + ((long)b * hw + p) * C + lane * 8;
      f32x4 u = *(const f32x4*)src, v = *(const f32x4*)(src + 4);
      fv[tt][0] = u[0]; fv[tt][1] = u[1]; fv[tt][2] = u[2]; fv[tt][3] = u[3];
      fv[tt][4] = v[0]; fv[tt][5] = v[1]; fv[tt][6] = v[2]; fv[tt][7] = v[3];
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) fv[tt][q] = 0.f;
    }
  }
#pragma unroll
  for (int rho = 0; rho < NR; ++rho) {
    float dv[8];
    f32x4 u = *(const f32x4*)&dgs[rho][lane * 8], v = *(const f32x4*)&dgs[rho][lane * 8 + 4];
    dv[0] = u[0]; dv[1] = u[1]; dv[2] = u[2]; dv[3] = u[3]; dv[4] = v[0]; dv[5] = v[1]; dv[6] = v[2]; dv[7] = v[3];
    const float M = ml[((long)b * NR + rho) * 2], Linv = 1.f / ml[((long)b * NR + rho) * 2 + 1];
    float acc[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = 0.f;
#pragma unroll
    for (int tt = 0; tt < ATT_TPW; ++tt) {
      float d = 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q) d = fmaf(dv[q], fv[tt][q], d);
      d = wave_sum(d);
      const int p = tok0 + tt;
      if (p < hw) {
        const float P = __expf(scores[((long)b * NR + rho) * hw + p] - M) * Linv;
        const float dm = p_drop > 0.f ? d * dropout_scale(p_drop, seed, 1, ((long)b * NR + rho) * hw + p) : d;
        const float ds = P * (dm - dgg[rho]);
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[q] = fmaf(ds, fv[tt][q], acc[q]);
      }
    }
    *(f32x4*)&wred[wv][rho][lane * 8] = f32x4{acc[0], acc[1], acc[2], acc[3]};
    *(f32x4*)&wred[wv][rho][lane * 8 + 4] = f32x4{acc[4], acc[5], acc[6], acc[7]};
  }
  __syncthreads();
  for (int i = t; i < NR * C; i += 256) {
    const int rho = i / C, k = i % C;
    const float s = (wred[0][rho][k] + wred[1][rho][k]) + (wred[2][rho][k] + wred[3][rho][k]);
    atomicAdd(&dr[((long)(rho >> 1) * nv + b * 2 + (rho & 1)) * C + k], s);
  }
}

size_t attention_bwd_ws_floats(int B, int hw, int C, int H) {
  const long nv = 2L * B;
  // dy[nv][C] | do[nv][HC] | dg[H][nv][C] | dr[H][nv][C] | da[nv][HC]
  return (size_t)(nv * C + nv * H * C + 2L * H * nv * C + nv * H * C);
}

int attention_bwd(const float* q, const float* f, int B, int hw, int C, int H, const float* w_qkvs,
                  const float* fc_w, const float* fc_b, const float* ln_w, const float* ln_b, const float* saved,
                  const float* d_out, float* g_w_qkvs, float* g_fc_w, float* g_fc_b, float* g_ln_w, float* g_ln_b,
                  float* ws, hipStream_t st, float p_attn, float p_out, unsigned long long seed) {
  (void)fc_b;
  (void)ln_b;
  if (C != 512) return fail(CWT_EARG, "attention: C must be 512");
  if (!(H == 1 || H == 2 || H == 4)) return fail(CWT_EARG, "attention: heads must be 1, 2 or 4");
  const int nv = 2 * B, NR = 2 * H;
  const long HC = (long)H * C;
  SavedLayout L = saved_layout(B, hw, C, H);
  const float* qp = saved + L.qp;
  const float* g = saved + L.g;
  const float* o = saved + L.o;
  const float* y = saved + L.y;
  float* dy = ws;
  float* dO = dy + (long)nv * C;
  float* dg = dO + (long)nv * HC;
  float* dr = dg + (long)H * nv * C;
  float* da = dr + (long)H * nv * C;
  const float inv_t = 1.0f / sqrtf((float)C);
  int rc;
  hipLaunchKernelGGL(ln_bwd_kernel, dim3(1), dim3(512), 0, st, d_out, y, saved + L.ln, ln_w, nv, dy, g_ln_w, g_ln_b,
                     g_fc_b, p_out, seed);
  CWT_LAUNCH_CHECK();
  OuterTerm none{nullptr, 0, nullptr, 0, 0, 0.f};
  OuterTerm tfc{dy, C, o, HC, 0, 1.f};
  if ((rc = launch_outer(g_fc_w, C, (int)HC, C, nv, tfc, none, none, 1, st))) return rc;
  CWT_HIP(hipMemsetAsync(dO, 0, sizeof(float) * nv * HC, st));
  if ((rc = launch_coldot(fc_w, 1, C, (int)HC, dy, nv, C, dO, 1.f, st))) return rc;
  CWT_HIP(hipMemsetAsync(dg, 0, sizeof(float) * H * nv * C, st));
  if ((rc = launch_coldot(w_qkvs, H, C, C, dO, nv, HC, dg, 1.f, st))) return rc;
  CWT_HIP(hipMemsetAsync(dr, 0, sizeof(float) * H * nv * C, st));
  const int nchunk = cdiv(hw, ATT_TPB);
  dim3 gb(nchunk, B);
  if (H == 1)
    hipLaunchKernelGGL((attn_bwd_kernel<2>), gb, dim3(256), 0, st, dg, g, f, saved + L.sc, saved + L.ml, hw, nv, dr,
                       p_attn, seed);
  else if (H == 2)
    hipLaunchKernelGGL((attn_bwd_kernel<4>), gb, dim3(256), 0, st, dg, g, f, saved + L.sc, saved + L.ml, hw, nv, dr,
                       p_attn, seed);
  else
    hipLaunchKernelGGL((attn_bwd_kernel<8>), gb, dim3(256), 0, st, dg, g, f, saved + L.sc, saved + L.ml, hw, nv, dr,
                       p_attn, seed);
  CWT_LAUNCH_CHECK();
  if ((rc = launch_rowdot(w_qkvs, (int)HC, C, dr, nv, C, (long)nv * C, C, nullptr, nullptr, 0, da, HC, inv_t, st)))
    return rc;
  OuterTerm t0{dO, HC, g, C, (long)nv * C, 1.f};
  OuterTerm t1{qp, HC, dr, C, (long)nv * C, inv_t};
  OuterTerm t2{da, HC, q, C, 0, 1.f};
  return launch_outer(g_w_qkvs, (int)HC, C, C, nv, t0, t1, t2, 3, st);
}

}  // namespace cwt

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
#include "pretrain.h"

#include <cstring>

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

// ---------------------------------------------------------------------------------------
// Inference tail with the token normalisation fused (test.py:190-197: f_hat = F.normalize(f_q),
// pred_q0 = W . f_q, W' = transformer(W, f_hat, f_hat)).  The token map is read ONCE, raw: per
// token p, inv_p = 1 / max(||f_p||, 1e-12) (so f_hat_p = inv_p f_p), the scores
// s = (r . f_p) inv_p, the baseline logits W . f_p, and the softmax partials with weight
// e inv_p on f_p.  No normalised copy of the map is written; the classifier then scales W'.f_p by
// inv_p (classify_scaled_kernel).  Rows are [B][NR][C] with rho = qi * H + h.
// ---------------------------------------------------------------------------------------
constexpr int TOK_TPW = 4;                 // tokens per wave
constexpr int TOK_NW = 8;                  // waves per workgroup (two per SIMD)
constexpr int TOK_TPB = TOK_NW * TOK_TPW;  // tokens per workgroup (one chunk)

template <int NR>
__global__ __launch_bounds__(TOK_NW * 64) void attn_tokens_kernel(const float* __restrict__ r,
                                                                  const float* __restrict__ f, int hw,
                                                                  const float* __restrict__ W0,
                                                                  float* __restrict__ part_g,
                                                                  float* __restrict__ part_ml,
                                                                  float* __restrict__ inv_norm,
                                                                  float* __restrict__ logits0) {
  static_assert(NR * TOK_TPW == 32, "NR rows x 4 tokens = the first 32 lanes of the butterfly");
  constexpr int C = 512;
  constexpr int NT = TOK_NW * 64;
  __shared__ __attribute__((aligned(16))) float rs[NR + 2][C];       // score rows, then the two rows of W0
  __shared__ __attribute__((aligned(16))) float wg[TOK_NW][NR][C];   // per-wave exp-weighted token sums
  __shared__ float wml[TOK_NW][NR][2];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int chunk = blockIdx.x, b = blockIdx.y, nchunk = gridDim.x;
  for (int i = t; i < (NR + 2) * (C / 4); i += NT) {
    const int row = i / (C / 4), c4 = i - row * (C / 4);
    f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
    if (row < NR)
      v = ((const f32x4*)(r + ((long)b * NR + row) * C))[c4];
    else if (W0)
      v = ((const f32x4*)(W0 + ((long)b * 2 + row - NR) * C))[c4];
    *(f32x4*)&rs[row][c4 * 4] = v;
  }
  // lane owns channels [4 lane, 4 lane + 4) and [256 + 4 lane, 256 + 4 lane + 4): every f load
  // and LDS access of the wave is one contiguous 1-KB row (conflict-free)
  const int tok0 = chunk * TOK_TPB + wv * TOK_TPW;
  f32x4 fa[TOK_TPW], fb[TOK_TPW];
#pragma unroll
  for (int tt = 0; tt < TOK_TPW; ++tt) {
    const int p = tok0 + tt;
    if (p < hw) {
      const float* src = f + ((long)b * hw + p) * C + 4 * lane;
      fa[tt] = *(const f32x4*)src;
      fb[tt] = *(const f32x4*)(src + 256);
    } else {
      fa[tt] = fb[tt] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  __syncthreads();
  auto dot8 = [](f32x4 a0, f32x4 a1, f32x4 b0, f32x4 b1) {
    float d = a0[0] * b0[0];
    d = fmaf(a0[1], b0[1], d);
    d = fmaf(a0[2], b0[2], d);
    d = fmaf(a0[3], b0[3], d);
    d = fmaf(a1[0], b1[0], d);
    d = fmaf(a1[1], b1[1], d);
    d = fmaf(a1[2], b1[2], d);
    return fmaf(a1[3], b1[3], d);
  };
  // 64 per-lane partial dot products, reduced over the wave by ONE butterfly:
  //   [tt * NR + rho] (32): r_rho . f_tt;   [32 + tt * 8 + j] (32): |f_tt|^2, W0_0 . f_tt, W0_1 . f_tt
  float v[64];
#pragma unroll
  for (int rho = 0; rho < NR; ++rho) {
    const f32x4 ra = *(const f32x4*)&rs[rho][4 * lane], rb = *(const f32x4*)&rs[rho][256 + 4 * lane];
#pragma unroll
    for (int tt = 0; tt < TOK_TPW; ++tt) v[tt * NR + rho] = dot8(ra, rb, fa[tt], fb[tt]);
  }
  {
    const f32x4 w0a = *(const f32x4*)&rs[NR][4 * lane], w0b = *(const f32x4*)&rs[NR][256 + 4 * lane];
    const f32x4 w1a = *(const f32x4*)&rs[NR + 1][4 * lane], w1b = *(const f32x4*)&rs[NR + 1][256 + 4 * lane];
#pragma unroll
    for (int tt = 0; tt < TOK_TPW; ++tt) {
      v[32 + tt * 8] = dot8(fa[tt], fb[tt], fa[tt], fb[tt]);
      v[32 + tt * 8 + 1] = dot8(w0a, w0b, fa[tt], fb[tt]);
      v[32 + tt * 8 + 2] = dot8(w1a, w1b, fa[tt], fb[tt]);
#pragma unroll
      for (int j = 3; j < 8; ++j) v[32 + tt * 8 + j] = 0.f;
    }
  }
  const float red = butterfly_sum<64>(v, lane);  // lane L: value L
  const bool score_lane = lane < 32;
  const int my_t = (lane & 31) / NR, my_rho = lane % NR;
  const int p = tok0 + my_t;
  const bool valid = score_lane && p < hw;
  const float nrm2 = __shfl(red, 32 + my_t * 8, 64);  // |f|^2 of this lane's token
  const float inv = 1.0f / fmaxf(sqrtf(nrm2), 1e-12f);
  if (valid && my_rho == 0) inv_norm[(long)b * hw + p] = inv;
  if (logits0 && lane >= 32 && ((lane & 7) == 1 || (lane & 7) == 2)) {  // W0 . f of token (lane - 32) / 8
    const int pt = tok0 + ((lane - 32) >> 3);
    if (pt < hw) logits0[((long)b * 2 + (lane & 7) - 1) * hw + pt] = red;
  }
  const float sc = valid ? red * inv : -INFINITY;
  // softmax partial per row over the wave's 4 tokens (score lanes of one row differ in bits 3, 4)
  float m = sc;
  m = fmaxf(m, __shfl_xor(m, 8, 64));
  m = fmaxf(m, __shfl_xor(m, 16, 64));
  const float e = valid ? __expf(sc - m) : 0.f;
  float l = e;
  l += __shfl_xor(l, 8, 64);
  l += __shfl_xor(l, 16, 64);
  const float wgt = e * inv;  // f_hat = inv f: the token's weight on the raw f
  f32x4 ga[NR], gb[NR];
#pragma unroll
  for (int rho = 0; rho < NR; ++rho) ga[rho] = gb[rho] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int tt = 0; tt < TOK_TPW; ++tt)
#pragma unroll
    for (int rho = 0; rho < NR; ++rho) {
      const float w = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wgt), tt * NR + rho));
      ga[rho] += w * fa[tt];
      gb[rho] += w * fb[tt];
    }
#pragma unroll
  for (int rho = 0; rho < NR; ++rho) {
    *(f32x4*)&wg[wv][rho][4 * lane] = ga[rho];
    *(f32x4*)&wg[wv][rho][256 + 4 * lane] = gb[rho];
  }
  if (lane < NR) {  // lane rho (token 0) carries its row's max and sum
    wml[wv][lane][0] = m;
    wml[wv][lane][1] = l;
  }
  __syncthreads();
  for (int i = t; i < NR * (C / 4); i += NT) {
    const int rho = i / (C / 4), c4 = i - rho * (C / 4);
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < TOK_NW; ++w) M = fmaxf(M, wml[w][rho][0]);
    f32x4 G = f32x4{0.f, 0.f, 0.f, 0.f};
    float L = 0.f;
#pragma unroll
    for (int w = 0; w < TOK_NW; ++w) {
      const float s = (wml[w][rho][0] == -INFINITY) ? 0.f : __expf(wml[w][rho][0] - M);
      G += s * *(const f32x4*)&wg[w][rho][c4 * 4];
      L = fmaf(s, wml[w][rho][1], L);
    }
    *(f32x4*)&part_g[(((long)b * nchunk + chunk) * NR + rho) * C + c4 * 4] = G;
    if (c4 == 0) {
      part_ml[(((long)b * nchunk + chunk) * NR + rho) * 2] = M;
      part_ml[(((long)b * nchunk + chunk) * NR + rho) * 2 + 1] = L;
    }
  }
}

// g[b][rho][k] = sum_c e^{m_c - M} G_c[k] / sum_c e^{m_c - M} l_c in ONE pass: the chunk maxima
// and sums go to LDS first (M from there), then each thread issues all its chunks' loads.
// Block = (64 channels, row rho, batch b); its 4 waves take every 4th chunk.
constexpr int TOK_MAXCHUNK = 512;
template <int NR>
__global__ __launch_bounds__(256) void attn_combine1_kernel(const float* __restrict__ part_g,
                                                            const float* __restrict__ part_ml, int nchunk,
                                                            float* __restrict__ g) {
  constexpr int C = 512;
  __shared__ float ms[TOK_MAXCHUNK], ls[TOK_MAXCHUNK];
  __shared__ float sg[4][64], red[4];
  const int t = threadIdx.x, kk = t & 63, cg = t >> 6;
  const int k = blockIdx.x * 64 + kk;
  const int rho = blockIdx.y, b = blockIdx.z;
  for (int c = t; c < nchunk; c += 256) {
    ms[c] = part_ml[(((long)b * nchunk + c) * NR + rho) * 2];
    ls[c] = part_ml[(((long)b * nchunk + c) * NR + rho) * 2 + 1];
  }
  __syncthreads();
  float M = -INFINITY;
  for (int c = kk; c < nchunk; c += 64) M = fmaxf(M, ms[c]);
  M = wave_max(M);
  const float* pg = part_g + ((long)b * nchunk * NR + rho) * C + k;
  float G = 0.f, L = 0.f;
  for (int c0 = cg; c0 < nchunk; c0 += 64) {  // 16 chunks per round, all loads in flight
    float gc[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) gc[u] = pg[(long)min(c0 + 4 * u, nchunk - 1) * NR * C];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int c = c0 + 4 * u;
      if (c >= nchunk) break;
      const float s = (ms[c] == -INFINITY) ? 0.f : __expf(ms[c] - M);
      G = fmaf(s, gc[u], G);
      L = fmaf(s, ls[c], L);
    }
  }
  sg[cg][kk] = G;
  if (kk == 0) red[cg] = L;
  __syncthreads();
  if (cg == 0) {
    const float Gs = (sg[0][kk] + sg[1][kk]) + (sg[2][kk] + sg[3][kk]);
    const float Ls = (red[0] + red[1]) + (red[2] + red[3]);
    g[((long)b * NR + rho) * C + k] = Gs / Ls;
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
// Inference with folded weights.  For fixed parameters the two products around the token pass
// fold into per-head 512 x 512 matrices (computed once per parameter version, attention_fold):
//   M_h = W_h^T W_h          =>  r_h = M_h q / sqrt(C)            (replaces W_h q, then W_h^T a)
//   P   = [fc_h W_h]_h       =>  y = P [g_h]_h + fc_b + q          (replaces W_h g, then fc)
// the same function re-associated once more (fp32 rounding only), 5 launches instead of 8 and
// 8 MB of weight reads per episode instead of 16.
// ---------------------------------------------------------------------------------------
size_t attention_fold_floats(int C, int H) { return 2 * (size_t)H * C * C; }

int attention_fold(const float* w_qkvs, const float* fc_w, int C, int H, float* fold, float* ws, size_t ws_floats,
                   hipStream_t st) {
  float* M = fold;                      // [H][C][C]
  float* P = fold + (size_t)H * C * C;  // [C][H*C]
  int rc;
  for (int h = 0; h < H; ++h) {
    PtGemm g;
    std::memset(&g, 0, sizeof(g));
    g.A = w_qkvs + (size_t)h * C * C;   // A(i, d) = W[h*C + d][i]
    g.sai = 1;
    g.sak = C;
    g.B = w_qkvs + (size_t)h * C * C;   // B(d, j) = W[h*C + d][j]
    g.sbk = C;
    g.sbj = 1;
    g.C = M + (size_t)h * C * C;
    g.ldc = C;
    g.M = C;
    g.N = C;
    g.K = C;
    if ((rc = launch_pt_gemm(g, ws, ws_floats, st))) return rc;
    std::memset(&g, 0, sizeof(g));
    g.A = fc_w + (size_t)h * C;         // A(j, d) = fc_w[j][h*C + d]
    g.sai = (long)H * C;
    g.sak = 1;
    g.B = w_qkvs + (size_t)h * C * C;   // B(d, k) = W[h*C + d][k]
    g.sbk = C;
    g.sbj = 1;
    g.C = P + (size_t)h * C;            // P[j][h*C + k]
    g.ldc = (long)H * C;
    g.M = C;
    g.N = C;
    g.K = C;
    if ((rc = launch_pt_gemm(g, ws, ws_floats, st))) return rc;
  }
  return 0;
}

size_t attention_infer_ws_floats(int B, int hw, int C, int H) {
  const long NR = 2L * H, nchunk = cdiv(hw, TOK_TPB);
  return (size_t)(B * NR * C + B * nchunk * NR * (C + 2) + B * NR * C + 2L * B * C);
}

// q [B][2][C] (the inner loop's W), f [B][hw][C] raw query features; outputs W' [B][2][C],
// inv_norm [B][hw] and, when logits0 is given, the baseline logits W . f [B][2][hw].
int attention_infer(const float* q, const float* f, int B, int hw, int C, int H, const float* fold, const float* fc_b,
                    const float* ln_w, const float* ln_b, float* out, float* inv_norm, float* logits0, float* ws,
                    hipStream_t st) {
  if (C != 512 || H != 4) return fail(CWT_EARG, "attention_infer: C = 512 and 4 heads (the fused token pass)");
  constexpr int NR = 8;
  const int nv = 2 * B, nchunk = cdiv(hw, TOK_TPB);
  if (nchunk > TOK_MAXCHUNK) return fail(CWT_EARG, "attention_infer: hw too large");
  const float* M = fold;
  const float* P = fold + (size_t)H * C * C;
  float* r = ws;                                  // [B][NR][C] = [nv][H][C]
  float* part_g = r + (size_t)B * NR * C;          // [B][nchunk][NR][C]
  float* part_ml = part_g + (size_t)B * nchunk * NR * C;
  float* g = part_ml + (size_t)B * nchunk * NR * 2;  // [B][NR][C] = [nv][H][C]
  float* y = g + (size_t)B * NR * C;              // [nv][C]
  int rc;
  // 1. r[v][h*C + k] = M_h[k] . q[v] / sqrt(C)
  if ((rc = launch_rowdot(M, H * C, C, q, nv, C, 0, H * C, nullptr, nullptr, 0, r, (long)H * C,
                          1.0f / sqrtf((float)C), st)))
    return rc;
  // 2. the token pass (normalisation, baseline logits, chunk partials)
  hipLaunchKernelGGL((attn_tokens_kernel<NR>), dim3(nchunk, B), dim3(TOK_NW * 64), 0, st, (const float*)r, f, hw, q, part_g,
                     part_ml, inv_norm, logits0);
  CWT_LAUNCH_CHECK();
  // 3. g = softmax-weighted token means
  hipLaunchKernelGGL((attn_combine1_kernel<NR>), dim3(C / 64, NR, B), dim3(256), 0, st, (const float*)part_g,
                     (const float*)part_ml, nchunk, g);
  CWT_LAUNCH_CHECK();
  // 4. y[v] = P . g[v] + fc_b + q[v]
  if ((rc = launch_rowdot(P, C, H * C, g, nv, (long)H * C, 0, C, fc_b, q, C, y, C, 1.f, st))) return rc;
  // 5. LayerNorm
  hipLaunchKernelGGL(layernorm_kernel, dim3(nv), dim3(64), 0, st, (const float*)y, ln_w, ln_b, out, (float*)nullptr,
                     1e-5f);
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

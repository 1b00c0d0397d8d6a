// Variant heads on the same features:
//
//  * CosCls, the cosine classifier (reference src/model/pspnet.py:290-313): per pixel
//      scores[k] = scale * (W_eff[k] . x / max(||x||_2, 1e-5) + bias[k])
//    with W_eff = g[k] * v[k] / ||v[k]|| under WeightNorm ('r'), else the stored weight, row-
//    normalised (eps 1e-5) in place first when weight_norm ('n').  Forward, and the backward
//    to the head's own parameters (weight / (g, v), bias, learnable scale 't'); the extractor
//    is frozen on every path that uses the head, so no input gradient.
//  * get_corr (reference src/model/model_util.py:101-109, the MMN / MatchNet correlation):
//      sim[b][i][j] = q_i . k_j / (max(||q_i||, 1e-12) max(||k_j||, 1e-12))
//    over the h*w tokens of two feature maps: a token normalisation pass, then an exact-fp32
//    NT GEMM on the fp32 matrix cores (v_mfma_f32_32x32x2_f32), [B][hw][hw] row-major.
//
// Features are the extractor's NHWC maps ([B][P][C], the token layout of the CWT kernels).
#include "common.h"
#include "kernels.h"

namespace cwt {

constexpr int HC_MAXN = 64;  // classes per launch of the cosine head (chunks of 8 in the kernels)

// ---- W_eff of the cosine head (one block, 256 threads; n <= 64, C = 512) ----
// mode bit 0: WeightNorm (W = g v / ||v||, torch._weight_norm, no eps); bit 1: weight_norm
// (rows normalised with eps 1e-5; without WeightNorm written back into v, as the reference's
// `self.cls.weight.data = F.normalize(...)` does -- with WeightNorm its pre-forward hook
// recomputes the weight from (g, v) after that assignment, so it has no effect).
__global__ void cos_weight_kernel(float* __restrict__ v, const float* __restrict__ gvec, int n, int C, int mode,
                                  float* __restrict__ w_eff, float* __restrict__ vnorm) {
  __shared__ float red[8];
  const int t = threadIdx.x;
  for (int k = 0; k < n; ++k) {
    float ss = 0.f;
    for (int c = t; c < C; c += blockDim.x) ss += v[(long)k * C + c] * v[(long)k * C + c];
    ss = wave_sum(ss);
    if ((t & 63) == 0) red[t >> 6] = ss;
    __syncthreads();
    float tot = 0.f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) tot += red[i];
    __syncthreads();
    const float nrm = sqrtf(tot);
    if (t == 0 && vnorm) vnorm[k] = nrm;
    float f = 1.f;
    if (mode & 1) {
      f = gvec[k] / nrm;
    } else if (mode & 2) {
      f = 1.f / fmaxf(nrm, 1e-5f);
    }
    for (int c = t; c < C; c += blockDim.x) {
      const float w = v[(long)k * C + c] * f;
      w_eff[(long)k * C + c] = w;
      if ((mode & 3) == 2) v[(long)k * C + c] = w;
    }
    __syncthreads();
  }
}

// ---- forward: one wave per pixel, lane = 8 channels; classes in chunks of 8 from LDS ----
__global__ __launch_bounds__(256) void cos_cls_fwd_kernel(const float* __restrict__ x, long P, int B, int n,
                                                          const float* __restrict__ w_eff,
                                                          const float* __restrict__ bias,
                                                          const float* __restrict__ scale, float* __restrict__ out) {
  constexpr int C = 512;
  __shared__ __attribute__((aligned(16))) float wl[HC_MAXN][C];
  for (int i = threadIdx.x; i < n * C; i += blockDim.x) (&wl[0][0])[i] = w_eff[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const long total = (long)B * P;
  const float sc = scale[0];
  for (long px = (long)blockIdx.x * 4 + (threadIdx.x >> 6); px < total; px += (long)gridDim.x * 4) {
    const float* xp = x + px * C + lane * 8;
    const f32x4 a = *(const f32x4*)xp, b = *(const f32x4*)(xp + 4);
    const float xv[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) ss = fmaf(xv[i], xv[i], ss);
    const float inv = 1.f / fmaxf(sqrtf(wave_sum_dpp(ss)), 1e-5f);
    const long bi = px / P, p = px - bi * P;
    for (int k0 = 0; k0 < n; k0 += 8) {
      float d[8];
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) {
        float s = 0.f;
        if (k0 + kk < n) {
          const f32x4 w0 = *(const f32x4*)&wl[k0 + kk][lane * 8], w1 = *(const f32x4*)&wl[k0 + kk][lane * 8 + 4];
          s = xv[0] * w0[0] + xv[1] * w0[1] + xv[2] * w0[2] + xv[3] * w0[3] + xv[4] * w1[0] + xv[5] * w1[1] +
              xv[6] * w1[2] + xv[7] * w1[3];
        }
        d[kk] = s;
      }
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) d[kk] = wave_sum_dpp(d[kk]);
      if (lane < 8 && k0 + lane < n) {
        float dv = d[0];
#pragma unroll
        for (int kk = 1; kk < 8; ++kk) dv = lane == kk ? d[kk] : dv;
        const float cosv = dv * inv + (bias ? bias[k0 + lane] : 0.f);
        out[(bi * n + k0 + lane) * P + p] = sc * cosv;
      }
    }
  }
}

// ---- backward to the head's parameters, fixed-order (deterministic) two-pass reduction ----
// pass 1 (block j of nb): partial[j][k][c] = sum over its pixels of dcos[k] * xhat[c] with
// dcos = scale * G; plus partial sums of dcos (bias) and of G * cos (scale), in part_s[j][k][2].
__global__ __launch_bounds__(256) void cos_cls_bwd_kernel(const float* __restrict__ x, long P, int B, int n,
                                                          const float* __restrict__ w_eff,
                                                          const float* __restrict__ bias,
                                                          const float* __restrict__ scale,
                                                          const float* __restrict__ G, float* __restrict__ part,
                                                          float* __restrict__ part_s) {
  constexpr int C = 512;
  __shared__ __attribute__((aligned(16))) float wl[8][C];
  __shared__ __attribute__((aligned(16))) float red[4][8][C];  // per wave, per class chunk
  __shared__ float reds[4][8][2];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const long total = (long)B * P;
  const float sc = scale[0];
  const long per = (total + gridDim.x - 1) / gridDim.x;
  const long p0 = blockIdx.x * per, p1 = min(total, p0 + per);
  for (int k0 = 0; k0 < n; k0 += 8) {
    __syncthreads();
    for (int i = threadIdx.x; i < 8 * C; i += blockDim.x) {
      const int kk = i / C;
      (&wl[0][0])[i] = k0 + kk < n ? w_eff[(long)(k0 + kk) * C + (i - kk * C)] : 0.f;
    }
    __syncthreads();
    float acc[8][8];
    float sb[8], ssc[8];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      sb[kk] = ssc[kk] = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[kk][i] = 0.f;
    }
    for (long px = p0 + wv; px < p1; px += 4) {
      const float* xp = x + px * C + lane * 8;
      const f32x4 a = *(const f32x4*)xp, b = *(const f32x4*)(xp + 4);
      float xv[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
      float ss = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) ss = fmaf(xv[i], xv[i], ss);
      const float inv = 1.f / fmaxf(sqrtf(wave_sum_dpp(ss)), 1e-5f);
#pragma unroll
      for (int i = 0; i < 8; ++i) xv[i] *= inv;
      const long bi = px / P, p = px - bi * P;
      float d[8];
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) {
        const f32x4 w0 = *(const f32x4*)&wl[kk][lane * 8], w1 = *(const f32x4*)&wl[kk][lane * 8 + 4];
        d[kk] = xv[0] * w0[0] + xv[1] * w0[1] + xv[2] * w0[2] + xv[3] * w0[3] + xv[4] * w1[0] + xv[5] * w1[1] +
                xv[6] * w1[2] + xv[7] * w1[3];
      }
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) {
        const float gk = k0 + kk < n ? G[(bi * n + k0 + kk) * P + p] : 0.f;
        const float dc = sc * gk;
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[kk][i] = fmaf(dc, xv[i], acc[kk][i]);
        const float cosv = wave_sum_dpp(d[kk]) + (bias && k0 + kk < n ? bias[k0 + kk] : 0.f);  // all lanes
        sb[kk] += dc;
        ssc[kk] = fmaf(gk, cosv, ssc[kk]);
      }
    }
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      *(f32x4*)&red[wv][kk][lane * 8] = f32x4{acc[kk][0], acc[kk][1], acc[kk][2], acc[kk][3]};
      *(f32x4*)&red[wv][kk][lane * 8 + 4] = f32x4{acc[kk][4], acc[kk][5], acc[kk][6], acc[kk][7]};
      if (lane == 0) {
        reds[wv][kk][0] = sb[kk];
        reds[wv][kk][1] = ssc[kk];
      }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 8 * C; i += blockDim.x) {
      const int kk = i / C, c = i - kk * C;
      if (k0 + kk < n)
        part[((long)blockIdx.x * n + k0 + kk) * C + c] =
            (red[0][kk][c] + red[1][kk][c]) + (red[2][kk][c] + red[3][kk][c]);
    }
    if (threadIdx.x < 16) {
      const int kk = threadIdx.x >> 1, w = threadIdx.x & 1;
      if (k0 + kk < n)
        part_s[((long)blockIdx.x * n + k0 + kk) * 2 + w] =
            (reds[0][kk][w] + reds[1][kk][w]) + (reds[2][kk][w] + reds[3][kk][w]);
    }
  }
}

// pass 2: sum the nb partials in block order; dW_eff -> (dv, dg) under WeightNorm, else dW;
// db[k]; dscale (one value).  One block of 256 threads.
__global__ void cos_cls_bwd_final_kernel(const float* __restrict__ part, const float* __restrict__ part_s, int nb,
                                         int n, int C, int mode, const float* __restrict__ v,
                                         const float* __restrict__ gvec, const float* __restrict__ vnorm,
                                         float* __restrict__ dv, float* __restrict__ dg, float* __restrict__ db,
                                         float* __restrict__ dscale) {
  __shared__ float red[8];
  const int t = threadIdx.x;
  for (int k = 0; k < n; ++k) {
    // dW_eff[k][c] for this thread's channels, and its dot with v-hat (WeightNorm)
    float dot = 0.f;
    for (int c = t; c < C; c += blockDim.x) {
      float s = 0.f;
      for (int j = 0; j < nb; ++j) s += part[((long)j * n + k) * C + c];
      if (mode & 1) {
        dot += s * v[(long)k * C + c];
        dv[(long)k * C + c] = s;  // dW_eff, finished below
      } else {
        dv[(long)k * C + c] = s;
      }
    }
    if (mode & 1) {
      dot = wave_sum(dot);
      if ((t & 63) == 0) red[t >> 6] = dot;
      __syncthreads();
      float tot = 0.f;
      for (int i = 0; i < (int)(blockDim.x >> 6); ++i) tot += red[i];
      __syncthreads();
      const float nv = vnorm[k], gk = gvec[k];
      const float dgk = tot / nv;  // dW . v / ||v||
      // dv = g/||v|| (dW - (dW . v-hat) v-hat)
      for (int c = t; c < C; c += blockDim.x) {
        const float vh = v[(long)k * C + c] / nv;
        dv[(long)k * C + c] = gk / nv * (dv[(long)k * C + c] - dgk * vh);
      }
      if (t == 0 && dg) dg[k] = dgk;
    }
    if (t == 0) {
      float sb = 0.f;
      for (int j = 0; j < nb; ++j) sb += part_s[((long)j * n + k) * 2];
      if (db) db[k] = sb;
    }
    __syncthreads();
  }
  if (t == 0 && dscale) {
    float s = 0.f;
    for (int j = 0; j < nb; ++j)
      for (int k = 0; k < n; ++k) s += part_s[((long)j * n + k) * 2 + 1];
    dscale[0] = s;
  }
}

// ---- get_corr ----
// tokens [T][C] -> [T][C] / max(||row||, eps)   (one wave per token)
__global__ __launch_bounds__(256) void token_normalize_kernel(const float* __restrict__ x, long T, int C, float eps,
                                                              float* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  for (long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6); r < T; r += (long)gridDim.x * 4) {
    const float* xr = x + r * C;
    float ss = 0.f;
    for (int c = lane; c < C; c += 64) ss = fmaf(xr[c], xr[c], ss);
    const float inv = 1.f / fmaxf(sqrtf(wave_sum_dpp(ss)), eps);
    for (int c = lane; c < C; c += 64) y[r * C + c] = xr[c] * inv;
  }
}

// C[b][i][j] = sum_k A[b][i][k] B[b][j][k]: 128 x 128 tile per 256-thread workgroup, four
// waves of 64 x 64 (2 x 2 v_mfma_f32_32x32x2_f32 blocks), K staged 16 deep through LDS in
// k-major form (A_s[k][i], B_s[k][j]: a lane's fragment element is one conflict-free read).
constexpr int CG_T = 128, CG_BK = 16;
__global__ __launch_bounds__(256) void corr_gemm_kernel(const float* __restrict__ A, const float* __restrict__ Bm,
                                                        int M, int N, int K, float* __restrict__ Cm) {
  __shared__ float As[2][CG_BK][CG_T + 4];
  __shared__ float Bs[2][CG_BK][CG_T + 4];
  const int b = blockIdx.z;
  const int i0 = blockIdx.y * CG_T, j0 = blockIdx.x * CG_T;
  A += (long)b * M * K;
  Bm += (long)b * N * K;
  Cm += (long)b * M * N;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int wi = (wv >> 1) * 64, wj = (wv & 1) * 64;
  // global -> register staging: each thread moves 2 float4 of A and 2 of B per K-tile
  f32x4 ra[2], rb[2];
  auto gload = [&](int kt) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int idx = t + q * 256;          // 512 float4 = 128 rows x 4 float4 (16 k)
      const int row = idx >> 2, kq = (idx & 3) * 4;
      const int k = kt * CG_BK + kq;
      const int ia = min(i0 + row, M - 1), jb = min(j0 + row, N - 1);
      ra[q] = k < K ? *(const f32x4*)(A + (long)ia * K + k) : f32x4{0.f, 0.f, 0.f, 0.f};
      rb[q] = k < K ? *(const f32x4*)(Bm + (long)jb * K + k) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int idx = t + q * 256;
      const int row = idx >> 2, kq = (idx & 3) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        As[buf][kq + e][row] = ra[q][e];
        Bs[buf][kq + e][row] = rb[q][e];
      }
    }
  };
  f32x16 acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[x][y][r] = 0.f;
  const int KT = (K + CG_BK - 1) / CG_BK;
  gload(0);
  sstore(0);
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < KT) gload(kt + 1);
#pragma unroll
    for (int ks = 0; ks < CG_BK; ks += 2) {
      const int kk = ks + (lane >> 5);
      float fa[2], fb[2];
#pragma unroll
      for (int x = 0; x < 2; ++x) fa[x] = As[buf][kk][wi + x * 32 + (lane & 31)];
#pragma unroll
      for (int y = 0; y < 2; ++y) fb[y] = Bs[buf][kk][wj + y * 32 + (lane & 31)];
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[x], fb[y], acc[x][y], 0, 0, 0);
    }
    if (kt + 1 < KT) {
      sstore(buf ^ 1);
      __syncthreads();
    }
  }
  // D layout of 32x32x2: column = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = i0 + wi + x * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int j = j0 + wj + y * 32 + (lane & 31);
        if (i < M && j < N) Cm[(long)i * N + j] = acc[x][y][r];
      }
}

int launch_cos_weight(float* v, const float* g, int n, int C, int mode, float* w_eff, float* vnorm, hipStream_t st) {
  hipLaunchKernelGGL(cos_weight_kernel, dim3(1), dim3(256), 0, st, v, g, n, C, mode, w_eff, vnorm);
  CWT_LAUNCH_CHECK();
  return 0;
}

int launch_cos_cls_fwd(const float* x, long P, int B, int n, const float* w_eff, const float* bias, const float* scale,
                       float* out, hipStream_t st) {
  const long total = (long)B * P;
  const int blocks = (int)std::min<long>(1024, (total + 3) / 4);
  hipLaunchKernelGGL(cos_cls_fwd_kernel, dim3(blocks), dim3(256), 0, st, x, P, B, n, w_eff, bias, scale, out);
  CWT_LAUNCH_CHECK();
  return 0;
}

int cos_cls_bwd_blocks(long total) { return (int)std::min<long>(64, std::max<long>(1, (total + 63) / 64)); }

int launch_cos_cls_bwd(const float* x, long P, int B, int n, const float* w_eff, const float* bias, const float* scale,
                       const float* G, float* part, float* part_s, int mode, const float* v, const float* g,
                       const float* vnorm, float* dv, float* dg, float* db, float* dscale, hipStream_t st) {
  const int nb = cos_cls_bwd_blocks((long)B * P);
  hipLaunchKernelGGL(cos_cls_bwd_kernel, dim3(nb), dim3(256), 0, st, x, P, B, n, w_eff, bias, scale, G, part, part_s);
  CWT_LAUNCH_CHECK();
  hipLaunchKernelGGL(cos_cls_bwd_final_kernel, dim3(1), dim3(256), 0, st, (const float*)part, (const float*)part_s, nb,
                     n, 512, mode, v, g, vnorm, dv, dg, db, dscale);
  CWT_LAUNCH_CHECK();
  return 0;
}

int launch_corr(const float* q, const float* k, int B, int Pq, int Pk, int C, float* qn, float* kn, float* sim,
                hipStream_t st) {
  hipLaunchKernelGGL(token_normalize_kernel, dim3((unsigned)std::min<long>(2048, ((long)B * Pq + 3) / 4)), dim3(256),
                     0, st, q, (long)B * Pq, C, 1e-12f, qn);
  CWT_LAUNCH_CHECK();
  hipLaunchKernelGGL(token_normalize_kernel, dim3((unsigned)std::min<long>(2048, ((long)B * Pk + 3) / 4)), dim3(256),
                     0, st, k, (long)B * Pk, C, 1e-12f, kn);
  CWT_LAUNCH_CHECK();
  dim3 grid(cdiv(Pk, CG_T), cdiv(Pq, CG_T), B);
  hipLaunchKernelGGL(corr_gemm_kernel, grid, dim3(256), 0, st, (const float*)qn, (const float*)kn, Pq, Pk, C, sim);
  CWT_LAUNCH_CHECK();
  return 0;
}

// C[b] = A[b] . Bm[b]^T (A [M][K], Bm [N][K], K % 4 == 0), exact fp32 (MatchNet's v . attn^T)
int launch_gemm_abt(const float* A, const float* Bm, int B, int M, int N, int K, float* Cm, hipStream_t st) {
  dim3 grid(cdiv(N, CG_T), cdiv(M, CG_T), B);
  hipLaunchKernelGGL(corr_gemm_kernel, grid, dim3(256), 0, st, A, Bm, M, N, K, Cm);
  CWT_LAUNCH_CHECK();
  return 0;
}

}  // namespace cwt

// Per-pixel kernels around the CWT:
//  * F.normalize(f, dim=1) over channels, fused with the baseline logits W0 . f
//    (reference test.py:192-194; train.py:247-250)
//  * the per-pixel classifier W' . f_hat (test.py:200-204; train.py:259-261) and its
//    backward w.r.t. W' (train.py:264 loss_q.backward)
//  * bilinear(align_corners) upsample + argmax + histc intersection/union/target + CE loss
//    sum, never materialising the S x S logits (util.py:237-308; test.py:214-224)
//  * the SGD(momentum, nesterov, weight_decay) step of the outer loop (optimizer.py:8-15)
#include "common.h"
#include "kernels.h"

namespace cwt {

// one wave per pixel, lane owns 8 channels (C = 512)
__global__ __launch_bounds__(256) void normalize_kernel(const float* __restrict__ f, long P, int Pb,
                                                        float* __restrict__ out, const float* __restrict__ W0,
                                                        float* __restrict__ logits0) {
  constexpr int C = 512;
  const int lane = threadIdx.x & 63;
  const long p = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (p >= P) return;
  const float* src = f + p * C + lane * 8;
  f32x4 u = *(const f32x4*)src, v = *(const f32x4*)(src + 4);
  float ss = u[0] * u[0] + u[1] * u[1] + u[2] * u[2] + u[3] * u[3] + v[0] * v[0] + v[1] * v[1] + v[2] * v[2] +
             v[3] * v[3];
  ss = wave_sum(ss);
  const float nrm = fmaxf(sqrtf(ss), 1e-12f);
  *(f32x4*)(out + p * C + lane * 8) = u / nrm;
  *(f32x4*)(out + p * C + lane * 8 + 4) = v / nrm;
  if (W0) {
    const int b = (int)(p / Pb);
    const long pp = p - (long)b * Pb;
    const float* w0 = W0 + (long)b * 2 * C + lane * 8;
    float s0 = 0.f, s1 = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      s0 = fmaf(w0[q], u[q], s0);
      s0 = fmaf(w0[4 + q], v[q], s0);
      s1 = fmaf(w0[C + q], u[q], s1);
      s1 = fmaf(w0[C + 4 + q], v[q], s1);
    }
    s0 = wave_sum(s0);
    s1 = wave_sum(s1);
    if (lane == 0) {
      logits0[(long)b * 2 * Pb + pp] = s0;
      logits0[(long)b * 2 * Pb + Pb + pp] = s1;
    }
  }
}

int launch_normalize(const float* f, int B, int Pb, float* out, const float* W0, float* logits0, hipStream_t st) {
  long P = (long)B * Pb;
  hipLaunchKernelGGL(normalize_kernel, dim3(cdiv(P, 4)), dim3(256), 0, st, f, P, Pb, out, W0, logits0);
  CWT_LAUNCH_CHECK();
  return 0;
}

__global__ __launch_bounds__(256) void classify_kernel(const float* __restrict__ W, const float* __restrict__ f,
                                                       long P, int Pb, float* __restrict__ logits) {
  constexpr int C = 512;
  const int lane = threadIdx.x & 63;
  const long p = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (p >= P) return;
  const int b = (int)(p / Pb);
  const long pp = p - (long)b * Pb;
  const float* src = f + p * C + lane * 8;
  f32x4 u = *(const f32x4*)src, v = *(const f32x4*)(src + 4);
  const float* w = W + (long)b * 2 * C + lane * 8;
  float s0 = 0.f, s1 = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    s0 = fmaf(w[q], u[q], s0);
    s0 = fmaf(w[4 + q], v[q], s0);
    s1 = fmaf(w[C + q], u[q], s1);
    s1 = fmaf(w[C + 4 + q], v[q], s1);
  }
  s0 = wave_sum(s0);
  s1 = wave_sum(s1);
  if (lane == 0) {
    logits[(long)b * 2 * Pb + pp] = s0;
    logits[(long)b * 2 * Pb + Pb + pp] = s1;
  }
}

// the classifier over raw features with the normalisation as a per-pixel scale (the fused
// inference tail): logits = (W' . f_p) inv_p = W' . f_hat_p (test.py:200-204)
__global__ __launch_bounds__(256) void classify_scaled_kernel(const float* __restrict__ W, const float* __restrict__ f,
                                                              const float* __restrict__ inv, long P, int Pb,
                                                              float* __restrict__ logits) {
  constexpr int C = 512;
  const int lane = threadIdx.x & 63;
  const long p = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (p >= P) return;
  const int b = (int)(p / Pb);
  const long pp = p - (long)b * Pb;
  const float* src = f + p * C + lane * 4;
  const f32x4 u = *(const f32x4*)src, v = *(const f32x4*)(src + 256);
  const float* w = W + (long)b * 2 * C + lane * 4;
  const f32x4 w0a = *(const f32x4*)w, w0b = *(const f32x4*)(w + 256);
  const f32x4 w1a = *(const f32x4*)(w + C), w1b = *(const f32x4*)(w + C + 256);
  float s0 = 0.f, s1 = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    s0 = fmaf(w0a[q], u[q], s0);
    s0 = fmaf(w0b[q], v[q], s0);
    s1 = fmaf(w1a[q], u[q], s1);
    s1 = fmaf(w1b[q], v[q], s1);
  }
  s0 = wave_sum_dpp(s0);
  s1 = wave_sum_dpp(s1);
  if (lane == 0) {
    const float iv = inv[p];
    logits[(long)b * 2 * Pb + pp] = s0 * iv;
    logits[(long)b * 2 * Pb + Pb + pp] = s1 * iv;
  }
}

int launch_classify_scaled(const float* W, const float* f, const float* inv, int B, int Pb, float* logits,
                           hipStream_t st) {
  long P = (long)B * Pb;
  hipLaunchKernelGGL(classify_scaled_kernel, dim3(cdiv(P, 4)), dim3(256), 0, st, W, f, inv, P, Pb, logits);
  CWT_LAUNCH_CHECK();
  return 0;
}

int launch_classify(const float* W, const float* f, int B, int Pb, float* logits, hipStream_t st) {
  long P = (long)B * Pb;
  hipLaunchKernelGGL(classify_kernel, dim3(cdiv(P, 4)), dim3(256), 0, st, W, f, P, Pb, logits);
  CWT_LAUNCH_CHECK();
  return 0;
}

// dW[b][c][k] += sum_p dl[b][c][p] f[b][p][k]; block = (pixel chunk of 64, b), lanes own channels.
__global__ __launch_bounds__(256) void classify_bwd_kernel(const float* __restrict__ dl, const float* __restrict__ f,
                                                           int Pb, float* __restrict__ dW) {
  constexpr int C = 512;
  __shared__ float red[4][2][C];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int b = blockIdx.y;
  const int p0 = blockIdx.x * 64 + wv * 16;
  float a0[8], a1[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) a0[q] = a1[q] = 0.f;
  for (int j = 0; j < 16; ++j) {
    const int p = p0 + j;
    if (p >= Pb) break;
    const float g0 = dl[(long)b * 2 * Pb + p], g1 = dl[(long)b * 2 * Pb + Pb + p];
    const float* src = f + ((long)b * Pb + p) * C + lane * 8;
    f32x4 u = *(const f32x4*)src, v = *(const f32x4*)(src + 4);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      a0[q] = fmaf(g0, u[q], a0[q]);
      a0[4 + q] = fmaf(g0, v[q], a0[4 + q]);
      a1[q] = fmaf(g1, u[q], a1[q]);
      a1[4 + q] = fmaf(g1, v[q], a1[4 + q]);
    }
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    red[wv][0][lane * 8 + q] = a0[q];
    red[wv][1][lane * 8 + q] = a1[q];
  }
  __syncthreads();
  for (int i = t; i < 2 * C; i += 256) {
    const int c = i / C, k = i % C;
    const float s = (red[0][c][k] + red[1][c][k]) + (red[2][c][k] + red[3][c][k]);
    atomicAdd(&dW[((long)b * 2 + c) * C + k], s);
  }
}

int launch_classify_bwd(const float* dl, const float* f, int B, int Pb, float* dW, hipStream_t st) {
  dim3 grid(cdiv(Pb, 64), B);
  hipLaunchKernelGGL(classify_bwd_kernel, grid, dim3(256), 0, st, dl, f, Pb, dW);
  CWT_LAUNCH_CHECK();
  return 0;
}

// counts[z][b][0..5] = {inter0, inter1, out0, out1, tgt0, tgt1} (uint32), ce[b] = {sum nll, count}
// blockIdx.z = 1 (when logits2 is given) scores a second logits tensor against the same target
// in the same launch (the episode's pred_q0 beside pred_q, test.py:192-204), without CE.
__global__ __launch_bounds__(256) void seg_metrics_kernel(const float* __restrict__ logits,
                                                          const float* __restrict__ logits2,
                                                          const int64_t* __restrict__ target, int h, int w, int S,
                                                          float sy, float sx, unsigned* __restrict__ counts,
                                                          double* __restrict__ ce) {
  __shared__ unsigned cnt[4][6];
  __shared__ double cel[4][2];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int b = blockIdx.y, z = blockIdx.z;
  const long npix = (long)S * S;
  const long plane = (long)h * w;
  const float* L0 = (z ? logits2 : logits) + (long)b * 2 * plane;
  if (z) ce = nullptr;
  const float* L1 = L0 + plane;
  unsigned c[6] = {0, 0, 0, 0, 0, 0};
  double nll = 0.0;
  unsigned nvalid = 0;
  for (long i = (long)blockIdx.x * 256 + t; i < npix; i += (long)gridDim.x * 256) {
    const int Y = (int)(i / S), X = (int)(i - (long)Y * S);
    Lerp ly = lerp_coord(Y, h, sy), lx = lerp_coord(X, w, sx);
    const float l0 = ly.l0 * (lx.l0 * L0[ly.i0 * w + lx.i0] + lx.l1 * L0[ly.i0 * w + lx.i1]) +
                     ly.l1 * (lx.l0 * L0[ly.i1 * w + lx.i0] + lx.l1 * L0[ly.i1 * w + lx.i1]);
    const float l1 = ly.l0 * (lx.l0 * L1[ly.i0 * w + lx.i0] + lx.l1 * L1[ly.i0 * w + lx.i1]) +
                     ly.l1 * (lx.l0 * L1[ly.i1 * w + lx.i0] + lx.l1 * L1[ly.i1 * w + lx.i1]);
    const int64_t tg = target[(long)b * npix + i];
    const int pred = (l1 > l0) ? 1 : 0;  // torch.argmax: first index on ties
    if (tg == 255) continue;
    c[2 + pred]++;
    if (tg == 0 || tg == 1) {
      c[4 + (int)tg]++;
      if (pred == tg) c[pred]++;
      const float m = fmaxf(l0, l1);
      const float lse = m + logf(expf(l0 - m) + expf(l1 - m));
      nll += (double)(lse - (tg == 1 ? l1 : l0));
      nvalid++;
    }
  }
#pragma unroll
  for (int k = 0; k < 6; ++k)
    for (int o = 32; o > 0; o >>= 1) c[k] += __shfl_xor(c[k], o, 64);
  for (int o = 32; o > 0; o >>= 1) {
    nll += __shfl_xor(nll, o, 64);
    nvalid += __shfl_xor(nvalid, o, 64);
  }
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < 6; ++k) cnt[wv][k] = c[k];
    cel[wv][0] = nll;
    cel[wv][1] = (double)nvalid;
  }
  __syncthreads();
  // per-block partials (no atomics, nothing to zero first); seg_metrics_final sums them in
  // block order, so the double CE sum is deterministic
  const long pb = ((long)z * gridDim.y + b) * gridDim.x + blockIdx.x;
  if (t < 6) counts[pb * 6 + t] = cnt[0][t] + cnt[1][t] + cnt[2][t] + cnt[3][t];
  if (ce && t < 2) ce[pb * 2 + t] = (cel[0][t] + cel[1][t]) + (cel[2][t] + cel[3][t]);
}

// one 256-thread block per batch item: thread k takes block k's partials, then a fixed-shape
// LDS tree (deterministic) gives [inter, union, target] x 2 classes and (nll sum, valid count)
__global__ __launch_bounds__(256) void seg_metrics_final_kernel(const unsigned* __restrict__ counts,
                                                                const double* __restrict__ ce_part, int nblk,
                                                                float* __restrict__ iut, float* __restrict__ iut2,
                                                                double* __restrict__ ce) {
  __shared__ unsigned c[6][256];
  __shared__ double d[2][256];
  const int b = blockIdx.x, t = threadIdx.x, z = blockIdx.y;
  const bool have = t < nblk;
  if (z) {  // the second logits tensor: its own counts plane, no CE
    counts += (long)gridDim.x * nblk * 6;
    iut = iut2;
    ce = nullptr;
  }
#pragma unroll
  for (int q = 0; q < 6; ++q) c[q][t] = have ? counts[((long)b * nblk + t) * 6 + q] : 0u;
  if (ce) {
    d[0][t] = have ? ce_part[((long)b * nblk + t) * 2] : 0.0;
    d[1][t] = have ? ce_part[((long)b * nblk + t) * 2 + 1] : 0.0;
  }
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) {
#pragma unroll
      for (int q = 0; q < 6; ++q) c[q][t] += c[q][t + o];
      if (ce) {
        d[0][t] += d[0][t + o];
        d[1][t] += d[1][t + o];
      }
    }
    __syncthreads();
  }
  if (t < 2) {
    iut[b * 6 + t] = (float)c[t][0];                                 // intersection
    iut[b * 6 + 2 + t] = (float)(c[2 + t][0] + c[4 + t][0] - c[t][0]);  // union = output + target - intersection
    iut[b * 6 + 4 + t] = (float)c[4 + t][0];                         // target
    if (ce) ce[b * 2 + t] = d[t][0];
  }
}

// counts_ws: [nz][B][nblk][6] unsigned, then (8-B aligned) [B][nblk][2] double partials
// (nz = 2 when logits2 / iut2 are given: both tensors scored in the same two launches)
int launch_seg_metrics(const float* logits, const int64_t* target, int B, int h, int w, int S, float* iut,
                       double* ce, unsigned* counts_ws, hipStream_t st, const float* logits2, float* iut2) {
  const long npix = (long)S * S;
  const int nblk = (int)std::min<long>(256, cdiv(npix, 256));
  const int nz = logits2 ? 2 : 1;
  if (logits2 && !iut2) return fail(CWT_EARG, "seg_metrics: a second logits tensor needs its iut output");
  double* ce_part = ce ? (double*)(counts_ws + (((long)nz * B * nblk * 6 + 1) & ~1L)) : nullptr;
  dim3 grid(nblk, B, nz);
  hipLaunchKernelGGL(seg_metrics_kernel, grid, dim3(256), 0, st, logits, logits2, target, h, w, S,
                     align_corners_scale(h, S), align_corners_scale(w, S), counts_ws, ce_part);
  CWT_LAUNCH_CHECK();
  hipLaunchKernelGGL(seg_metrics_final_kernel, dim3(B, nz), dim3(256), 0, st, (const unsigned*)counts_ws,
                     (const double*)ce_part, nblk, iut, iut2, ce);
  CWT_LAUNCH_CHECK();
  return 0;
}

__global__ void sgd_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ buf, long n,
                           float lr, float mom, float wd, int nesterov, int first) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float pv = p[i];
    float d = g[i];
    if (wd != 0.f) d = d + wd * pv;
    if (mom != 0.f) {
      const float b = first ? d : mom * buf[i] + d;
      buf[i] = b;
      d = nesterov ? d + mom * b : b;
    }
    p[i] = pv - lr * d;
  }
}

int launch_sgd(float* p, const float* g, float* buf, long n, float lr, float mom, float wd, int nesterov, int first,
               hipStream_t st) {
  int blocks = (int)std::min<long>(2048, cdiv(n, 256));
  hipLaunchKernelGGL(sgd_kernel, dim3(blocks), dim3(256), 0, st, p, g, buf, n, lr, mom, wd, nesterov, first);
  CWT_LAUNCH_CHECK();
  return 0;
}

// intersectionAndUnionGPU on argmax maps: counts[0..K) inter, [K..2K) output, [2K..3K) target
__global__ void iou_preds_kernel(const int64_t* __restrict__ preds, const int64_t* __restrict__ target, long n, int K,
                                 int ignore, unsigned* __restrict__ counts) {
  __shared__ unsigned c[48];
  if (threadIdx.x < 48) c[threadIdx.x] = 0;
  __syncthreads();
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int64_t t = target[i];
    if (t == ignore) continue;
    const int64_t p = preds[i];
    if (p >= 0 && p < K) {
      atomicAdd(&c[K + (int)p], 1u);
      if (p == t) atomicAdd(&c[(int)p], 1u);
    }
    if (t >= 0 && t < K) atomicAdd(&c[2 * K + (int)t], 1u);
  }
  __syncthreads();
  if (threadIdx.x < 3 * K && c[threadIdx.x]) atomicAdd(&counts[threadIdx.x], c[threadIdx.x]);
}

__global__ void iou_preds_final_kernel(const unsigned* counts, int K, float* iut) {
  const int k = threadIdx.x;
  if (k >= K) return;
  iut[k] = (float)counts[k];
  iut[K + k] = (float)(counts[K + k] + counts[2 * K + k] - counts[k]);
  iut[2 * K + k] = (float)counts[2 * K + k];
}

int launch_iou_preds(const int64_t* preds, const int64_t* target, long n, int K, int ignore, float* iut,
                     unsigned* counts_ws, hipStream_t st) {
  CWT_HIP(hipMemsetAsync(counts_ws, 0, sizeof(unsigned) * 3 * K, st));
  int blocks = (int)std::min<long>(512, cdiv(n, 256));
  hipLaunchKernelGGL(iou_preds_kernel, dim3(std::max(blocks, 1)), dim3(256), 0, st, preds, target, n, K, ignore,
                     counts_ws);
  CWT_LAUNCH_CHECK();
  hipLaunchKernelGGL(iou_preds_final_kernel, dim3(1), dim3(64), 0, st, (const unsigned*)counts_ws, K, iut);
  CWT_LAUNCH_CHECK();
  return 0;
}

}  // namespace cwt

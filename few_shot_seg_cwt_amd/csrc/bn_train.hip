// Training-mode BatchNorm of the extractor (nn.BatchNorm2d with training=True, momentum 0.1)
// and the bottleneck's Dropout2d.  The reference's do_epoch calls model.train() at the start
// of every epoch and model.eval() only before the first query extraction (train.py:184,245),
// so the FIRST support extraction of each epoch runs every BN of the PSPNet on batch
// statistics, moves the running statistics by momentum 0.1 (unbiased variance), and drops
// whole bottleneck channels with Dropout2d(p=args.dropout) (pspnet.py:124-129).  Every later
// extraction of the epoch is eval mode over the updated running statistics.
//
// The conv kernels run with scale = 1, shift = 0, no residual, no ReLU (raw conv output in
// the activation layout); per conv then:
//   bn_stats_kernel    per (256-row block, channel) Welford partials (n, mean, M2)
//   bn_finalize_kernel one thread per channel: Chan merge of the partials in double, batch
//                      scale/shift, running-statistic update, eval fold rewritten
//   bn_apply_kernel    y = [relu](y * sc + sh [+ res]) [* Dropout2d mask], in place, 8 channels
//                      per thread (two 16 B lines of the S-layout, one of bf16 / fp32)
// HBM-bound byte work (two reads + one write of the activation); it runs once per epoch.
#include "common.h"
#include "kernels.h"

namespace cwt {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kBnRows = 256;  // rows per stats block (64 per row group of 4)

__device__ __forceinline__ float act_load1(const void* y, int layout, int ld, int C, long row, int c) {
  if (layout == ACT_F32) return ((const float*)y)[row * ld + c];
  if (layout == ACT_BF16) return (float)((const __bf16*)y)[row * C + c];
  const __bf16* p = (const __bf16*)y + (row * (C >> 5) + (c >> 5)) * 64 + (c & 31);
  return (float)p[0] + (float)p[32];
}

__device__ __forceinline__ void act_load8(const void* y, int layout, int ld, int C, long row, int c0, float* v) {
  if (layout == ACT_F32) {
    const float* p = (const float*)y + row * ld + c0;
    const f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[q] = a[q];
      v[q + 4] = b[q];
    }
  } else if (layout == ACT_BF16) {
    const bf16x8 h = *(const bf16x8*)((const __bf16*)y + row * C + c0);
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = (float)h[q];
  } else {
    const __bf16* p = (const __bf16*)y + (row * (C >> 5) + (c0 >> 5)) * 64 + (c0 & 31);
    const bf16x8 h = *(const bf16x8*)p, l = *(const bf16x8*)(p + 32);
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = (float)h[q] + (float)l[q];
  }
}

__device__ __forceinline__ void act_store8(void* y, int layout, int ld, int C, long row, int c0, const float* v) {
  if (layout == ACT_F32) {
    float* p = (float*)y + row * ld + c0;
    *(f32x4*)p = f32x4{v[0], v[1], v[2], v[3]};
    *(f32x4*)(p + 4) = f32x4{v[4], v[5], v[6], v[7]};
  } else if (layout == ACT_BF16) {
    bf16x8 h;
#pragma unroll
    for (int q = 0; q < 8; ++q) h[q] = (__bf16)v[q];
    *(bf16x8*)((__bf16*)y + row * C + c0) = h;
  } else {
    bf16x8 h, l;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      h[q] = (__bf16)v[q];
      l[q] = (__bf16)(v[q] - (float)h[q]);
    }
    __bf16* p = (__bf16*)y + (row * (C >> 5) + (c0 >> 5)) * 64 + (c0 & 31);
    *(bf16x8*)p = h;
    *(bf16x8*)(p + 32) = l;
  }
}

// grid (cdiv(M, 256), cdiv(C, 64)); partial planes part[k][blk][C], k = n, mean, M2
__global__ __launch_bounds__(256) void bn_stats_kernel(const void* __restrict__ y, int layout, int ld, long M, int C,
                                                       float* __restrict__ part) {
  __shared__ float sn[4][64], sm[4][64], sq[4][64];
  const int lane = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + lane;
  const long r0 = (long)blockIdx.x * kBnRows;
  float n = 0.f, mean = 0.f, m2 = 0.f;
  if (c < C) {
    for (int i = rg; i < kBnRows; i += 4) {
      const long r = r0 + i;
      if (r >= M) break;
      const float v = act_load1(y, layout, ld, C, r, c);
      n += 1.f;
      const float d = v - mean;
      mean += d / n;
      m2 += d * (v - mean);
    }
  }
  sn[rg][lane] = n;
  sm[rg][lane] = mean;
  sq[rg][lane] = m2;
  __syncthreads();
  if (rg == 0 && c < C) {
    for (int g = 1; g < 4; ++g) {  // Chan merge of the 4 row groups
      const float nb = sn[g][lane];
      if (nb == 0.f) continue;
      const float nt = n + nb, d = sm[g][lane] - mean;
      mean += d * (nb / nt);
      m2 += sq[g][lane] + d * d * (n * nb / nt);
      n = nt;
    }
    const long plane = (long)gridDim.x * C;
    const long o = (long)blockIdx.x * C + c;
    part[o] = n;
    part[plane + o] = mean;
    part[2 * plane + o] = m2;
  }
}

// one thread per channel: batch scale/shift into bsc[0..C) / bsc[C..2C), running stats and the
// eval fold updated in place (torch: running_var uses the unbiased M2 / (n - 1))
__global__ void bn_finalize_kernel(const float* __restrict__ part, int nblk, int C, float* __restrict__ bn,
                                   float* __restrict__ scale, float* __restrict__ shift, float eps, float momentum,
                                   float* __restrict__ bsc) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const long plane = (long)nblk * C;
  double n = 0.0, mean = 0.0, m2 = 0.0;
  for (int b = 0; b < nblk; ++b) {
    const double nb = part[(long)b * C + c];
    if (nb == 0.0) continue;
    const double mb = part[plane + (long)b * C + c], qb = part[2 * plane + (long)b * C + c];
    const double nt = n + nb, d = mb - mean;
    mean += d * (nb / nt);
    m2 += qb + d * d * (n * nb / nt);
    n = nt;
  }
  const float gamma = bn[c], beta = bn[C + c];
  const float var_b = (float)(m2 / n);
  const float mu = (float)mean;
  const float sc = gamma / sqrtf(var_b + eps);
  bsc[c] = sc;
  bsc[C + c] = beta - mu * sc;
  const float rm = (1.f - momentum) * bn[2 * C + c] + momentum * mu;
  const float rv = (1.f - momentum) * bn[3 * C + c] + momentum * (float)(m2 / (n - 1.0));
  bn[2 * C + c] = rm;
  bn[3 * C + c] = rv;
  const float esc = gamma * (1.0f / sqrtf(rv + eps));  // as load_conv's host fold
  scale[c] = esc;
  shift[c] = beta - rm * esc;
}

__global__ __launch_bounds__(256) void bn_apply_kernel(BnTrainArgs a, const float* __restrict__ bsc) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int cg = a.C >> 3;
  if (idx >= a.M * cg) return;
  const long row = idx / cg;
  const int c0 = (int)(idx - row * cg) * 8;
  float v[8], r[8];
  act_load8(a.y, a.layout, a.ld, a.C, row, c0, v);
  if (a.res) act_load8(a.res, a.layout, a.res_ld, a.C, row, c0, r);
  const long img = row / a.rows_per_image;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int c = c0 + q;
    float t = fmaf(v[q], bsc[c], bsc[a.C + c]);
    if (a.res) t += r[q];
    if (a.relu) t = fmaxf(t, 0.f);
    if (a.drop_p > 0.f) t *= dropout_scale(a.drop_p, a.seed, 3, (unsigned long long)img * a.C + c);
    v[q] = t;
  }
  act_store8(a.y, a.layout, a.ld, a.C, row, c0, v);
}

size_t bn_train_part_floats(long M, int C) { return (size_t)3 * cdiv(M, (long)kBnRows) * C; }

int launch_bn_train(const BnTrainArgs& a, float* part, size_t part_floats, float* batch_sc, hipStream_t st) {
  if (a.M < 2) return fail(CWT_EARG, "Expected more than 1 value per channel when training (BatchNorm2d)");
  if (a.C % 64 != 0 || (a.layout == ACT_F32 && (a.ld % 4 != 0 || a.res_ld % 4 != 0)))
    return fail(CWT_EARG, "bn_train: C % 64 == 0 and 16 B aligned rows required");
  if (bn_train_part_floats(a.M, a.C) > part_floats) return fail(CWT_ESTATE, "bn_train: partial workspace too small");
  const int nblk = (int)cdiv(a.M, (long)kBnRows);
  hipLaunchKernelGGL(bn_stats_kernel, dim3(nblk, a.C / 64), dim3(256), 0, st, (const void*)a.y, a.layout, a.ld, a.M,
                     a.C, part);
  CWT_LAUNCH_CHECK();
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(cdiv(a.C, 256)), dim3(256), 0, st, (const float*)part, nblk, a.C, a.bn,
                     a.scale, a.shift, a.eps, a.momentum, batch_sc);
  CWT_LAUNCH_CHECK();
  const long total = a.M * (a.C / 8);
  hipLaunchKernelGGL(bn_apply_kernel, dim3(cdiv(total, 256L)), dim3(256), 0, st, a, (const float*)batch_sc);
  CWT_LAUNCH_CHECK();
  return 0;
}

__global__ void scale_cols_kernel(const float* __restrict__ src, float* __restrict__ dst, long n, int period,
                                  const float* __restrict__ sc) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i] * sc[i % period];
}

int launch_scale_cols(const float* src, float* dst, long n, int period, const float* sc, hipStream_t st) {
  hipLaunchKernelGGL(scale_cols_kernel, dim3(cdiv(n, 256L)), dim3(256), 0, st, src, dst, n, period, sc);
  CWT_LAUNCH_CHECK();
  return 0;
}

}  // namespace cwt

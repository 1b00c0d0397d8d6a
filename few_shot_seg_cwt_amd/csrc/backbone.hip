// Byte-moving pieces of the frozen extractor around the MFMA convs:
//  * stem conv1 (3->64, 3x3 s2 p1, K = 27: too thin for the implicit GEMM) + BN + ReLU,
//    reading the caller's NCHW image and writing NHWC            (resnet.py:111-112,147)
//  * maxpool 3x3 s2 p1 (-inf padding)                           (resnet.py:118)
//  * PPM adaptive average pooling for all bins in one sweep     (pspnet.py:26)
//  * the PPM branch of the bottleneck conv, folded: small-M GEMMs over the pooled cells and
//    a separable interpolation of their per-tap products   (pspnet.py:19-38,124-128); the
//    concat buffer of the reference (torch.cat) is never materialised
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "common.h"
#include "kernels.h"

namespace cwt {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// One thread per output pixel, all 64 output channels; weights [ci][ky][kx][co] in LDS.
// SPLIT: write the S-layout [pix][2][hi 32 | lo 32] bf16 (conv_x3s.hip) instead of fp32 NHWC.
template <bool SPLIT>
__global__ __launch_bounds__(256) void stem_conv1_kernel(const float* __restrict__ img, int N, int S,
                                                         const float* __restrict__ w,
                                                         const float* __restrict__ scale,
                                                         const float* __restrict__ shift,
                                                         float* __restrict__ out, int Ho, float floor_) {
  __shared__ float ws[27 * 64];
  __shared__ float ss[64], bs[64];
  for (int i = threadIdx.x; i < 27 * 64; i += blockDim.x) ws[i] = w[i];
  if (threadIdx.x < 64) {
    ss[threadIdx.x] = scale[threadIdx.x];
    bs[threadIdx.x] = shift[threadIdx.x];
  }
  __syncthreads();
  long pix = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)N * Ho * Ho;
  if (pix >= total) return;
  int n = (int)(pix / ((long)Ho * Ho));
  int rem = (int)(pix - (long)n * Ho * Ho);
  int oh = rem / Ho, ow = rem - (rem / Ho) * Ho;
  float in[27];
#pragma unroll
  for (int ci = 0; ci < 3; ++ci)
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        int ih = oh * 2 - 1 + ky, iw = ow * 2 - 1 + kx;
        float v = 0.f;
        if ((unsigned)ih < (unsigned)S && (unsigned)iw < (unsigned)S)
          v = img[(((long)n * 3 + ci) * S + ih) * S + iw];
        in[ci * 9 + ky * 3 + kx] = v;
      }
  float* o = out + pix * 64;
#pragma unroll
  for (int c8 = 0; c8 < 8; ++c8) {
    float r[8];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c4 = c8 * 2 + h;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < 27; ++k) {
        f32x4 wv = *(const f32x4*)&ws[k * 64 + c4 * 4];
        acc += in[k] * wv;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) r[h * 4 + q] = fmaxf(fmaf(acc[q], ss[c4 * 4 + q], bs[c4 * 4 + q]), floor_);
    }
    if (SPLIT) {
      bf16x8 hi, lo;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        hi[q] = (__bf16)r[q];
        lo[q] = (__bf16)(r[q] - (float)hi[q]);
      }
      __bf16* sp = (__bf16*)out + pix * 128 + (c8 >> 2) * 64 + (c8 & 3) * 8;
      *(bf16x8*)sp = hi;
      *(bf16x8*)(sp + 32) = lo;
    } else {
      *(f32x4*)(o + c8 * 8) = f32x4{r[0], r[1], r[2], r[3]};
      *(f32x4*)(o + c8 * 8 + 4) = f32x4{r[4], r[5], r[6], r[7]};
    }
  }
}

// S-layout output: one thread per (pixel, 8 output channels); a wave covers 8 pixels and
// writes them as 2 KB of contiguous lines (hi and lo chunks of each 32-channel block).
// BF16: the same with plain bf16 NHWC output (1 KB of contiguous lines per wave).
template <bool BF16>
__global__ __launch_bounds__(256) void stem_conv1_s_kernel(const float* __restrict__ img, int N, int S,
                                                           const float* __restrict__ w,
                                                           const float* __restrict__ scale,
                                                           const float* __restrict__ shift,
                                                           __bf16* __restrict__ out, int Ho, float floor_) {
  __shared__ float ws[27 * 64];
  for (int i = threadIdx.x; i < 27 * 64; i += blockDim.x) ws[i] = w[i];
  __syncthreads();
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)N * Ho * Ho * 8;
  if (idx >= total) return;
  const int g = (int)(idx & 7);
  const long pix = idx >> 3;
  const int n = (int)(pix / ((long)Ho * Ho));
  const int rem = (int)(pix - (long)n * Ho * Ho);
  const int oh = rem / Ho, ow = rem - (rem / Ho) * Ho;
  f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int ci = 0; ci < 3; ++ci)
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int ih = oh * 2 - 1 + ky, iw = ow * 2 - 1 + kx;
        float v = 0.f;
        if ((unsigned)ih < (unsigned)S && (unsigned)iw < (unsigned)S) v = img[(((long)n * 3 + ci) * S + ih) * S + iw];
        const int k = ci * 9 + ky * 3 + kx;
        a0 += v * *(const f32x4*)&ws[k * 64 + g * 8];
        a1 += v * *(const f32x4*)&ws[k * 64 + g * 8 + 4];
      }
  bf16x8 hi, lo;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int c = g * 8 + q;
    const float r = fmaxf(fmaf(q < 4 ? a0[q & 3] : a1[q & 3], scale[c], shift[c]), floor_);
    hi[q] = (__bf16)r;
    lo[q] = (__bf16)(r - (float)hi[q]);
  }
  if (BF16) {
    *(bf16x8*)(out + pix * 64 + g * 8) = hi;
  } else {
    __bf16* sp = out + pix * 128 + (g >> 2) * 64 + (g & 3) * 8;
    *(bf16x8*)sp = hi;
    *(bf16x8*)(sp + 32) = lo;
  }
}

// The stem conv on the exact f32 matrix cores (round 3).  K = 27 taps (padded to 28) x 64
// output channels x 16 pixels per wave step: D[16 ch][16 pix] = W[16 ch][4 k] . I[4 k][16 pix]
// by v_mfma_f32_16x16x4_f32 (an fmaf chain per output, so plain fp32 arithmetic), 7 k-steps x
// 4 channel blocks = 28 MFMAs per 16 pixels.  The 16 rows of channel block nb hold channels
// chan(nb, r) = 32 (nb >> 1) + 8 (r >> 2) + 4 (nb & 1) + (r & 3), so D lane l (pixel l & 15,
// rows 4 (l >> 4) .. +3) ends up with channels 8j .. 8j + 7 and 32 + 8j .. 32 + 8j + 7 (j = l >> 4):
// two 16-B hi and two 16-B lo stores of the S-layout (or two of plain bf16) per lane, no
// shuffle.  A lane's weights (28), BN scale / shift (16 + 16) stay in registers while the wave
// walks its 16-pixel groups; the image reads are 4-B gathers from L2 (2.7 MB image per episode).
// The VALU form above gave every (pixel, 8 channels) thread 216 FMAs behind 54 LDS weight reads
// and ran at 26-33 us for 2 x 237^2 pixels, 6x its byte floor.  OUT: 0 the S-layout, 1 plain
// bf16 NHWC, 2 fp32 NHWC (the fp32-width stacks, round 5: the lane's 16 channels as four 16-B
// stores; the one-pixel-per-thread VALU kernel's 64-channel rows took 32 us alone, its stores
// scattered 16 B per 256-B row across the wave)
template <int OUT>
__global__ __launch_bounds__(256) void stem_conv1_mfma_kernel(const float* __restrict__ img, int N, int S,
                                                              const float* __restrict__ w,
                                                              const float* __restrict__ scale,
                                                              const float* __restrict__ shift,
                                                              void* __restrict__ out_, int Ho, float floor_,
                                                              int ngroups) {
  constexpr bool BF16 = OUT == 1;
  __bf16* out = (__bf16*)out_;
  const int lane = threadIdx.x & 63, j = lane >> 4, c16 = lane & 15;
  const int wave = (int)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
  const int nwaves = (int)(gridDim.x * (blockDim.x >> 6));
  // A operand: lane supplies W[row c16][k = 4s + j] of every channel block
  float a[4][7];
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) {
    const int ch = 32 * (nb >> 1) + 8 * (c16 >> 2) + 4 * (nb & 1) + (c16 & 3);
#pragma unroll
    for (int s = 0; s < 7; ++s) {
      const int k = 4 * s + j;
      a[nb][s] = k < 27 ? w[k * 64 + ch] : 0.f;
    }
  }
  // this lane's output channels: nb -> chan(nb, 4j + i)
  float sc[4][4], sh[4][4];
#pragma unroll
  for (int nb = 0; nb < 4; ++nb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ch = 32 * (nb >> 1) + 8 * j + 4 * (nb & 1) + i;
      sc[nb][i] = scale[ch];
      sh[nb][i] = shift[ch];
    }
  const long hw = (long)Ho * Ho, total = (long)N * hw;
  // the gathers of group grp + nwaves are issued before group grp's MFMAs (one group ahead)
  auto gather = [&](int grp, float (&b)[7]) {
    const long pix = (long)grp * 16 + c16;
    const long pc = pix < total ? pix : total - 1;  // tail lanes compute a valid pixel, never stored
    const int n = (int)(pc / hw);
    const int rem = (int)(pc - (long)n * hw);
    const int oh = rem / Ho, ow = rem - oh * Ho;
    const float* ib = img + (long)n * 3 * S * S;
#pragma unroll
    for (int s = 0; s < 7; ++s) {
      const int k = 4 * s + j;
      const int ci = k / 9, t = k - 9 * ci, ky = t / 3, kx = t - 3 * ky;
      const int ih = 2 * oh - 1 + ky, iw = 2 * ow - 1 + kx;
      const bool ok = k < 27 && (unsigned)ih < (unsigned)S && (unsigned)iw < (unsigned)S;
      b[s] = ok ? ib[((long)ci * S + ih) * S + iw] : 0.f;
    }
  };
  float bn[7];
  if (wave < ngroups) gather(wave, bn);
  for (int grp = wave; grp < ngroups; grp += nwaves) {
    const long pix = (long)grp * 16 + c16;
    float b[7];
#pragma unroll
    for (int s = 0; s < 7; ++s) b[s] = bn[s];
    if (grp + nwaves < ngroups) gather(grp + nwaves, bn);
    f32x4 acc[4];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      acc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 7; ++s) acc[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[nb][s], b[s], acc[nb], 0, 0, 0);
    }
    if (pix >= total) continue;
    // channel block pair h = 0: channels 8j..8j+7 (nb 0, 1); h = 1: 32 + 8j .. (nb 2, 3)
    if constexpr (OUT == 2) {
      float* of = (float*)out_ + pix * 64;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        f32x4 r0, r1;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          r0[i] = fmaxf(fmaf(acc[2 * h][i], sc[2 * h][i], sh[2 * h][i]), floor_);
          r1[i] = fmaxf(fmaf(acc[2 * h + 1][i], sc[2 * h + 1][i], sh[2 * h + 1][i]), floor_);
        }
        *(f32x4*)(of + 32 * h + 8 * j) = r0;
        *(f32x4*)(of + 32 * h + 8 * j + 4) = r1;
      }
      continue;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      bf16x8 hi, lo;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int nb = 2 * h + (q >> 2), i = q & 3;
        const float r = fmaxf(fmaf(acc[nb][i], sc[nb][i], sh[nb][i]), floor_);
        hi[q] = (__bf16)r;
        lo[q] = (__bf16)(r - (float)hi[q]);
      }
      if (BF16) {
        *(bf16x8*)(out + pix * 64 + 32 * h + 8 * j) = hi;
      } else {
        __bf16* sp = out + pix * 128 + 64 * h + 8 * j;
        *(bf16x8*)sp = hi;
        *(bf16x8*)(sp + 32) = lo;
      }
    }
  }
}

int launch_stem_conv1(const float* img, int N, int S, const float* w27x64, const float* scale,
                      const float* shift, float* out, int Ho, hipStream_t st, int layout, int relu) {
  long total = (long)N * Ho * Ho;
  const float floor_ = relu ? 0.f : -INFINITY;  // relu = 0: raw conv (training-mode BN follows)
  static const bool valu = getenv("CWT_STEM_VALU") && atoi(getenv("CWT_STEM_VALU"));  // A/B switch
  const int ngroups = (int)cdiv(total, 16);
  // ~gpw groups of 16 pixels per wave (4 waves per block); CWT_STEM_GPW for A/B
  static const int gpw = getenv("CWT_STEM_GPW") ? std::max(1, atoi(getenv("CWT_STEM_GPW"))) : 4;
  const int grid = (int)std::min<long>(cdiv(ngroups, 4 * gpw), 8192);
  if (layout == ACT_SPLIT && !valu)
    hipLaunchKernelGGL(stem_conv1_mfma_kernel<0>, dim3(grid), dim3(256), 0, st, img, N, S, w27x64, scale, shift,
                       (void*)out, Ho, floor_, ngroups);
  else if (layout == ACT_BF16 && !valu)
    hipLaunchKernelGGL(stem_conv1_mfma_kernel<1>, dim3(grid), dim3(256), 0, st, img, N, S, w27x64, scale, shift,
                       (void*)out, Ho, floor_, ngroups);
  else if (!valu && layout != ACT_SPLIT && layout != ACT_BF16)  // fp32 NHWC: the exact f32 MFMA form
    hipLaunchKernelGGL(stem_conv1_mfma_kernel<2>, dim3(grid), dim3(256), 0, st, img, N, S, w27x64, scale, shift,
                       (void*)out, Ho, floor_, ngroups);
  else if (layout == ACT_SPLIT)
    hipLaunchKernelGGL(stem_conv1_s_kernel<false>, dim3(cdiv(total * 8, 256)), dim3(256), 0, st, img, N, S, w27x64,
                       scale, shift, (__bf16*)out, Ho, floor_);
  else if (layout == ACT_BF16)
    hipLaunchKernelGGL(stem_conv1_s_kernel<true>, dim3(cdiv(total * 8, 256)), dim3(256), 0, st, img, N, S, w27x64,
                       scale, shift, (__bf16*)out, Ho, floor_);
  else
    hipLaunchKernelGGL(stem_conv1_kernel<false>, dim3(cdiv(total, 256)), dim3(256), 0, st, img, N, S, w27x64, scale,
                       shift, out, Ho, floor_);
  CWT_LAUNCH_CHECK();
  return 0;
}

__global__ void maxpool3s2_kernel(const float* __restrict__ in, int N, int H, int W, int C,
                                  float* __restrict__ out, int Ho, int Wo) {
  const int c4n = C >> 2;
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)N * Ho * Wo * c4n;
  if (idx >= total) return;
  int c4 = (int)(idx % c4n);
  long pix = idx / c4n;
  int ow = (int)(pix % Wo);
  int oh = (int)((pix / Wo) % Ho);
  int n = (int)(pix / ((long)Wo * Ho));
  f32x4 m = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
    int ih = oh * 2 - 1 + ky;
    if ((unsigned)ih >= (unsigned)H) continue;
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      int iw = ow * 2 - 1 + kx;
      if ((unsigned)iw >= (unsigned)W) continue;
      f32x4 v = *(const f32x4*)(in + (((long)n * H + ih) * W + iw) * C + c4 * 4);
#pragma unroll
      for (int q = 0; q < 4; ++q) m[q] = fmaxf(m[q], v[q]);
    }
  }
  *(f32x4*)(out + pix * C + c4 * 4) = m;
}

int launch_maxpool3s2(const float* in, int N, int H, int W, int C, float* out, int Ho, int Wo,
                      hipStream_t st) {
  long total = (long)N * Ho * Wo * (C / 4);
  hipLaunchKernelGGL(maxpool3s2_kernel, dim3(cdiv(total, 256)), dim3(256), 0, st, in, N, H, W, C, out, Ho, Wo);
  CWT_LAUNCH_CHECK();
  return 0;
}

// maxpool 3x3 s2 p1 on the S-layout: one thread per (pixel, 8 channels); max of hi + lo
// (exact in fp32), re-split (same sum).
__global__ void maxpool3s2_s_kernel(const __bf16* __restrict__ in, int N, int H, int W, int C,
                                    __bf16* __restrict__ out, int Ho, int Wo) {
  const int g8 = C >> 3;
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)N * Ho * Wo * g8;
  if (idx >= total) return;
  const int g = (int)(idx % g8);
  const long pix = idx / g8;
  const int ow = (int)(pix % Wo);
  const int oh = (int)((pix / Wo) % Ho);
  const int n = (int)(pix / ((long)Wo * Ho));
  const int coff = (g >> 2) * 64 + (g & 3) * 8;  // within a pixel's C*2 bf16
  float m[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) m[q] = -INFINITY;
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
    int ih = oh * 2 - 1 + ky;
    if ((unsigned)ih >= (unsigned)H) continue;
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      int iw = ow * 2 - 1 + kx;
      if ((unsigned)iw >= (unsigned)W) continue;
      const __bf16* sp = in + (((long)n * H + ih) * W + iw) * (2L * C) + coff;
      const bf16x8 hi = *(const bf16x8*)sp, lo = *(const bf16x8*)(sp + 32);
#pragma unroll
      for (int q = 0; q < 8; ++q) m[q] = fmaxf(m[q], (float)hi[q] + (float)lo[q]);
    }
  }
  bf16x8 hi, lo;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    hi[q] = (__bf16)m[q];
    lo[q] = (__bf16)(m[q] - (float)hi[q]);
  }
  __bf16* dp = out + pix * (2L * C) + coff;
  *(bf16x8*)dp = hi;
  *(bf16x8*)(dp + 32) = lo;
}

// The same with two horizontally adjacent outputs per thread (round 3): their windows share
// input column 2*ow+1, so 15 pixel loads (hi + lo each) make two outputs instead of 18 making
// one; the channel group is the fastest index, so a wave still reads whole 128-B lines.
__global__ void maxpool3s2_s2_kernel(const __bf16* __restrict__ in, int N, int H, int W, int C,
                                     __bf16* __restrict__ out, int Ho, int Wo) {
  const int g8 = C >> 3, Wp = (Wo + 1) >> 1;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)N * Ho * Wp * g8;
  if (idx >= total) return;
  const int g = (int)(idx % g8);
  const long pp = idx / g8;
  const int owp = (int)(pp % Wp);
  const long nh = pp / Wp;
  const int oh = (int)(nh % Ho);
  const int n = (int)(nh / Ho);
  const int ow = 2 * owp;
  const int coff = (g >> 2) * 64 + (g & 3) * 8;
  float m0[8], m1[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) m0[q] = m1[q] = -INFINITY;
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
    const int ih = oh * 2 - 1 + ky;
    if ((unsigned)ih >= (unsigned)H) continue;
    const __bf16* rp = in + ((long)n * H + ih) * W * (2L * C) + coff;
#pragma unroll
    for (int kx = 0; kx < 5; ++kx) {
      const int iw = ow * 2 - 1 + kx;
      if ((unsigned)iw >= (unsigned)W) continue;
      const __bf16* sp = rp + (long)iw * (2L * C);
      const bf16x8 hi = *(const bf16x8*)sp, lo = *(const bf16x8*)(sp + 32);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float v = (float)hi[q] + (float)lo[q];
        if (kx < 3) m0[q] = fmaxf(m0[q], v);
        if (kx >= 2) m1[q] = fmaxf(m1[q], v);
      }
    }
  }
  const long pix = ((long)n * Ho + oh) * Wo + ow;
#pragma unroll
  for (int o = 0; o < 2; ++o) {
    if (ow + o >= Wo) break;
    bf16x8 hi, lo;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float m = o ? m1[q] : m0[q];
      hi[q] = (__bf16)m;
      lo[q] = (__bf16)(m - (float)hi[q]);
    }
    __bf16* dp = out + (pix + o) * (2L * C) + coff;
    *(bf16x8*)dp = hi;
    *(bf16x8*)(dp + 32) = lo;
  }
}

int launch_maxpool3s2_s(const __bf16* in, int N, int H, int W, int C, __bf16* out, int Ho, int Wo, hipStream_t st) {
  if (C % 32) return fail(CWT_EARG, "maxpool_s: C % 32");
  static const bool one = getenv("CWT_MAXPOOL1") && atoi(getenv("CWT_MAXPOOL1"));  // A/B switch
  if (!one) {
    const long total = (long)N * Ho * ((Wo + 1) / 2) * (C / 8);
    hipLaunchKernelGGL(maxpool3s2_s2_kernel, dim3(cdiv(total, 256)), dim3(256), 0, st, in, N, H, W, C, out, Ho, Wo);
    CWT_LAUNCH_CHECK();
    return 0;
  }
  long total = (long)N * Ho * Wo * (C / 8);
  hipLaunchKernelGGL(maxpool3s2_s_kernel, dim3(cdiv(total, 256)), dim3(256), 0, st, in, N, H, W, C, out, Ho, Wo);
  CWT_LAUNCH_CHECK();
  return 0;
}

// maxpool 3x3 s2 p1 on bf16 NHWC: one thread per (pixel, 8 channels); max is exact in bf16.
__global__ void maxpool3s2_b16_kernel(const __bf16* __restrict__ in, int N, int H, int W, int C,
                                      __bf16* __restrict__ out, int Ho, int Wo) {
  const int g8 = C >> 3;
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)N * Ho * Wo * g8;
  if (idx >= total) return;
  const int g = (int)(idx % g8);
  const long pix = idx / g8;
  const int ow = (int)(pix % Wo);
  const int oh = (int)((pix / Wo) % Ho);
  const int n = (int)(pix / ((long)Wo * Ho));
  float m[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) m[q] = -INFINITY;
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
    int ih = oh * 2 - 1 + ky;
    if ((unsigned)ih >= (unsigned)H) continue;
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      int iw = ow * 2 - 1 + kx;
      if ((unsigned)iw >= (unsigned)W) continue;
      const bf16x8 v = *(const bf16x8*)(in + (((long)n * H + ih) * W + iw) * C + g * 8);
#pragma unroll
      for (int q = 0; q < 8; ++q) m[q] = fmaxf(m[q], (float)v[q]);
    }
  }
  bf16x8 o;
#pragma unroll
  for (int q = 0; q < 8; ++q) o[q] = (__bf16)m[q];
  *(bf16x8*)(out + pix * C + g * 8) = o;
}

int launch_maxpool3s2_b16(const __bf16* in, int N, int H, int W, int C, __bf16* out, int Ho, int Wo,
                          hipStream_t st) {
  if (C % 8) return fail(CWT_EARG, "maxpool_b16: C % 8");
  long total = (long)N * Ho * Wo * (C / 8);
  hipLaunchKernelGGL(maxpool3s2_b16_kernel, dim3(cdiv(total, 256)), dim3(256), 0, st, in, N, H, W, C, out, Ho, Wo);
  CWT_LAUNCH_CHECK();
  return 0;
}

// Adaptive average pooling for all bins (pspnet.py:26), in three passes that each issue at
// most ~14 independent loads per thread:
//   segment boundaries = every window start / end along an axis (the windows of all bins
//   are unions of consecutive "elementary segments");
//   (1) rowseg[n][y][xs][c]  = sum of x[n][y][x][c] over x in x-segment xs
//   (2) blk[n][ys][xs][c]    = sum of rowseg over y in y-segment ys
//   (3) pooled[cell][c]      = ((sum of blk over the cell's segments) / kh) / kw
// (The summation order differs from aten's window loop at fp32 rounding level.)
struct PPMSegs {
  int nseg;
  int b[17];   // boundaries b[0] = 0 < ... < b[nseg] = in
  int w0[16];  // window k covers segments [w0[k], w1[k])
  int w1[16];
  int wst[16], wen[16];
  int nwin;
};

static PPMSegs make_segs(int in, const int* bins, int nbins) {
  PPMSegs sg;
  memset(&sg, 0, sizeof(sg));
  int bnd[40], nb = 0;
  for (int k = 0; k < nbins; ++k)
    for (int i = 0; i < bins[k]; ++i) {
      const int st = (i * in) / bins[k], en = ((i + 1) * in + bins[k] - 1) / bins[k];
      sg.wst[sg.nwin] = st;
      sg.wen[sg.nwin] = en;
      ++sg.nwin;
      bnd[nb++] = st;
      bnd[nb++] = en;
    }
  std::sort(bnd, bnd + nb);
  nb = (int)(std::unique(bnd, bnd + nb) - bnd);
  sg.nseg = nb - 1;
  for (int q = 0; q < nb; ++q) sg.b[q] = bnd[q];
  for (int k = 0; k < sg.nwin; ++k) {
    sg.w0[k] = (int)(std::lower_bound(bnd, bnd + nb, sg.wst[k]) - bnd);
    sg.w1[k] = (int)(std::lower_bound(bnd, bnd + nb, sg.wen[k]) - bnd);
  }
  return sg;
}

constexpr int PPM_MAXSEG = 16;  // longest elementary segment handled without a loop

// LAYOUT: ACT_SPLIT = x is the S-layout (pixel stride 2*C bf16; value = hi + lo), ACT_BF16 =
// bf16 NHWC (pixel stride C), ACT_F32 = fp32 (pixel stride ld).
template <int LAYOUT>
__global__ void ppm_rowseg_kernel(const float* __restrict__ x, int N, int h, int w, int ld, int C, PPMSegs sx,
                                  float* __restrict__ rowseg) {
  constexpr bool SPLIT = LAYOUT == ACT_SPLIT;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)N * h * sx.nseg * C;
  if (idx >= total) return;
  const int c = (int)(idx % C);
  const long r = idx / C;
  const int xs = (int)(r % sx.nseg);
  const long ny = r / sx.nseg;
  const int x0 = sx.b[xs], len = sx.b[xs + 1] - x0;
  const float* src = x + (ny * w + x0) * (long)ld + c;
  const __bf16* ssrc = (const __bf16*)x + (ny * w + x0) * (2L * C) + (c >> 5) * 64 + (c & 31);
  const __bf16* bsrc = (const __bf16*)x + (ny * w + x0) * (long)C + c;
  float s = 0.f;
  for (int u0 = 0; u0 < len; u0 += PPM_MAXSEG) {
    float v[PPM_MAXSEG];
#pragma unroll
    for (int u = 0; u < PPM_MAXSEG; ++u) {
      const long o = (long)min(u0 + u, len - 1);
      if (SPLIT)
        v[u] = (float)ssrc[o * 2 * C] + (float)ssrc[o * 2 * C + 32];
      else if (LAYOUT == ACT_BF16)
        v[u] = (float)bsrc[o * C];
      else
        v[u] = src[o * ld];
    }
#pragma unroll
    for (int u = 0; u < PPM_MAXSEG; ++u)
      if (u0 + u < len) s += v[u];
  }
  rowseg[idx] = s;
}

// The same pass over the S-layout / bf16 map with 8 channels per thread (round 3): one 16-B hi
// and one 16-B lo load per pixel (8 per pixel for bf16) instead of two 2-B loads per channel,
// and two 16-B stores.  The per-channel sum runs over the segment's pixels in the same order as
// the scalar form (identical result).
template <int LAYOUT>
__global__ void ppm_rowseg8_kernel(const __bf16* __restrict__ x, int N, int h, int w, int C, PPMSegs sx,
                                   float* __restrict__ rowseg) {
  constexpr bool SPLIT = LAYOUT == ACT_SPLIT;
  const int C8 = C >> 3;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)N * h * sx.nseg * C8;
  if (idx >= total) return;
  const int c8 = (int)(idx % C8);
  const long r = idx / C8;
  const int xs = (int)(r % sx.nseg);
  const long ny = r / sx.nseg;
  const int x0 = sx.b[xs], len = sx.b[xs + 1] - x0;
  const long pstride = SPLIT ? 2L * C : (long)C;
  const __bf16* src = x + (ny * w + x0) * pstride + (SPLIT ? (c8 >> 2) * 64 + (c8 & 3) * 8 : c8 * 8);
  float s[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) s[q] = 0.f;
  for (int u0 = 0; u0 < len; u0 += 8) {
    bf16x8 hv[8], lv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const long o = (long)min(u0 + u, len - 1) * pstride;
      hv[u] = *(const bf16x8*)(src + o);
      if (SPLIT) lv[u] = *(const bf16x8*)(src + o + 32);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (u0 + u < len)
#pragma unroll
        for (int q = 0; q < 8; ++q) s[q] += SPLIT ? (float)hv[u][q] + (float)lv[u][q] : (float)hv[u][q];
  }
  float* d = rowseg + idx * 8;
  *(f32x4*)d = f32x4{s[0], s[1], s[2], s[3]};
  *(f32x4*)(d + 4) = f32x4{s[4], s[5], s[6], s[7]};
}

__global__ void ppm_blk_kernel(const float* __restrict__ rowseg, int N, int h, int C, PPMSegs sx, PPMSegs sy,
                               float* __restrict__ blk) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)N * sy.nseg * sx.nseg * C;
  if (idx >= total) return;
  const int c = (int)(idx % C);
  long r = idx / C;
  const int xs = (int)(r % sx.nseg);
  r /= sx.nseg;
  const int ys = (int)(r % sy.nseg);
  const int n = (int)(r / sy.nseg);
  const int y0 = sy.b[ys], len = sy.b[ys + 1] - y0;
  const long rstride = (long)sx.nseg * C;
  const float* src = rowseg + (((long)n * h + y0) * sx.nseg + xs) * C + c;
  float s = 0.f;
  for (int u0 = 0; u0 < len; u0 += PPM_MAXSEG) {
    float v[PPM_MAXSEG];
#pragma unroll
    for (int u = 0; u < PPM_MAXSEG; ++u) v[u] = src[min(u0 + u, len - 1) * rstride];
#pragma unroll
    for (int u = 0; u < PPM_MAXSEG; ++u)
      if (u0 + u < len) s += v[u];
  }
  blk[idx] = s;
}

// pooled (bin-major, [sum_b N*b*b][C]); one thread per (n, cell, c)
__global__ void ppm_cell_kernel(const float* __restrict__ blk, int N, int C, PPMSegs sx, PPMSegs sy, int b0, int b1,
                                int b2, int b3, float* __restrict__ pooled) {
  const int bins[4] = {b0, b1, b2, b3};
  const int ncells = b0 * b0 + b1 * b1 + b2 * b2 + b3 * b3;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)N * ncells * C;
  if (idx >= total) return;
  const int c = (int)(idx % C);
  const int cell = (int)((idx / C) % ncells);
  const int n = (int)(idx / ((long)C * ncells));
  int base = 0, woff = 0, k = 0;
  while (cell >= base + bins[k] * bins[k]) {
    base += bins[k] * bins[k];
    woff += bins[k];
    ++k;
  }
  const int b = bins[k];
  const int i = (cell - base) / b, j = (cell - base) % b;
  const int ya = sy.w0[woff + i], yb = sy.w1[woff + i];
  const int xa = sx.w0[woff + j], xb = sx.w1[woff + j];
  float s = 0.f;
  for (int ys = ya; ys < yb; ++ys) {
    float v[PPM_MAXSEG];
    const float* src = blk + (((long)n * sy.nseg + ys) * sx.nseg) * C + c;
#pragma unroll
    for (int u = 0; u < PPM_MAXSEG; ++u) v[u] = src[(long)min(xa + u, xb - 1) * C];
#pragma unroll
    for (int u = 0; u < PPM_MAXSEG; ++u)
      if (xa + u < xb) s += v[u];
  }
  const float kh = (float)(sy.wen[woff + i] - sy.wst[woff + i]), kw = (float)(sx.wen[woff + j] - sx.wst[woff + j]);
  pooled[((long)base * N + (long)n * b * b + i * b + j) * C + c] = (s / kh) / kw;
}

// ws: rowseg [N][h][nseg_x][C] followed by blk [N][nseg_y][nseg_x][C]
int launch_ppm(const float* x, int N, int h, int w, int ld, const int* bins, int nbins, float* ws,
               float* pooled, hipStream_t st, int layout) {
  if (nbins != 4) return fail(CWT_EARG, "PPM expects 4 bins");
  const PPMSegs sx = make_segs(w, bins, nbins), sy = make_segs(h, bins, nbins);
  if (sx.nwin > 16 || sx.nseg > 16 || sy.nseg > 16) return fail(CWT_EARG, "PPM: too many windows");
  const int C = 2048;
  float* rowseg = ws;
  float* blk = ws + (long)N * h * sx.nseg * C;
  const long t1 = (long)N * h * sx.nseg * C;
  if (layout == ACT_SPLIT)
    hipLaunchKernelGGL(ppm_rowseg8_kernel<ACT_SPLIT>, dim3(cdiv(t1 / 8, 256)), dim3(256), 0, st, (const __bf16*)x, N,
                       h, w, C, sx, rowseg);
  else if (layout == ACT_BF16)
    hipLaunchKernelGGL(ppm_rowseg8_kernel<ACT_BF16>, dim3(cdiv(t1 / 8, 256)), dim3(256), 0, st, (const __bf16*)x, N,
                       h, w, C, sx, rowseg);
  else
    hipLaunchKernelGGL(ppm_rowseg_kernel<ACT_F32>, dim3(cdiv(t1, 256)), dim3(256), 0, st, x, N, h, w, ld, C, sx,
                       rowseg);
  CWT_LAUNCH_CHECK();
  const long t2 = (long)N * sy.nseg * sx.nseg * C;
  hipLaunchKernelGGL(ppm_blk_kernel, dim3(cdiv(t2, 256)), dim3(256), 0, st, (const float*)rowseg, N, h, C, sx, sy,
                     blk);
  CWT_LAUNCH_CHECK();
  int ncells = 0;
  for (int k = 0; k < nbins; ++k) ncells += bins[k] * bins[k];
  const long t3 = (long)N * ncells * C;
  hipLaunchKernelGGL(ppm_cell_kernel, dim3(cdiv(t3, 256)), dim3(256), 0, st, (const float*)blk, N, C, sx, sy, bins[0],
                     bins[1], bins[2], bins[3], pooled);
  CWT_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------------------------------
// PPM branch of the bottleneck conv, folded (pspnet.py:19-38,124-128).
//
// The bottleneck conv reads concat[layer4 (2048 ch), up_b(P_b) (4 x 512 ch)], where
// P_b = relu(BN(conv1x1(pool_b(x)))) lives on a b x b grid (b = 1, 2, 3, 6) and up_b is the
// bilinear align_corners upsample to h x w.  Both the upsample and the conv are linear, so
//   conv3x3(W_b, up_b(P_b))(y, x) = sum_{ky,kx} sum_{i,j} u_b(y+ky-1, i) u_b(x+kx-1, j) Q_b[i][j][ky][kx]
// with Q_b[i][j][tap] = W_b[tap] . P_b[i][j] (a 512 x 4608 GEMM over the b*b cells) and
// u_b the 1-D interpolation weights (zero outside [0, h): the conv's zero padding).  The
// bottleneck conv then only runs over the 2048 layer4 channels (half its FLOPs) with the
// PPM field F added in its epilogue as a residual (BN scale pre-folded into Q's weights).
// ---------------------------------------------------------------------------------------

// Small-M fp32 GEMM, block-diagonal over up to 4 problems sharing N and K:
//   part[ks][m][n] = sum_{k in chunk ks} A[m][k] Bt_p[k][n]   for rows m of problem p.
// Weights are stored K-major so a wave streams 64 consecutive n of one k row (coalesced);
// the A block (SG_MB rows x kc) sits in LDS and is read as broadcasts.  Each wave owns 64
// columns over the whole chunk, so no cross-wave reduction; chunks are summed in fixed
// order by smallm_finish_kernel (deterministic).
constexpr int SG_MB = 24;  // rows per workgroup: the A block (24 x 64 fp32) fits the scalar cache
typedef const float __attribute__((address_space(4))) const_f32;
struct SmallGemmArgs {
  const float* A;      // [Mtot][lda]
  const float* Bt[4];  // [K][N] per problem
  float* part;         // [nks][Mtot][N]
  int row0[4], M[4], wg0[5];
  int np, Mtot, N, K, lda, nks;
};

// Each lane first issues the loads of its whole B column chunk (KC values in flight), then
// runs rows x KC FMAs whose A operand is wave-uniform: read with scalar loads (SGPR operands
// of v_fma), so the broadcast costs neither LDS bandwidth nor VGPRs.
template <int KC>
__global__ __launch_bounds__(256) void smallm_gemm_kernel(SmallGemmArgs g) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  int p = 0;
  while (p + 1 < g.np && (int)blockIdx.x >= g.wg0[p + 1]) ++p;
  int w = (int)blockIdx.x - g.wg0[p];
  const int nnb = g.N / 256;
  const int nb = w % nnb;
  w /= nnb;
  const int ks = w % g.nks;
  const int mb = w / g.nks;
  const int m0 = g.row0[p] + mb * SG_MB;
  const int rows = min(SG_MB, g.row0[p] + g.M[p] - m0);
  const int k0 = ks * KC;
  const int n = nb * 256 + wv * 64 + lane;
  const float* b = g.Bt[p] + (long)k0 * g.N + n;
  float bv[KC];
#pragma unroll
  for (int k = 0; k < KC; ++k) bv[k] = b[(long)k * g.N];
  float* o = g.part + ((long)ks * g.Mtot + m0) * g.N + n;
  for (int r0 = 0; r0 < rows; r0 += 4) {
    float acc[4];
    const_f32* ar[4];  // constant address space: uniform reads become s_load
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      acc[r] = 0.f;
      ar[r] = (const_f32*)(g.A + (long)min(m0 + r0 + r, g.Mtot - 1) * g.lda + k0);  // clamped: a valid row
    }
#pragma unroll
    for (int k = 0; k < KC; ++k)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[r] = fmaf(ar[r][k], bv[k], acc[r]);
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (r0 + r < rows) o[(long)(r0 + r) * g.N] = acc[r];
  }
}

// out[m][n] = sum_ks part[ks][m][n] (fixed order), then for problems with a BN:
// relu(scale[n] * s + shift[n]).
struct SmallFinishArgs {
  const float* scale[4];
  const float* shift[4];
  int row0[5];
  int np;
};
__global__ void smallm_finish_kernel(const float* __restrict__ part, int nks, int Mtot, int N, SmallFinishArgs f,
                                     float* __restrict__ out) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)Mtot * (N >> 2);
  if (idx >= total) return;
  const long e = idx * 4;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  const long cs = (long)Mtot * N;
  for (int k0 = 0; k0 < nks; k0 += 8) {  // 8 loads in flight, summed in chunk order
    f32x4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = *(const f32x4*)(part + min(k0 + u, nks - 1) * cs + e);
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (k0 + u < nks) s += v[u];
  }
  const int m = (int)(e / N), n = (int)(e % N);
  int p = 0;
  while (p + 1 < f.np && m >= f.row0[p + 1]) ++p;
  if (f.scale[p]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) s[q] = fmaxf(fmaf(s[q], f.scale[p][n + q], f.shift[p][n + q]), 0.f);
  }
  *(f32x4*)(out + e) = s;
}

int launch_smallm_gemm(const float* A, int lda, const float* const* Bt, const int* M, int np, int N, int K, int kc,
                       float* part, size_t part_floats, const float* const* scale, const float* const* shift,
                       float* out, hipStream_t st) {
  if (np < 1 || np > 4 || N % 256 != 0 || (kc != 32 && kc != 64) || K % kc != 0)
    return fail(CWT_EARG, "smallm_gemm: need 1..4 problems, N % 256 == 0, kc in {32, 64}, K % kc == 0");
  SmallGemmArgs g;
  memset(&g, 0, sizeof(g));
  SmallFinishArgs f;
  memset(&f, 0, sizeof(f));
  g.A = A;
  g.part = part;
  g.np = f.np = np;
  g.N = N;
  g.K = K;
  g.lda = lda;
  g.nks = K / kc;
  int row = 0, wg = 0;
  for (int q = 0; q < np; ++q) {
    g.Bt[q] = Bt[q];
    g.row0[q] = f.row0[q] = row;
    g.M[q] = M[q];
    g.wg0[q] = wg;
    f.scale[q] = scale ? scale[q] : nullptr;
    f.shift[q] = shift ? shift[q] : nullptr;
    row += M[q];
    wg += cdiv(M[q], SG_MB) * g.nks * (N / 256);
  }
  g.wg0[np] = wg;
  f.row0[np] = row;
  g.Mtot = row;
  if ((size_t)g.nks * row * N > part_floats) return fail(CWT_ESTATE, "smallm_gemm: partial workspace too small");
  if (kc == 32)
    hipLaunchKernelGGL(smallm_gemm_kernel<32>, dim3(wg), dim3(256), 0, st, g);
  else
    hipLaunchKernelGGL(smallm_gemm_kernel<64>, dim3(wg), dim3(256), 0, st, g);
  CWT_LAUNCH_CHECK();
  const long total = (long)row * (N / 4);
  hipLaunchKernelGGL(smallm_finish_kernel, dim3(cdiv(total, 256)), dim3(256), 0, st, (const float*)part, g.nks, row,
                     N, f, out);
  CWT_LAUNCH_CHECK();
  return 0;
}

// Few-row form of the two PPM GEMMs (one or two episodes: <= kPpmGemmMaxRows cells) on the
// exact f32 matrix cores: v_mfma_f32_16x16x4_f32 is an fmaf chain per output (MI355X_MICROARCH
// "f32 in"), so this is plain fp32 arithmetic in a fixed order.  The VALU form of this GEMM is
// LDS-bound (a 64-lane broadcast read per 4 FMAs), the split-K VALU form is bound by its
// partials; here each workgroup owns up to 32 rows x 64 columns of one problem over a K slice:
//  * its W waves take 64 consecutive k each, all loaded up front; a lane loads A[row l&15][4 k] and, for 4 k rows,
//    B[k][4 columns] as 16-B vectors, and column block cb of the MFMA holds the columns
//    n0 + 4j + cb (j = l&15), so B lines and the output rows are contiguous 256-B segments;
//  * the W per-wave 16x64 tiles are summed in wave order through LDS (deterministic), then
//    BN + ReLU (one K slice) or a partial row of [ks][Mtot][N] for smallm_finish_kernel;
//  * tiles (problem, K slice, strip, row group), row group fastest, are dealt to the 8 XCDs in
//    contiguous runs, so the row groups re-reading one weight strip share an L2.
struct PpmMfmaArgs {
  const float* A;
  const float* Bt[4];
  const float* scale[4];
  const float* shift[4];
  float* out;
  int row0[4], M[4], nrg[4], tile0[5];
  int np, N, lda, ksl, nks, nstrips, Mtot, per_xcd;
};

template <int W, int RTW, int KI>
__global__ __launch_bounds__(64 * W) void ppm_mfma_kernel(PpmMfmaArgs g) {
  static_assert(W >= 4, "the reduction gives waves 0..3 one output register each");
  __shared__ __attribute__((aligned(16))) float red[W * 16 * 64];
  const int tile = (int)(blockIdx.x & 7) * g.per_xcd + (int)(blockIdx.x >> 3);
  if (tile >= g.tile0[g.np]) return;  // padding of the XCD runs: the whole workgroup leaves
  int p = 0;
  while (p + 1 < g.np && tile >= g.tile0[p + 1]) ++p;
  int local = tile - g.tile0[p];
  const int rg = local % g.nrg[p];
  local /= g.nrg[p];
  const int strip = local % g.nstrips, ks = local / g.nstrips;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, g4 = lane >> 4, c16 = lane & 15;
  const int m0 = g.row0[p] + rg * RTW * 16, mend = g.row0[p] + g.M[p];
  const int n0 = strip * 64 + 4 * c16;
  const int kb = ks * g.ksl + wv * 16 * KI;  // ksl == W * 16 * KI (checked at launch)
  const float* ar[RTW];
#pragma unroll
  for (int rt = 0; rt < RTW; ++rt)  // rows past the problem read a valid row; never stored
    ar[rt] = g.A + (long)min(m0 + rt * 16 + c16, mend - 1) * g.lda + kb + 4 * g4;
  const float* bp = g.Bt[p] + (long)(kb + 4 * g4) * g.N + n0;
  f32x4 acc[RTW][4];
#pragma unroll
  for (int rt = 0; rt < RTW; ++rt)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) acc[rt][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  // The wave's whole K range (KI steps of 16 k) is loaded up front: at one or two workgroups
  // per CU a prefetch of one step leaves every step waiting out a memory round trip.
  f32x4 a[KI][RTW], b[KI][4];
#pragma unroll
  for (int i = 0; i < KI; ++i) {
#pragma unroll
    for (int rt = 0; rt < RTW; ++rt) a[i][rt] = *(const f32x4*)(ar[rt] + 16 * i);
#pragma unroll
    for (int q = 0; q < 4; ++q) b[i][q] = *(const f32x4*)(bp + (long)(16 * i + q) * g.N);
  }
  __builtin_amdgcn_sched_barrier(0);  // keep every load ahead of the first MFMA
#pragma unroll
  for (int i = 0; i < KI; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int rt = 0; rt < RTW; ++rt)
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
          acc[rt][cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][rt][q], b[i][q][cb], acc[rt][cb], 0, 0, 0);
  const float* sc = g.nks == 1 ? g.scale[p] : nullptr;
  const float* sh = g.shift[p];
  float* o = g.out + (long)ks * g.Mtot * g.N + n0;
#pragma unroll
  for (int rt = 0; rt < RTW; ++rt) {
    if (m0 + rt * 16 >= mend) break;  // uniform
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int v = 0; v < 4; ++v) red[(wv * 16 + v * 4 + cb) * 64 + lane] = acc[rt][cb][v];
    __syncthreads();
    if (wv < 4) {  // D row 4*g4 + v, column block cb; summed over the waves in order
      const int v = wv;
      f32x4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int w = 0; w < W; ++w)
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) s[cb] += red[(w * 16 + v * 4 + cb) * 64 + lane];
      const int row = m0 + rt * 16 + 4 * g4 + v;
      if (row < mend) {
        if (sc) {
#pragma unroll
          for (int q = 0; q < 4; ++q) s[q] = fmaxf(fmaf(s[q], sc[n0 + q], sh[n0 + q]), 0.f);
        }
        *(f32x4*)(o + (long)row * g.N) = s;
      }
    }
    __syncthreads();
  }
}

int launch_ppm_gemm(const float* A, int lda, const float* const* Bt, const int* M, int np, int N, int K,
                    const float* const* scale, const float* const* shift, float* part, size_t part_floats,
                    float* out, hipStream_t st) {
  // K = 512 (the per-tap fold, N = 4608): one K slice, 8 waves; K = 2048 (the 1x1 conv, N = 512:
  // only 8 strips) in 8 slices of 4 waves, summed by smallm_finish_kernel.
  const int nks = K == 2048 ? 8 : 1, W = K == 2048 ? 4 : 8;
  constexpr int RTW = 2, KI = 4;  // 64 k per wave: 512 = 8 waves x 64, 2048 = 8 slices x 4 waves x 64
  if (np < 1 || np > 4 || N % 64 != 0 || (K != 512 && K != 2048) || lda < K || lda % 4 ||
      ((uintptr_t)A & 15))
    return fail(CWT_EARG, "ppm_gemm: need 1..4 problems, N % 64 == 0, K in {512, 2048}, 16-B aligned rows");
  PpmMfmaArgs g;
  memset(&g, 0, sizeof(g));
  SmallFinishArgs f;
  memset(&f, 0, sizeof(f));
  g.A = A;
  g.np = f.np = np;
  g.N = N;
  g.lda = lda;
  g.ksl = K / nks;
  g.nks = nks;
  g.nstrips = N / 64;
  int row = 0, tiles = 0;
  for (int q = 0; q < np; ++q) {
    if (M[q] < 1) return fail(CWT_EARG, "ppm_gemm: empty problem");
    g.Bt[q] = Bt[q];
    g.scale[q] = f.scale[q] = scale ? scale[q] : nullptr;
    g.shift[q] = f.shift[q] = shift ? shift[q] : nullptr;
    g.row0[q] = f.row0[q] = row;
    g.M[q] = M[q];
    g.nrg[q] = cdiv(M[q], RTW * 16);
    g.tile0[q] = tiles;
    row += M[q];
    tiles += g.nrg[q] * g.nstrips * nks;
  }
  g.tile0[np] = tiles;
  f.row0[np] = row;
  g.Mtot = row;
  g.per_xcd = cdiv(tiles, 8);
  g.out = nks == 1 ? out : part;
  if (nks > 1 && (size_t)nks * row * N > part_floats) return fail(CWT_ESTATE, "ppm_gemm: partial workspace too small");
  const dim3 grid(8 * g.per_xcd);
  if (W == 8)
    hipLaunchKernelGGL((ppm_mfma_kernel<8, RTW, KI>), grid, dim3(512), 0, st, g);
  else
    hipLaunchKernelGGL((ppm_mfma_kernel<4, RTW, KI>), grid, dim3(256), 0, st, g);
  CWT_LAUNCH_CHECK();
  if (nks > 1) {
    const long total = (long)row * (N / 4);
    hipLaunchKernelGGL(smallm_finish_kernel, dim3(cdiv(total, 256)), dim3(256), 0, st, (const float*)part, nks, row,
                       N, f, out);
    CWT_LAUNCH_CHECK();
  }
  return 0;
}

// Interpolation table for destination p in [-1, out] (the 3x3 conv's zero padding outside
// [0, out)): source cells i0, i1 with weights l0, l1 of the align_corners upsample in -> out.
struct LerpEntry {
  int i0, i1;
  float l0, l1;
};
__device__ __forceinline__ LerpEntry lerp_entry(int p, int out, int in) {
  LerpEntry e{0, 0, 0.f, 0.f};
  if (p < 0 || p >= out) return e;
  const float sc = (out > 1) ? (float)(in - 1) / (float)(out - 1) : 0.f;
  const Lerp l = lerp_coord(p, in, sc);
  e.i0 = l.i0;
  e.i1 = l.i1;
  e.l0 = l.l0;
  e.l1 = l.l1;
  return e;
}

struct PPMBins {
  int b[4];
  int cell0[4];  // first cell (per image) of bin k in the bin-major cell order: 0, 1, 5, 14
  int row0[4];   // first grid row of bin k among the 12 rows (1 + 2 + 3 + 6): 0, 1, 3, 6
};

constexpr int PPM_MAXS = 160;  // largest feature side the field kernels take (641 -> 81)

// Pass 1 (columns): R[n][row][x][ky][c] = sum_{kx} sum_{j in {i0, i1}(x+kx-1)} u Q[cell(row, j)][ky*3+kx][c].
// Workgroup = (n, grid row, 64 channels); Q for the row's cells staged in LDS.
__global__ __launch_bounds__(256) void ppm_field_cols_kernel(const float* __restrict__ Q, int N, int w, PPMBins bn,
                                                             float* __restrict__ R) {
  __shared__ f32x4 qs[6 * 9 * 16];
  __shared__ LerpEntry tab[PPM_MAXS + 2];
  const int t = threadIdx.x;
  const int n = blockIdx.x / 12, row = blockIdx.x % 12, c0 = blockIdx.y * 64;
  int k = 3;
  while (row < bn.row0[k]) --k;
  const int b = bn.b[k], i = row - bn.row0[k];
  const long cell0 = (long)bn.cell0[k] * N + (long)n * b * b + (long)i * b;  // first cell of this grid row
  for (int e = t; e < b * 9 * 16; e += 256) {
    const int c4 = e & 15, jt = e >> 4;  // jt = j * 9 + tap
    qs[e] = *(const f32x4*)(Q + (cell0 + jt / 9) * 4608 + (jt % 9) * 512 + c0 + 4 * c4);
  }
  for (int p = t; p < w + 2; p += 256) tab[p] = lerp_entry(p - 1, w, b);
  __syncthreads();
  for (int e = t; e < w * 3 * 16; e += 256) {
    const int c4 = e & 15, xk = e >> 4;
    const int x = xk / 3, ky = xk - 3 * (xk / 3);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const LerpEntry l = tab[x + kx];  // destination x + kx - 1
      acc += l.l0 * qs[(l.i0 * 9 + ky * 3 + kx) * 16 + c4];
      acc += l.l1 * qs[(l.i1 * 9 + ky * 3 + kx) * 16 + c4];
    }
    *(f32x4*)(R + ((((long)n * 12 + row) * w + x) * 3 + ky) * 512 + c0 + 4 * c4) = acc;
  }
}

// Pass 2 (rows): F[n][y][x][c] = sum_{k, ky} sum_{i in {i0, i1}(y+ky-1)} u_k R[n][row(k, i)][x][ky][c].
// Workgroup = (n, x, 64 channels); the 12 x 3 R vectors of this column staged in LDS.
__global__ __launch_bounds__(256) void ppm_field_rows_kernel(const float* __restrict__ R, int N, int h, int w,
                                                             PPMBins bn, float* __restrict__ F) {
  __shared__ f32x4 rs[12 * 3 * 16];
  __shared__ LerpEntry tab[4][PPM_MAXS + 2];
  const int t = threadIdx.x;
  const int n = blockIdx.x / w, x = blockIdx.x % w, c0 = blockIdx.y * 64;
  for (int e = t; e < 12 * 3 * 16; e += 256) {
    const int c4 = e & 15, rk = e >> 4;  // rk = row * 3 + ky
    rs[e] = *(const f32x4*)(R + ((((long)n * 12 + rk / 3) * w + x) * 3 + rk % 3) * 512 + c0 + 4 * c4);
  }
  for (int e = t; e < 4 * (h + 2); e += 256) {
    const int k = e / (h + 2), p = e - k * (h + 2);
    tab[k][p] = lerp_entry(p - 1, h, bn.b[k]);
  }
  __syncthreads();
  for (int e = t; e < h * 16; e += 256) {
    const int c4 = e & 15, y = e >> 4;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const LerpEntry l = tab[k][y + ky];  // destination y + ky - 1
        acc += l.l0 * rs[((bn.row0[k] + l.i0) * 3 + ky) * 16 + c4];
        acc += l.l1 * rs[((bn.row0[k] + l.i1) * 3 + ky) * 16 + c4];
      }
    *(f32x4*)(F + (((long)n * h + y) * w + x) * 512 + c0 + 4 * c4) = acc;
  }
}

int launch_ppm_field(const float* Q, int N, int h, int w, const int* bins, float* R, float* F, hipStream_t st) {
  PPMBins bn;
  int cell = 0, row = 0;
  for (int k = 0; k < 4; ++k) {
    bn.b[k] = bins[k];
    bn.cell0[k] = cell;
    bn.row0[k] = row;
    cell += bins[k] * bins[k];
    row += bins[k];
  }
  if (row != 12 || bins[3] > 6 || h > PPM_MAXS || w > PPM_MAXS)
    return fail(CWT_EARG, "PPM field expects bins {1,2,3,6} and a feature side <= 160");
  hipLaunchKernelGGL(ppm_field_cols_kernel, dim3(N * 12, 8), dim3(256), 0, st, Q, N, w, bn, R);
  CWT_LAUNCH_CHECK();
  hipLaunchKernelGGL(ppm_field_rows_kernel, dim3(N * w, 8), dim3(256), 0, st, (const float*)R, N, h, w, bn, F);
  CWT_LAUNCH_CHECK();
  return 0;
}


// Adjoint of the PPM field (stage-1 pretraining, pretrain.hip): dQ = field^T(dF), gathered in
// fixed order (no atomics), the two passes of launch_ppm_field in reverse.
// Pass 1 (rows): dR[n][row(k, i)][x][ky][c] = sum_y u_k(y+ky-1 -> i) dF[n][y][x][c].
// Workgroup = (n, x, 64 channels); the dF column (h x 64 channels) staged in LDS.
__global__ __launch_bounds__(256) void ppm_field_bwd_rows_kernel(const float* __restrict__ dF, int N, int h, int w,
                                                                 PPMBins bn, float* __restrict__ dR) {
  __shared__ f32x4 gs[PPM_MAXS * 16];
  __shared__ LerpEntry tab[4][PPM_MAXS + 2];
  const int t = threadIdx.x;
  const int n = blockIdx.x / w, x = blockIdx.x % w, c0 = blockIdx.y * 64;
  for (int e = t; e < h * 16; e += 256) {
    const int c4 = e & 15, y = e >> 4;
    gs[e] = *(const f32x4*)(dF + (((long)n * h + y) * w + x) * 512 + c0 + 4 * c4);
  }
  for (int e = t; e < 4 * (h + 2); e += 256) {
    const int k = e / (h + 2), p = e - k * (h + 2);
    tab[k][p] = lerp_entry(p - 1, h, bn.b[k]);
  }
  __syncthreads();
  for (int e = t; e < 12 * 3 * 16; e += 256) {
    const int c4 = e & 15, rk = e >> 4;
    const int row = rk / 3, ky = rk - 3 * row;
    int k = 3;
    while (row < bn.row0[k]) --k;
    const int i = row - bn.row0[k];
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int y = 0; y < h; ++y) {
      const LerpEntry l = tab[k][y + ky];  // destination y + ky - 1
      const float u = (l.i0 == i ? l.l0 : 0.f) + (l.i1 == i ? l.l1 : 0.f);
      acc += u * gs[y * 16 + c4];
    }
    *(f32x4*)(dR + ((((long)n * 12 + row) * w + x) * 3 + ky) * 512 + c0 + 4 * c4) = acc;
  }
}

// Pass 2 (columns): dQ[cell(row, j)][ky*3+kx][c] = sum_x u(x+kx-1 -> j) dR[n][row][x][ky][c].
// Workgroup = (n, grid row, 64 channels); dR staged in LDS 32 columns at a time.
constexpr int PPM_BWD_XC = 32;
__global__ __launch_bounds__(256) void ppm_field_bwd_cols_kernel(const float* __restrict__ dR, int N, int w,
                                                                 PPMBins bn, float* __restrict__ dQ) {
  __shared__ f32x4 rs[PPM_BWD_XC * 3 * 16];
  __shared__ LerpEntry tab[PPM_MAXS + 2];
  const int t = threadIdx.x;
  const int n = blockIdx.x / 12, row = blockIdx.x % 12, c0 = blockIdx.y * 64;
  int k = 3;
  while (row < bn.row0[k]) --k;
  const int b = bn.b[k], i = row - bn.row0[k];
  const long cell0 = (long)bn.cell0[k] * N + (long)n * b * b + (long)i * b;
  for (int p = t; p < w + 2; p += 256) tab[p] = lerp_entry(p - 1, w, b);
  const int nout = b * 9 * 16;  // (j, tap, c4), at most 864: 4 per thread
  f32x4 acc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int xc = 0; xc < w; xc += PPM_BWD_XC) {
    const int nx = min(PPM_BWD_XC, w - xc);
    __syncthreads();
    for (int e = t; e < nx * 3 * 16; e += 256) {
      const int c4 = e & 15, xk = e >> 4;  // xk = x * 3 + ky
      rs[e] = *(const f32x4*)(dR + ((((long)n * 12 + row) * w + xc + xk / 3) * 3 + xk % 3) * 512 + c0 + 4 * c4);
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = t + 256 * q;
      if (e >= nout) break;
      const int c4 = e & 15, jt = e >> 4;
      const int j = jt / 9, tap = jt - 9 * j, ky = tap / 3, kx = tap - 3 * ky;
      for (int xl = 0; xl < nx; ++xl) {
        const LerpEntry l = tab[xc + xl + kx];  // destination x + kx - 1
        const float u = (l.i0 == j ? l.l0 : 0.f) + (l.i1 == j ? l.l1 : 0.f);
        acc[q] += u * rs[(xl * 3 + ky) * 16 + c4];
      }
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int e = t + 256 * q;
    if (e >= nout) break;
    const int c4 = e & 15, jt = e >> 4;
    *(f32x4*)(dQ + (cell0 + jt / 9) * 4608 + (jt % 9) * 512 + c0 + 4 * c4) = acc[q];
  }
}

int launch_ppm_field_bwd(const float* dF, int N, int h, int w, const int* bins, float* dR, float* dQ, hipStream_t st) {
  PPMBins bn;
  int cell = 0, row = 0;
  for (int k = 0; k < 4; ++k) {
    bn.b[k] = bins[k];
    bn.cell0[k] = cell;
    bn.row0[k] = row;
    cell += bins[k] * bins[k];
    row += bins[k];
  }
  if (row != 12 || bins[3] > 6 || h > PPM_MAXS || w > PPM_MAXS)
    return fail(CWT_EARG, "PPM field adjoint expects bins {1,2,3,6} and a feature side <= 160");
  hipLaunchKernelGGL(ppm_field_bwd_rows_kernel, dim3(N * w, 8), dim3(256), 0, st, dF, N, h, w, bn, dR);
  CWT_LAUNCH_CHECK();
  hipLaunchKernelGGL(ppm_field_bwd_cols_kernel, dim3(N * 12, 8), dim3(256), 0, st, (const float*)dR, N, w, bn, dQ);
  CWT_LAUNCH_CHECK();
  return 0;
}

}  // namespace cwt

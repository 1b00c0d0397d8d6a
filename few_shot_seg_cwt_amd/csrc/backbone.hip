// Byte-moving pieces of the frozen extractor around the MFMA convs:
//  * stem conv1 (3->64, 3x3 s2 p1, K = 27: too thin for the implicit GEMM) + BN + ReLU,
//    reading the caller's NCHW image and writing NHWC            (resnet.py:111-112,147)
//  * maxpool 3x3 s2 p1 (-inf padding)                           (resnet.py:118)
//  * PPM adaptive average pooling for all bins in one sweep     (pspnet.py:26)
//  * PPM bilinear(align_corners) upsample written straight into the concat buffer
//    channel slices, so torch.cat never materialises a copy  (pspnet.py:37-38)
#include "common.h"
#include "kernels.h"

namespace cwt {

// One thread per output pixel, all 64 output channels; weights [ci][ky][kx][co] in LDS.
__global__ __launch_bounds__(256) void stem_conv1_kernel(const float* __restrict__ img, int N, int S,
                                                         const float* __restrict__ w,
                                                         const float* __restrict__ scale,
                                                         const float* __restrict__ shift,
                                                         float* __restrict__ out, int Ho) {
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
  for (int c4 = 0; c4 < 16; ++c4) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 27; ++k) {
      f32x4 wv = *(const f32x4*)&ws[k * 64 + c4 * 4];
      acc += in[k] * wv;
    }
    f32x4 r;
#pragma unroll
    for (int q = 0; q < 4; ++q) r[q] = fmaxf(fmaf(acc[q], ss[c4 * 4 + q], bs[c4 * 4 + q]), 0.f);
    *(f32x4*)(o + c4 * 4) = r;
  }
}

int launch_stem_conv1(const float* img, int N, int S, const float* w27x64, const float* scale,
                      const float* shift, float* out, int Ho, hipStream_t st) {
  long total = (long)N * Ho * Ho;
  hipLaunchKernelGGL(stem_conv1_kernel, dim3(cdiv(total, 256)), dim3(256), 0, st, img, N, S, w27x64, scale,
                     shift, out, Ho);
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

// Adaptive-pool windows: start = floor(i*in/b), end = ceil((i+1)*in/b)
// (aten adaptive_avg_pool2d start_index/end_index).
struct PPMWindows {
  int nwin;
  int st[16], en[16];
};

static PPMWindows make_windows(int in, const int* bins, int nbins) {
  PPMWindows wd;
  wd.nwin = 0;
  for (int b = 0; b < nbins; ++b)
    for (int i = 0; i < bins[b]; ++i) {
      wd.st[wd.nwin] = (i * in) / bins[b];
      wd.en[wd.nwin] = ((i + 1) * in + bins[b] - 1) / bins[b];
      ++wd.nwin;
    }
  return wd;
}

// colsum[n][y][win][c] = sum_{x in window} cat[n][y][x][c]; one thread per (n, y, c4).
__global__ void ppm_colsum_kernel(const float* __restrict__ cat, int N, int h, int w, int ld, int C,
                                  PPMWindows wd, float* __restrict__ colsum) {
  const int c4n = C >> 2;
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)N * h * c4n;
  if (idx >= total) return;
  int c4 = (int)(idx % c4n);
  long ny = idx / c4n;  // n*h + y
  f32x4 acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float* row = cat + ny * w * (long)ld + c4 * 4;
  for (int x = 0; x < w; ++x) {
    f32x4 v = *(const f32x4*)(row + (long)x * ld);
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (i < wd.nwin && x >= wd.st[i] && x < wd.en[i]) acc[i] += v;
  }
  float* o = colsum + ny * (long)wd.nwin * C + c4 * 4;
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if (i < wd.nwin) *(f32x4*)(o + (long)i * C) = acc[i];
}

// pooled (bin-major, [sum_b N*b*b][C]) = ((sum over window rows of colsum) / kh) / kw
__global__ void ppm_pool_kernel(const float* __restrict__ colsum, int N, int h, int C, PPMWindows wr,
                                PPMWindows wc, int nbins, int b0, int b1, int b2, int b3,
                                float* __restrict__ pooled) {
  const int bins[4] = {b0, b1, b2, b3};
  int ncells = 0;
  for (int k = 0; k < nbins; ++k) ncells += bins[k] * bins[k];
  const int c4n = C >> 2;
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)N * ncells * c4n;
  if (idx >= total) return;
  int c4 = (int)(idx % c4n);
  int cell = (int)((idx / c4n) % ncells);
  int n = (int)(idx / ((long)c4n * ncells));
  int base = 0, woff = 0, k = 0;
  while (cell >= base + bins[k] * bins[k]) {
    base += bins[k] * bins[k];
    woff += bins[k];
    ++k;
  }
  const int b = bins[k];
  const int i = (cell - base) / b, j = (cell - base) % b;
  const int wrow = woff + i, wcol = woff + j;
  int ys = wr.st[wrow], ye = wr.en[wrow];
  int xs = wc.st[wcol], xe = wc.en[wcol];
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  for (int y = ys; y < ye; ++y)
    s += *(const f32x4*)(colsum + (((long)n * h + y) * wc.nwin + wcol) * C + c4 * 4);
  const float kh = (float)(ye - ys), kw = (float)(xe - xs);
  f32x4 r;
#pragma unroll
  for (int q = 0; q < 4; ++q) r[q] = (s[q] / kh) / kw;
  long out_row = (long)base * N + (long)n * b * b + i * b + j;
  *(f32x4*)(pooled + out_row * C + c4 * 4) = r;
}

int launch_ppm(const float* cat, int N, int h, int w, int ld, const int* bins, int nbins, float* colsum,
               float* pooled, hipStream_t st) {
  if (nbins != 4) return fail(CWT_EARG, "PPM expects 4 bins");
  PPMWindows wc = make_windows(w, bins, nbins);
  PPMWindows wr = make_windows(h, bins, nbins);
  if (wc.nwin > 16) return fail(CWT_EARG, "PPM: too many windows");
  const int C = 2048;
  int ncells = 0;
  for (int b = 0; b < nbins; ++b) ncells += bins[b] * bins[b];
  long t1 = (long)N * h * (C / 4);
  hipLaunchKernelGGL(ppm_colsum_kernel, dim3(cdiv(t1, 256)), dim3(256), 0, st, cat, N, h, w, ld, C, wc, colsum);
  CWT_LAUNCH_CHECK();
  long t2 = (long)N * ncells * (C / 4);
  hipLaunchKernelGGL(ppm_pool_kernel, dim3(cdiv(t2, 256)), dim3(256), 0, st, colsum, N, h, C, wr, wc, nbins,
                     bins[0], bins[1], bins[2], bins[3], pooled);
  CWT_LAUNCH_CHECK();
  return 0;
}

// cat[n][y][x][off + bin*red + c] = bilinear(ppm_out_bin[n][b][b][red]) (align_corners=True)
__global__ void ppm_upsample_kernel(const float* __restrict__ ppm_out, int N, int h, int w, int nbins,
                                    int b0, int b1, int b2, int b3, int red, float* __restrict__ cat, int ld,
                                    int off) {
  const int c4n = nbins * red / 4;
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)N * h * w * c4n;
  if (idx >= total) return;
  int c4 = (int)(idx % c4n);
  long pix = idx / c4n;
  int x = (int)(pix % w);
  int y = (int)((pix / w) % h);
  int n = (int)(pix / ((long)w * h));
  int bin = (c4 * 4) / red;
  int c = c4 * 4 - bin * red;
  int bins[4] = {b0, b1, b2, b3};
  int base = 0;
  for (int k = 0; k < bin; ++k) base += bins[k] * bins[k];
  int b = bins[bin];
  const float sy = (h > 1) ? (float)(b - 1) / (float)(h - 1) : 0.f;
  const float sx = (w > 1) ? (float)(b - 1) / (float)(w - 1) : 0.f;
  Lerp ly = lerp_coord(y, b, sy), lx = lerp_coord(x, b, sx);
  const float* src = ppm_out + ((long)base * N + (long)n * b * b) * red + c;
  f32x4 v00 = *(const f32x4*)(src + ((long)ly.i0 * b + lx.i0) * red);
  f32x4 v01 = *(const f32x4*)(src + ((long)ly.i0 * b + lx.i1) * red);
  f32x4 v10 = *(const f32x4*)(src + ((long)ly.i1 * b + lx.i0) * red);
  f32x4 v11 = *(const f32x4*)(src + ((long)ly.i1 * b + lx.i1) * red);
  f32x4 r;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    r[q] = ly.l0 * (lx.l0 * v00[q] + lx.l1 * v01[q]) + ly.l1 * (lx.l0 * v10[q] + lx.l1 * v11[q]);
  *(f32x4*)(cat + pix * ld + off + bin * red + c) = r;
}

int launch_ppm_upsample(const float* ppm_out, int N, int h, int w, const int* bins, int nbins, int red, float* cat,
                        int ld, int off, hipStream_t st) {
  if (nbins != 4) return fail(CWT_EARG, "PPM expects 4 bins");
  long total = (long)N * h * w * (nbins * red / 4);
  hipLaunchKernelGGL(ppm_upsample_kernel, dim3(cdiv(total, 256)), dim3(256), 0, st, ppm_out, N, h, w, nbins,
                     bins[0], bins[1], bins[2], bins[3], red, cat, ld, off);
  CWT_LAUNCH_CHECK();
  return 0;
}

}  // namespace cwt

// Stage-1 pretraining (reference src/pretrain.py:104-121,163-219): the kernels of one SGD step
// of the whole PSPNet (every conv, BN, the PPM branch, the bottleneck and the 1x1 classifier)
// that the frozen-extractor path does not have: conv weight gradients, training-mode BN
// forward with saved statistics and its backward, max-pool / adaptive-pool / bilinear adjoints,
// the label-smoothed CE of the upsampled logits with its gradient, and a strided fp32 GEMM for
// the few-row products (PPM cells, classifier).  Conv forward and input gradients reuse the
// exact-fp32 implicit-GEMM conv (conv.hip): the input gradient of a conv is a conv of the output
// gradient with the transposed, tap-flipped weights (stride-2 convs: of the zero-interleaved
// output gradient).  Everything is fp32 (training-mode BN amplifies rounding: DESIGN.md A11).
#include <algorithm>

#include "common.h"
#include "kernels.h"
#include "pretrain.h"

namespace cwt {

// ------------------------------------------------------------------------------------------
// Conv weight gradient on the exact f32 matrix cores (v_mfma_f32_32x32x2_f32):
//   gw[co][kk] = sum_m dy[m][co] * X(m, kk),   kk = packed_k(ci, tap) (conv.hip's K order)
// a GEMM (Co x K) reduced over the output pixels m.  Workgroup tile BM (co) x BN (kk), 4 waves
// 2 x 2; the pixel range of split blockIdx.z is walked 32 pixels at a time: dy rows and the
// gathered input rows (BN/32 (channel block, tap) groups of 32 channels) go to LDS row-major
// (one row per pixel), register prefetch two chunks ahead during the MFMAs.  The lane
// operands are single floats (A[co][pixel], B[pixel][kk] of a 2-pixel k-step), read
// conflict-free from consecutive LDS words.  Output: the split's slab [Co][K] (summed in fixed
// order by wgrad_reduce_kernel: deterministic) or gw itself when there is one split.
// ------------------------------------------------------------------------------------------
template <int BM, int BN>
__global__ __launch_bounds__(256, 2) void conv_wgrad_f32(WgradArgs a) {
  constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 32, TN = WN / 32;
  constexpr int A_LD = BM / 32, B_LD = BN / 32;  // float4 per thread per 32-pixel chunk
  __shared__ float sA[2][32][BM];
  __shared__ float sB[2][32][BN];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int wm = wv >> 1, wn = wv & 1;
  const int co0 = blockIdx.x * BM, k0 = blockIdx.y * BN;
  const int split = blockIdx.z;
  const long m_begin = (long)split * a.chunks_per_split * 32;
  const long m_end = std::min<long>(a.M, m_begin + (long)a.chunks_per_split * 32);
  const int taps = a.kh * a.kw;
  const int HoWo = a.Ho * a.Wo;

  // per-thread gather geometry: the (channel block, tap) of each B group is fixed for the
  // workgroup; the pixel of each loaded row advances by 32 per chunk (no divisions in the loop)
  int b_coff[B_LD], b_dy[B_LD], b_dx[B_LD], b_n[B_LD], b_oh[B_LD], b_ow[B_LD];
#pragma unroll
  for (int j = 0; j < B_LD; ++j) {
    const int idx = t + 256 * j;
    const int row = idx / (BN / 4), rem = idx % (BN / 4);
    const int grp = rem >> 3, c4 = rem & 7;
    const int ks = k0 / 32 + grp;
    const int cb = ks / taps, tap = ks - cb * taps;
    const int ky = tap / a.kw, kx = tap - ky * a.kw;
    b_coff[j] = cb * 32 + 4 * c4;
    b_dy[j] = ky * a.dil - a.pad;
    b_dx[j] = kx * a.dil - a.pad;
    const long m = m_begin + row;
    const int n = (int)(m / HoWo), rr = (int)(m - (long)n * HoWo);
    b_n[j] = n;
    b_oh[j] = rr / a.Wo;
    b_ow[j] = rr - b_oh[j] * a.Wo;
  }
  // two register sets: the chunk two ahead is in flight while one chunk is in the MFMAs
  f32x4 ra[A_LD], rb[B_LD], ra2[A_LD], rb2[B_LD];
  // mc = the chunk's first pixel; loads happen in chunk order, B geometry is at mc
  auto load_chunk = [&](long mc, f32x4(&A)[A_LD], f32x4(&B)[B_LD]) {
#pragma unroll
    for (int j = 0; j < A_LD; ++j) {
      const int idx = t + 256 * j;
      const int row = idx / (BM / 4), c4 = idx % (BM / 4);
      const long m = mc + row;
      A[j] = (m < m_end) ? *(const f32x4*)(a.dy + m * a.dy_ld + co0 + 4 * c4) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int j = 0; j < B_LD; ++j) {
      const int idx = t + 256 * j;
      const int row = idx / (BN / 4);
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (mc + row < m_end) {
        const int ih = b_oh[j] * a.stride + b_dy[j], iw = b_ow[j] * a.stride + b_dx[j];
        if ((unsigned)ih < (unsigned)a.Hi && (unsigned)iw < (unsigned)a.Wi)
          v = *(const f32x4*)(a.x + ((long)(b_n[j] * a.Hi + ih) * a.Wi + iw) * a.x_ld + b_coff[j]);
      }
      B[j] = v;
    }
  };
  auto advance_chunk = [&]() {  // every loaded row's pixel += 32
#pragma unroll
    for (int j = 0; j < B_LD; ++j) {
      b_ow[j] += 32;
      while (b_ow[j] >= a.Wo) {
        b_ow[j] -= a.Wo;
        if (++b_oh[j] == a.Ho) {
          b_oh[j] = 0;
          ++b_n[j];
        }
      }
    }
  };
  auto store_chunk = [&](int buf, const f32x4(&A)[A_LD], const f32x4(&B)[B_LD]) {
#pragma unroll
    for (int j = 0; j < A_LD; ++j) {
      const int idx = t + 256 * j;
      *(f32x4*)&sA[buf][idx / (BM / 4)][4 * (idx % (BM / 4))] = A[j];
    }
#pragma unroll
    for (int j = 0; j < B_LD; ++j) {
      const int idx = t + 256 * j;
      *(f32x4*)&sB[buf][idx / (BN / 4)][4 * (idx % (BN / 4))] = B[j];
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int h = lane >> 5, l31 = lane & 31;
  auto compute = [&](int cur) {
#pragma unroll 4
    for (int s = 0; s < 16; ++s) {
      float av[TM], bv[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) av[i] = sA[cur][2 * s + h][wm * WM + i * 32 + l31];
#pragma unroll
      for (int j = 0; j < TN; ++j) bv[j] = sB[cur][2 * s + h][wn * WN + j * 32 + l31];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
  };
  if (m_begin < m_end) {
    load_chunk(m_begin, ra, rb);
    store_chunk(0, ra, rb);
    if (m_begin + 32 < m_end) {
      advance_chunk();
      load_chunk(m_begin + 32, ra, rb);
    }
    __syncthreads();
    int cur = 0;
    long mc = m_begin;
    // invariant at the top of each half: LDS[cur] holds chunk mc, one register set chunk mc+32
    while (true) {
      if (mc + 64 < m_end) {
        advance_chunk();
        load_chunk(mc + 64, ra2, rb2);
      }
      compute(cur);
      if (mc + 32 < m_end) store_chunk(cur ^ 1, ra, rb);
      __syncthreads();
      cur ^= 1;
      mc += 32;
      if (mc >= m_end) break;
      if (mc + 64 < m_end) {
        advance_chunk();
        load_chunk(mc + 64, ra, rb);
      }
      compute(cur);
      if (mc + 32 < m_end) store_chunk(cur ^ 1, ra2, rb2);
      __syncthreads();
      cur ^= 1;
      mc += 32;
      if (mc >= m_end) break;
    }
  }
  float* out = a.out + (long)split * a.Co * a.K;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int kk = k0 + wn * WN + j * 32 + l31;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = co0 + wm * WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        out[(long)co * a.K + kk] = acc[i][j][r];
      }
    }
}

// dst[i] = sum_s slab[s][i] in split order (deterministic); f32x4 per thread
__global__ void slab_reduce_kernel(const float* __restrict__ slabs, int nsplit, long n4, float* __restrict__ dst) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  const f32x4* s = (const f32x4*)slabs;
  f32x4 v = s[i];
  for (int k = 1; k < nsplit; ++k) v += s[(long)k * n4 + i];
  ((f32x4*)dst)[i] = v;
}

int launch_slab_reduce(const float* slabs, int nsplit, long n, float* dst, hipStream_t st) {
  if (n % 4) return fail(CWT_EARG, "slab_reduce: n % 4 != 0");
  hipLaunchKernelGGL(slab_reduce_kernel, dim3(cdiv(n / 4, 256)), dim3(256), 0, st, slabs, nsplit, n / 4, dst);
  CWT_LAUNCH_CHECK();
  return 0;
}

// Split of the pixel reduction: enough workgroups to cover the CUs a few times, >= 8 chunks
// (256 pixels) per split, slabs within the workspace.
int wgrad_splits(long M, int Co, int K, int bm, int bn, size_t ws_floats) {
  const long tiles = (long)(Co / bm) * (K / bn);
  const long chunks = (M + 31) / 32;
  int ns = 1;
  while (tiles * ns < 1024 && chunks / (ns * 2) >= 8 && (size_t)(ns * 2) * Co * K <= ws_floats) ns *= 2;
  return ns;
}

int launch_conv_wgrad(WgradArgs a, float* gw, float* ws, size_t ws_floats, hipStream_t st) {
  if (a.Co % 64 || a.K % 64 || a.x_ld % 4 || a.dy_ld % 4 || (a.K / (a.kh * a.kw)) % 32)
    return fail(CWT_EARG, "conv_wgrad: Co, K multiples of 64, Ci of 32, 16-B rows required");
  const int bm = (a.Co % 128 == 0) ? 128 : 64;
  const int bn = (a.K % 128 == 0 && a.Co >= 128) ? 128 : 64;
  const int ns = wgrad_splits(a.M, a.Co, a.K, bm, bn, ws_floats);
  const long chunks = (a.M + 31) / 32;
  a.chunks_per_split = (int)((chunks + ns - 1) / ns);
  const int nsplit = (int)((chunks + a.chunks_per_split - 1) / a.chunks_per_split);
  a.out = nsplit > 1 ? ws : gw;
  dim3 grid(a.Co / bm, a.K / bn, nsplit);
  if (bm == 128 && bn == 128)
    hipLaunchKernelGGL((conv_wgrad_f32<128, 128>), grid, dim3(256), 0, st, a);
  else if (bm == 128)
    hipLaunchKernelGGL((conv_wgrad_f32<128, 64>), grid, dim3(256), 0, st, a);
  else if (bn == 128)
    hipLaunchKernelGGL((conv_wgrad_f32<64, 128>), grid, dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((conv_wgrad_f32<64, 64>), grid, dim3(256), 0, st, a);
  CWT_LAUNCH_CHECK();
  if (nsplit > 1) return launch_slab_reduce(ws, nsplit, (long)a.Co * a.K, gw, st);
  return 0;
}

// Input-gradient weights of a conv: wt[ci][packed_k(co, taps-1-tap)] = w[co][packed_k(ci, tap)]
// (transposed channels, flipped taps: the input gradient is a conv of dy with them).
__global__ void wt_transpose_kernel(const float* __restrict__ w, float* __restrict__ wt, int Co, int Ci, int taps) {
  const long n = (long)Co * Ci * taps;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int ci = (int)(i % Ci);
    const long r = i / Ci;
    const int tap = (int)(r % taps);
    const int co = (int)(r / taps);
    wt[(long)ci * Co * taps + packed_k(co, taps - 1 - tap, taps)] = w[(long)co * Ci * taps + packed_k(ci, tap, taps)];
  }
}

int launch_wt_transpose(const float* w, float* wt, int Co, int Ci, int taps, hipStream_t st) {
  const long n = (long)Co * Ci * taps;
  hipLaunchKernelGGL(wt_transpose_kernel, dim3((unsigned)std::min<long>(8192, cdiv(n, 256))), dim3(256), 0, st, w, wt,
                     Co, Ci, taps);
  CWT_LAUNCH_CHECK();
  return 0;
}

// Zero-interleave of a stride-2 conv's output gradient: z[n][2i][2j][c] = dy[n][i][j][c], zeros
// elsewhere (z is Hi x Wi); the input gradient is then a stride-1 conv of z.
__global__ void zero_insert_kernel(const float* __restrict__ dy, int N, int Ho, int Wo, int C, float* __restrict__ z,
                                   int Hi, int Wi) {
  const long total = (long)N * Hi * Wi * (C / 4);
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c4 = (int)(i % (C / 4));
  const long p = i / (C / 4);
  const int x = (int)(p % Wi), y = (int)((p / Wi) % Hi), n = (int)(p / ((long)Wi * Hi));
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
  if (!(y & 1) && !(x & 1) && (y >> 1) < Ho && (x >> 1) < Wo)
    v = *(const f32x4*)(dy + (((long)n * Ho + (y >> 1)) * Wo + (x >> 1)) * C + 4 * c4);
  *(f32x4*)(z + p * C + 4 * c4) = v;
}

int launch_zero_insert(const float* dy, int N, int Ho, int Wo, int C, float* z, int Hi, int Wi, hipStream_t st) {
  const long total = (long)N * Hi * Wi * (C / 4);
  hipLaunchKernelGGL(zero_insert_kernel, dim3(cdiv(total, 256)), dim3(256), 0, st, dy, N, Ho, Wo, C, z, Hi, Wi);
  CWT_LAUNCH_CHECK();
  return 0;
}

// Stem conv1 (3 -> 64, 3x3 s2 p1 over the NCHW image) weight gradient, weights laid out
// [ci*9 + tap][co] as launch_stem_conv1 reads them.  Block b sums pixels [b*P, (b+1)*P) into a
// slab of 27 x 64: 64-pixel tiles of dy and of the 27-tap patches staged in LDS.
constexpr int kStemPix = 64;
__global__ __launch_bounds__(256) void stem1_wgrad_kernel(const float* __restrict__ img, int N, int S,
                                                          const float* __restrict__ dy, int Ho, long pix_per_blk,
                                                          float* __restrict__ slabs) {
  __shared__ float sd[kStemPix][64];
  __shared__ float sp[kStemPix][28];
  const int t = threadIdx.x;
  const long M = (long)N * Ho * Ho;
  const long p0 = (long)blockIdx.x * pix_per_blk, p1 = std::min(M, p0 + pix_per_blk);
  float acc[7];
#pragma unroll
  for (int q = 0; q < 7; ++q) acc[q] = 0.f;
  for (long pc = p0; pc < p1; pc += kStemPix) {
    for (int i = t; i < kStemPix * 16; i += 256) {
      const int r = i >> 4, c4 = i & 15;
      const long m = pc + r;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (m < p1) v = *(const f32x4*)(dy + m * 64 + 4 * c4);
      *(f32x4*)&sd[r][4 * c4] = v;
    }
    for (int i = t; i < kStemPix * 27; i += 256) {
      const int r = i / 27, k = i - r * 27;
      const long m = pc + r;
      float v = 0.f;
      if (m < p1) {
        const int n = (int)(m / ((long)Ho * Ho)), rr = (int)(m - (long)n * Ho * Ho);
        const int oh = rr / Ho, ow = rr - oh * Ho;
        const int ci = k / 9, tap = k - ci * 9;
        const int ih = 2 * oh - 1 + tap / 3, iw = 2 * ow - 1 + tap % 3;
        if ((unsigned)ih < (unsigned)S && (unsigned)iw < (unsigned)S) v = img[(((long)n * 3 + ci) * S + ih) * S + iw];
      }
      sp[r][k] = v;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 7; ++q) {
      const int o = t + 256 * q;
      if (o < 27 * 64) {
        const int k = o >> 6, co = o & 63;
        float s = acc[q];
        for (int r = 0; r < kStemPix; ++r) s = fmaf(sd[r][co], sp[r][k], s);
        acc[q] = s;
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int q = 0; q < 7; ++q) {
    const int o = t + 256 * q;
    if (o < 27 * 64) slabs[(long)blockIdx.x * 27 * 64 + o] = acc[q];
  }
}

int launch_stem1_wgrad(const float* img, int N, int S, const float* dy, int Ho, float* gw, float* ws, size_t ws_floats,
                       hipStream_t st) {
  const long M = (long)N * Ho * Ho;
  int nblk = (int)std::min<long>(512, cdiv(M, 4 * kStemPix));
  while ((size_t)nblk * 27 * 64 > ws_floats && nblk > 1) nblk /= 2;
  const long per = ((M + nblk - 1) / nblk + kStemPix - 1) / kStemPix * kStemPix;
  nblk = (int)((M + per - 1) / per);
  hipLaunchKernelGGL(stem1_wgrad_kernel, dim3(nblk), dim3(256), 0, st, img, N, S, dy, Ho, per, ws);
  CWT_LAUNCH_CHECK();
  return launch_slab_reduce(ws, nblk, 27L * 64, gw, st);
}

// ------------------------------------------------------------------------------------------
// Training-mode BatchNorm with saved statistics (forward) and its backward.
//   forward: Welford partials per (256-row block, channel) -> per channel (Chan merge in
//            double) mean, 1/sqrt(var_b + eps), running statistics moved by `momentum`
//            (unbiased variance) -- nn.BatchNorm2d training=True; eval mode takes the running
//            statistics instead -- then out = [relu](g * (y - mu) * istd + b [+ res]) [* drop].
//   backward (torch's batch_norm_backward, training): with g the gradient at the BN output,
//            dgamma = sum g * xhat, dbeta = sum g,
//            dy = gamma * istd * (g - dbeta / M - xhat * dgamma / M).
// ------------------------------------------------------------------------------------------
// Row blocking of the per-channel reductions: at most kBnBlocks blocks of >= 256 rows (the
// per-channel merge over the blocks then stays short), 4 row groups x 64 channels per block.
constexpr int kBnBlocks = 256;
static inline int bn_nblk(long M) { return (int)std::min<long>(kBnBlocks, cdiv(M, 256L)); }
static inline long bn_rows_per_blk(long M) { return ((M + bn_nblk(M) - 1) / bn_nblk(M) + 3) & ~3L; }

// per (row block, channel): n, mean, M2 from shifted sums (shift = the thread's first value, no
// per-element division), the 4 row groups merged by Chan's formula
__global__ __launch_bounds__(256) void ptbn_stats_kernel(const float* __restrict__ y, int ld, long M, int C, long rpb,
                                                         float* __restrict__ part) {
  __shared__ float sn[4][64], sm[4][64], sq[4][64];
  const int lane = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + lane;
  const long r0 = (long)blockIdx.x * rpb, r1 = std::min(M, r0 + rpb);
  float n = 0.f, mean = 0.f, m2 = 0.f;
  if (c < C && r0 + rg < r1) {
    const float K = y[(r0 + rg) * ld + c];
    float s1 = 0.f, s2 = 0.f;
    int k = 0;
#pragma unroll 4
    for (long r = r0 + rg; r < r1; r += 4) {
      const float d = y[r * ld + c] - K;
      s1 += d;
      s2 = fmaf(d, d, s2);
      ++k;
    }
    n = (float)k;
    mean = K + s1 / n;
    m2 = fmaxf(s2 - s1 * (s1 / n), 0.f);
  }
  sn[rg][lane] = n;
  sm[rg][lane] = mean;
  sq[rg][lane] = m2;
  __syncthreads();
  if (rg == 0 && c < C) {
    for (int g = 1; g < 4; ++g) {
      const float nb = sn[g][lane];
      if (nb == 0.f) continue;
      const float nt = n + nb, d = sm[g][lane] - mean;
      mean += d * (nb / nt);
      m2 += sq[g][lane] + d * d * (n * nb / nt);
      n = nt;
    }
    const long plane = (long)gridDim.x * C, o = (long)blockIdx.x * C + c;
    part[o] = n;
    part[plane + o] = mean;
    part[2 * plane + o] = m2;
  }
}

// stats[0..C) mean, [C..2C) 1/sqrt(var + eps) of the batch (train) or of the running statistics (eval).
// 256 threads per 64 channels: row group g merges the partials of blocks b = g (mod 4) (loads in
// batches of 8), then the 4 group results are merged in group order (Chan, double).
__global__ __launch_bounds__(256) void ptbn_finalize_kernel(const float* __restrict__ part, int nblk, int C,
                                                            float* __restrict__ run, float eps, float momentum,
                                                            int train, float* __restrict__ stats) {
  __shared__ double sn[4][64], sm[4][64], sq[4][64];
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  if (!train) {
    if (g == 0 && c < C) {
      stats[c] = run[c];
      stats[C + c] = 1.0f / sqrtf(run[C + c] + eps);
    }
    return;
  }
  const long plane = (long)nblk * C;
  double n = 0.0, mean = 0.0, m2 = 0.0;
  if (c < C) {
    for (int b0 = g; b0 < nblk; b0 += 32) {
      float pn[8], pm[8], pq[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int b = b0 + 4 * k;
        const long o = (long)min(b, nblk - 1) * C + c;
        pn[k] = b < nblk ? part[o] : 0.f;
        pm[k] = part[plane + o];
        pq[k] = part[2 * plane + o];
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const double nb = pn[k];
        if (nb == 0.0) continue;
        const double nt = n + nb, d = (double)pm[k] - mean;
        mean += d * (nb / nt);
        m2 += (double)pq[k] + d * d * (n * nb / nt);
        n = nt;
      }
    }
  }
  sn[g][lane] = n;
  sm[g][lane] = mean;
  sq[g][lane] = m2;
  __syncthreads();
  if (g != 0 || c >= C) return;
  for (int k = 1; k < 4; ++k) {
    const double nb = sn[k][lane];
    if (nb == 0.0) continue;
    const double nt = n + nb, d = sm[k][lane] - mean;
    mean += d * (nb / nt);
    m2 += sq[k][lane] + d * d * (n * nb / nt);
    n = nt;
  }
  const float mu = (float)mean, var_b = (float)(m2 / n);
  stats[c] = mu;
  stats[C + c] = 1.0f / sqrtf(var_b + eps);
  run[c] = (1.f - momentum) * run[c] + momentum * mu;
  run[C + c] = (1.f - momentum) * run[C + c] + momentum * (float)(m2 / (n - 1.0));
}

// out = [relu](gamma (y - mu) istd + beta [+ res]) (the residual itself a raw conv output under
// its own BN when res_stats != null); drop_p > 0: Dropout2d (image, channel) mask after the ReLU,
// the pre-dropout value kept in out_pre (the ReLU mask of the backward).  4 channels per thread.
__global__ __launch_bounds__(256) void ptbn_apply_kernel(PtBnApply a) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int cg = a.C >> 2;
  if (idx >= a.M * cg) return;
  const long row = idx / cg;
  const int c0 = (int)(idx - row * cg) * 4;
  const f32x4 y = *(const f32x4*)(a.y + row * a.y_ld + c0);
  f32x4 r = {0.f, 0.f, 0.f, 0.f};
  if (a.res) r = *(const f32x4*)(a.res + row * a.res_ld + c0);
  const long img = row / a.rows_per_image;
  f32x4 o, pre;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = c0 + q;
    float v = fmaf(a.gamma[c], (y[q] - a.stats[c]) * a.stats[a.C + c], a.beta[c]);
    if (a.res) {
      float rv = r[q];
      if (a.res_stats) rv = fmaf(a.res_gamma[c], (rv - a.res_stats[c]) * a.res_stats[a.C + c], a.res_beta[c]);
      v += rv;
    }
    if (a.relu) v = fmaxf(v, 0.f);
    pre[q] = v;
    if (a.drop_p > 0.f) v *= dropout_scale(a.drop_p, a.seed, 3, (unsigned long long)img * a.C + c);
    o[q] = v;
  }
  *(f32x4*)(a.out + row * a.out_ld + c0) = o;
  if (a.out_pre) *(f32x4*)(a.out_pre + row * a.out_ld + c0) = pre;
}

// ReLU mask of a BN without residual, recomputed from its raw input exactly as ptbn_apply_kernel
// evaluated it (the same expression: the same float result)
__device__ __forceinline__ bool ptbn_relu_on(const PtBnBwd& a, float y, float mu, float is, int c) {
  return fmaf(a.gamma[c], (y - mu) * is, a.beta[c]) > 0.f;
}

// Gradient at the BN output: g = dout [* drop mask] [* (act > 0)]
__device__ __forceinline__ float ptbn_grad_at(const PtBnBwd& a, long row, int c, float y, float mu, float is) {
  float g = a.dout[row * a.dout_ld + c];
  if (a.drop_p > 0.f) g *= dropout_scale(a.drop_p, a.seed, 3, (unsigned long long)(row / a.rows_per_image) * a.C + c);
  if (a.act ? !(a.act[row * a.act_ld + c] > 0.f) : (a.relu_from_y && !ptbn_relu_on(a, y, mu, is, c))) g = 0.f;
  return g;
}

// per (row block, channel) partial sums of g and g * xhat (fixed order)
__global__ __launch_bounds__(256) void ptbn_bwd_stats_kernel(PtBnBwd a, long rpb, float* __restrict__ part) {
  __shared__ float s1[4][64], s2[4][64];
  const int lane = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + lane;
  const long r0 = (long)blockIdx.x * rpb, r1 = std::min(a.M, r0 + rpb);
  float sg = 0.f, sgx = 0.f;
  if (c < a.C) {
    const float mu = a.stats[c], is = a.stats[a.C + c];
#pragma unroll 4
    for (long r = r0 + rg; r < r1; r += 4) {
      const float yv = a.y[r * a.y_ld + c];
      const float g = ptbn_grad_at(a, r, c, yv, mu, is);
      sg += g;
      sgx = fmaf(g, (yv - mu) * is, sgx);
    }
  }
  s1[rg][lane] = sg;
  s2[rg][lane] = sgx;
  __syncthreads();
  if (rg == 0 && c < a.C) {
    sg = ((s1[0][lane] + s1[1][lane]) + s1[2][lane]) + s1[3][lane];
    sgx = ((s2[0][lane] + s2[1][lane]) + s2[2][lane]) + s2[3][lane];
    const long plane = (long)gridDim.x * a.C, o = (long)blockIdx.x * a.C + c;
    part[o] = sg;
    part[plane + o] = sgx;
  }
}

// dbeta, dgamma (written to the parameter gradients) summed over the blocks in double: 4 row
// groups of 64 channels each sum the blocks b = g (mod 4), then the groups in order
__global__ __launch_bounds__(256) void ptbn_bwd_finalize_kernel(const float* __restrict__ part, int nblk, int C,
                                                                float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                                float* __restrict__ sums) {
  __shared__ double s1[4][64], s2[4][64];
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const long plane = (long)nblk * C;
  double sg = 0.0, sgx = 0.0;
  if (c < C) {
    for (int b0 = g; b0 < nblk; b0 += 32) {
      float p1[8], p2[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int b = b0 + 4 * k;
        const long o = (long)min(b, nblk - 1) * C + c;
        p1[k] = b < nblk ? part[o] : 0.f;
        p2[k] = b < nblk ? part[plane + o] : 0.f;
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        sg += p1[k];
        sgx += p2[k];
      }
    }
  }
  s1[g][lane] = sg;
  s2[g][lane] = sgx;
  __syncthreads();
  if (g != 0 || c >= C) return;
  sg = ((s1[0][lane] + s1[1][lane]) + s1[2][lane]) + s1[3][lane];
  sgx = ((s2[0][lane] + s2[1][lane]) + s2[2][lane]) + s2[3][lane];
  dbeta[c] = (float)sg;
  dgamma[c] = (float)sgx;
  sums[c] = (float)sg;
  sums[C + c] = (float)sgx;
}

// dy = gamma istd (g - sum_g / M - xhat sum_gx / M); optionally g itself into g_out (the
// gradient of an identity residual).  4 channels per thread.
__global__ __launch_bounds__(256) void ptbn_bwd_apply_kernel(PtBnBwd a, const float* __restrict__ sums) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int cg = a.C >> 2;
  if (idx >= a.M * cg) return;
  const long row = idx / cg;
  const int c0 = (int)(idx - row * cg) * 4;
  f32x4 g = *(const f32x4*)(a.dout + row * a.dout_ld + c0);
  const f32x4 y = *(const f32x4*)(a.y + row * a.y_ld + c0);
  f32x4 act = {1.f, 1.f, 1.f, 1.f};
  if (a.act) act = *(const f32x4*)(a.act + row * a.act_ld + c0);
  const float inv_m = 1.0f / (float)a.M;
  const long img = row / a.rows_per_image;
  f32x4 dy;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = c0 + q;
    const float mu = a.stats[c], is = a.stats[a.C + c];
    if (a.drop_p > 0.f) g[q] *= dropout_scale(a.drop_p, a.seed, 3, (unsigned long long)img * a.C + c);
    if (a.act ? !(act[q] > 0.f) : (a.relu_from_y && !ptbn_relu_on(a, y[q], mu, is, c))) g[q] = 0.f;
    const float xh = (y[q] - mu) * is;
    dy[q] = a.gamma[c] * is * (g[q] - sums[c] * inv_m - xh * (sums[a.C + c] * inv_m));
  }
  *(f32x4*)(a.dy + row * a.dy_ld + c0) = dy;
  if (a.g_out) *(f32x4*)(a.g_out + row * a.g_ld + c0) = g;
}

size_t ptbn_part_floats(long M, int C) { return (size_t)3 * bn_nblk(M) * C; }

int launch_ptbn_fwd(const float* y, int ld, long M, int C, float* run, float eps, float momentum, int train,
                    float* stats, float* part, size_t part_floats, hipStream_t st) {
  if (train && M < 2) return fail(CWT_EARG, "Expected more than 1 value per channel when training (BatchNorm2d)");
  const int nblk = bn_nblk(M);
  if (train) {
    if (ptbn_part_floats(M, C) > part_floats) return fail(CWT_ESTATE, "ptbn: partial workspace too small");
    hipLaunchKernelGGL(ptbn_stats_kernel, dim3(nblk, cdiv(C, 64)), dim3(256), 0, st, y, ld, M, C, bn_rows_per_blk(M),
                       part);
    CWT_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(ptbn_finalize_kernel, dim3(cdiv(C, 64)), dim3(256), 0, st, (const float*)part, nblk, C, run, eps,
                     momentum, train, stats);
  CWT_LAUNCH_CHECK();
  return 0;
}

int launch_ptbn_apply(const PtBnApply& a, hipStream_t st) {
  if (a.C % 4 || a.y_ld % 4 || a.out_ld % 4 || (a.res && a.res_ld % 4)) return fail(CWT_EARG, "ptbn_apply: alignment");
  const long total = a.M * (a.C / 4);
  hipLaunchKernelGGL(ptbn_apply_kernel, dim3(cdiv(total, 256)), dim3(256), 0, st, a);
  CWT_LAUNCH_CHECK();
  return 0;
}

int launch_ptbn_bwd(const PtBnBwd& a, float* dgamma, float* dbeta, float* part, size_t part_floats, float* sums,
                    hipStream_t st) {
  if (a.C % 4 || a.dout_ld % 4 || a.y_ld % 4 || a.dy_ld % 4 || (a.act && a.act_ld % 4) || (a.g_out && a.g_ld % 4))
    return fail(CWT_EARG, "ptbn_bwd: alignment");
  const int nblk = bn_nblk(a.M);
  if ((size_t)2 * nblk * a.C > part_floats) return fail(CWT_ESTATE, "ptbn_bwd: partial workspace too small");
  hipLaunchKernelGGL(ptbn_bwd_stats_kernel, dim3(nblk, cdiv(a.C, 64)), dim3(256), 0, st, a, bn_rows_per_blk(a.M), part);
  CWT_LAUNCH_CHECK();
  hipLaunchKernelGGL(ptbn_bwd_finalize_kernel, dim3(cdiv(a.C, 64)), dim3(256), 0, st, (const float*)part, nblk, a.C,
                     dgamma, dbeta, sums);
  CWT_LAUNCH_CHECK();
  const long total = a.M * (a.C / 4);
  hipLaunchKernelGGL(ptbn_bwd_apply_kernel, dim3(cdiv(total, 256)), dim3(256), 0, st, a, (const float*)sums);
  CWT_LAUNCH_CHECK();
  return 0;
}

// ------------------------------------------------------------------------------------------
// Max pool 3x3 s2 p1 with the window argmax (0..8, first maximum in scan order as PyTorch's CPU
// kernel), and its adjoint in gather form: input pixel (y, x) sums the gradients of the <= 4
// windows whose argmax it is (deterministic, no atomics).
// ------------------------------------------------------------------------------------------
__global__ void maxpool_idx_kernel(const float* __restrict__ in, int N, int H, int C, float* __restrict__ out,
                                   uint8_t* __restrict__ idx, int Ho) {
  const long total = (long)N * Ho * Ho * C;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c = (int)(i % C);
  const long p = i / C;
  const int ox = (int)(p % Ho), oy = (int)((p / Ho) % Ho), n = (int)(p / ((long)Ho * Ho));
  float m = -INFINITY;
  int best = 0;
  for (int k = 0; k < 9; ++k) {
    const int y = 2 * oy - 1 + k / 3, x = 2 * ox - 1 + k % 3;
    if ((unsigned)y < (unsigned)H && (unsigned)x < (unsigned)H) {
      const float v = in[(((long)n * H + y) * H + x) * C + c];
      if (v > m || isnan(v)) {
        m = v;
        best = k;
      }
    }
  }
  out[i] = m;
  idx[i] = (uint8_t)best;
}

__global__ void maxpool_bwd_kernel(const float* __restrict__ dout, const uint8_t* __restrict__ idx, int N, int H, int C,
                                   int Ho, float* __restrict__ din) {
  const long total = (long)N * H * H * C;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c = (int)(i % C);
  const long p = i / C;
  const int x = (int)(p % H), y = (int)((p / H) % H), n = (int)(p / ((long)H * H));
  float s = 0.f;
  // windows oy with 2 oy - 1 <= y <= 2 oy + 1
  for (int oy = (y > 0 ? y : 1) / 2; oy <= std::min(Ho - 1, (y + 1) / 2); ++oy)
    for (int ox = (x > 0 ? x : 1) / 2; ox <= std::min(Ho - 1, (x + 1) / 2); ++ox) {
      const int k = (y - 2 * oy + 1) * 3 + (x - 2 * ox + 1);
      if (k < 0 || k > 8) continue;
      const long o = (((long)n * Ho + oy) * Ho + ox) * C + c;
      if (idx[o] == k) s += dout[o];
    }
  din[i] = s;
}

int launch_maxpool_idx(const float* in, int N, int H, int C, float* out, uint8_t* idx, int Ho, hipStream_t st) {
  const long total = (long)N * Ho * Ho * C;
  hipLaunchKernelGGL(maxpool_idx_kernel, dim3(cdiv(total, 256)), dim3(256), 0, st, in, N, H, C, out, idx, Ho);
  CWT_LAUNCH_CHECK();
  return 0;
}

int launch_maxpool_bwd(const float* dout, const uint8_t* idx, int N, int H, int C, int Ho, float* din, hipStream_t st) {
  const long total = (long)N * H * H * C;
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(cdiv(total, 256)), dim3(256), 0, st, dout, idx, N, H, C, Ho, din);
  CWT_LAUNCH_CHECK();
  return 0;
}

// ------------------------------------------------------------------------------------------
// PPM branch (pspnet.py:19-38) backward outside the folded field (backbone.hip):
//   adaptive-average-pool adjoint: dx[n][y][x][c] += sum over the bins' windows holding (y, x)
//             of dpooled / kh / kw (torch adaptive_avg_pool2d_backward), added in place
// ------------------------------------------------------------------------------------------
// pooled gradient rows bin-major as launch_ppm writes them: bin k's rows [base_k N, (base_k + b^2) N);
// 4 channels per thread, only the windows near (y, x) b / h per bin and axis visited
__global__ void avgpool_bwd_kernel(const float* __restrict__ dpool, int N, int h, int C, int b0, int b1, int b2, int b3,
                                   float* __restrict__ dx, int ld) {
  const int cg = C >> 2;
  const long total = (long)N * h * h * cg;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c0 = (int)(i % cg) * 4;
  const long p = i / cg;
  const int x = (int)(p % h), y = (int)((p / h) % h), n = (int)(p / ((long)h * h));
  const int bins[4] = {b0, b1, b2, b3};
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  int base = 0;
  for (int k = 0; k < 4; ++k) {
    const int b = bins[k];
    const int cy = (y * b) / h, cx = (x * b) / h;  // windows [floor(i h / b), ceil((i+1) h / b)) near y / b * h
    for (int ci = max(0, cy - 2); ci <= min(b - 1, cy + 2); ++ci) {
      const int ya = (ci * h) / b, yb = ((ci + 1) * h + b - 1) / b;
      if (y < ya || y >= yb) continue;
      for (int cj = max(0, cx - 2); cj <= min(b - 1, cx + 2); ++cj) {
        const int xa = (cj * h) / b, xb = ((cj + 1) * h + b - 1) / b;
        if (x < xa || x >= xb) continue;
        const f32x4 g = *(const f32x4*)(dpool + ((long)base * N + (long)n * b * b + ci * b + cj) * C + c0);
        const float kh = (float)(yb - ya), kw = (float)(xb - xa);
#pragma unroll
        for (int q = 0; q < 4; ++q) s[q] += g[q] / kh / kw;
      }
    }
    base += b * b;
  }
  f32x4* d = (f32x4*)(dx + p * ld + c0);
  *d = *d + s;
}

int launch_avgpool_bwd(const float* dpool, int N, int h, int C, const int* bins, float* dx, int ld, hipStream_t st) {
  if (C % 4 || ld % 4) return fail(CWT_EARG, "avgpool_bwd: alignment");
  const long total = (long)N * h * h * (C / 4);
  hipLaunchKernelGGL(avgpool_bwd_kernel, dim3(cdiv(total, 256)), dim3(256), 0, st, dpool, N, h, C, bins[0], bins[1],
                     bins[2], bins[3], dx, ld);
  CWT_LAUNCH_CHECK();
  return 0;
}

// ------------------------------------------------------------------------------------------
// Strided fp32 GEMM for the few-row products (PPM cells, the classifier):
//   C[i][j] (ldc) = sum_k A[i*sai + k*sak] * B[k*sbk + j*sbj]   (split-K over blockIdx.z into
// slabs summed in order by slab_reduce, or straight into C).  64 x 64 tile, 4 x 4 per thread.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void pt_gemm_kernel(PtGemm g) {
  __shared__ float As[16][64 + 4];
  __shared__ float Bs[16][64 + 4];
  const int t = threadIdx.x;
  const int i0 = blockIdx.x * 64, j0 = blockIdx.y * 64;
  const long kb = (long)blockIdx.z * g.k_per_split, ke = std::min<long>(g.K, kb + g.k_per_split);
  const int ti = t & 15, tj = t >> 4;
  float acc[4][4] = {};
  for (long k0 = kb; k0 < ke; k0 += 16) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = t + 256 * q;
      const int r = e & 63, kk = e >> 6;
      const long k = k0 + kk;
      const int i = i0 + r, j = j0 + r;
      As[kk][r] = (i < g.M && k < ke) ? g.A[(long)i * g.sai + k * g.sak] : 0.f;
      Bs[kk][r] = (j < g.N && k < ke) ? g.B[k * g.sbk + (long)j * g.sbj] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      float av[4], bv[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        av[q] = As[kk][ti * 4 + q];
        bv[q] = Bs[kk][tj * 4 + q];
      }
#pragma unroll
      for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[p][q] = fmaf(av[p], bv[q], acc[p][q]);
    }
    __syncthreads();
  }
  float* out = g.slab ? g.slab + (long)blockIdx.z * g.M * g.N : g.C;
  const long ld = g.slab ? g.N : g.ldc;
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = i0 + ti * 4 + p, j = j0 + tj * 4 + q;
      if (i < g.M && j < g.N) out[(long)i * ld + j] = acc[p][q];
    }
}

__global__ void slab_reduce_2d_kernel(const float* __restrict__ slabs, int nsplit, int M, int N, float* __restrict__ C,
                                      long ldc) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)M * N) return;
  float v = slabs[i];
  for (int k = 1; k < nsplit; ++k) v += slabs[(long)k * M * N + i];
  C[(i / N) * ldc + i % N] = v;
}

// The PPM-branch columns of the bottleneck weights (input channels 2048 + 512 i + ci) in GEMM
// form for the folded PPM field:  dir 0  wq[i][ci][tap * 512 + co] = w[co][packed_k(2048 + 512 i + ci, tap)];
// dir 1 writes wq back into w (the weight gradient).  32 x 32 tiles transposed through LDS.
__global__ __launch_bounds__(256) void ppm_wq_kernel(float* __restrict__ w, long w_ld, float* __restrict__ wq, int dir) {
  __shared__ float tile[32][33];
  const int i = blockIdx.x / 9, tap = blockIdx.x % 9;
  const int cb = blockIdx.y, co0 = blockIdx.z * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const long kb = packed_k(2048 + 512 * i + 32 * cb, tap, 9);  // the block's 32 channels are contiguous
  float* q = wq + ((long)i * 512 + 32 * cb) * 4608 + tap * 512 + co0;
  if (dir == 0) {
    for (int r = ty; r < 32; r += 8) tile[r][tx] = w[(long)(co0 + r) * w_ld + kb + tx];
    __syncthreads();
    for (int r = ty; r < 32; r += 8) q[(long)r * 4608 + tx] = tile[tx][r];
  } else {
    for (int r = ty; r < 32; r += 8) tile[r][tx] = q[(long)r * 4608 + tx];
    __syncthreads();
    for (int r = ty; r < 32; r += 8) w[(long)(co0 + r) * w_ld + kb + tx] = tile[tx][r];
  }
}

int launch_ppm_wq(float* w, long w_ld, float* wq, int dir, hipStream_t st) {
  hipLaunchKernelGGL(ppm_wq_kernel, dim3(36, 16, 16), dim3(256), 0, st, w, w_ld, wq, dir);
  CWT_LAUNCH_CHECK();
  return 0;
}

int launch_pt_gemm(PtGemm g, float* ws, size_t ws_floats, hipStream_t st) {
  const long tiles = (long)cdiv(g.M, 64) * cdiv(g.N, 64);
  int ns = 1;
  while (tiles * ns < 512 && g.K / (ns * 2) >= 256 && (size_t)(ns * 2) * g.M * g.N <= ws_floats) ns *= 2;
  g.k_per_split = (int)(((g.K + ns - 1) / ns + 15) / 16 * 16);
  ns = (int)((g.K + g.k_per_split - 1) / g.k_per_split);
  g.slab = ns > 1 ? ws : nullptr;
  hipLaunchKernelGGL(pt_gemm_kernel, dim3(cdiv(g.M, 64), cdiv(g.N, 64), ns), dim3(256), 0, st, g);
  CWT_LAUNCH_CHECK();
  if (ns > 1) {
    hipLaunchKernelGGL(slab_reduce_2d_kernel, dim3(cdiv((long)g.M * g.N, 256)), dim3(256), 0, st, (const float*)ws, ns,
                       g.M, g.N, g.C, g.ldc);
    CWT_LAUNCH_CHECK();
  }
  return 0;
}

// ------------------------------------------------------------------------------------------
// Label-smoothed CE of the upsampled logits (pretrain.py:163-219 compute_loss / cross_entropy,
// PSPNet.classify pspnet.py:183-187): logits [N][h][w][NC] (NHWC), bilinear align_corners to
// S x S, log_softmax over the classes, one-hot of the target (255 -> class 0) smoothed to
// 1 - eps / eps / (NC - 1), loss = mean over non-255 pixels of -sum(onehot * logp).  Gradient
// at the high-res logits (p - onehot) / n_valid, taken to the low-res grid by the separable
// adjoint of the upsample:
//   pass 1 (one thread per high-res row Y and low-res column segment [8j, 8j+8) when
//           S - 1 == 8 (w - 1), else per output column): each pixel's gradient split between
//           its two source columns -> R[n][Y][j][c] (row-resolved, columns reduced);
//   pass 2: dlogits[n][i][j][c] = sum_Y u_Y(i) R[n][Y][j][c] (fixed order).
// The loss sum and the valid count come out as per-block partials (fixed-order final sum).
// ------------------------------------------------------------------------------------------
template <int NC>
__global__ __launch_bounds__(64) void seg_ce_rows_kernel(PtLoss a, float* __restrict__ R, double* __restrict__ part) {
  const int n = blockIdx.z, Y = blockIdx.y;
  const int j = blockIdx.x * 64 + threadIdx.x;  // low-res column: this thread owns the high-res X with lerp i0 == j
  const int S = a.S, h = a.h, w = a.w;
  const float sy = align_corners_scale(h, S), sx = align_corners_scale(w, S);
  const Lerp ly = lerp_coord(Y, h, sy);
  double lsum = 0.0;
  unsigned cnt = 0;
  float rl[NC], rr[NC];  // unscaled gradient parts for column j (left) and j + 1 (right)
#pragma unroll
  for (int c = 0; c < NC; ++c) rl[c] = rr[c] = 0.f;
  if (j < w) {
    const int xa = max(0, (int)floorf((float)j / sx) - 2), xb = min(S, (int)ceilf((float)(j + 1) / sx) + 2);
    const float* L0 = a.logits + (((long)n * h + ly.i0) * w) * NC;
    const float* L1 = a.logits + (((long)n * h + ly.i1) * w) * NC;
    const int64_t* tg = a.target + ((long)n * S + Y) * S;
    for (int X = xa; X < xb; ++X) {
      const Lerp lx = lerp_coord(X, w, sx);
      if (lx.i0 != j) continue;
      const int y = (int)tg[X];
      if (y == a.ignore) continue;
      float z[NC];
      float m = -INFINITY;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        z[c] = ly.l0 * (lx.l0 * L0[lx.i0 * NC + c] + lx.l1 * L0[lx.i1 * NC + c]) +
               ly.l1 * (lx.l0 * L1[lx.i0 * NC + c] + lx.l1 * L1[lx.i1 * NC + c]);
        m = fmaxf(m, z[c]);
      }
      float se = 0.f;
#pragma unroll
      for (int c = 0; c < NC; ++c) se += expf(z[c] - m);
      const float lse = m + logf(se);
      const int yc = (y < 0 || y >= NC) ? 0 : y;
      float l = 0.f;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const float oh = (c == yc) ? a.on : a.off;
        const float logp = z[c] - lse;
        l -= oh * logp;
        const float g = expf(logp) - oh;
        rl[c] = fmaf(lx.l0, g, rl[c]);
        rr[c] = fmaf(lx.l1, g, rr[c]);
      }
      lsum += (double)l;
      ++cnt;
    }
    const long o = (((long)n * S + Y) * (w + 1) + j) * NC;
#pragma unroll
    for (int c = 0; c < NC; ++c) R[o + c] = rl[c];
#pragma unroll
    for (int c = 0; c < NC; ++c) a.Rr[o + NC + c] = rr[c];
  }
  // block partial of the loss sum and count (fixed order through LDS)
  __shared__ double sl[64];
  __shared__ unsigned sc[64];
  sl[threadIdx.x] = lsum;
  sc[threadIdx.x] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    unsigned k = 0;
    for (int i = 0; i < 64; ++i) {
      s += sl[i];
      k += sc[i];
    }
    const long b = ((long)n * gridDim.y + Y) * gridDim.x + blockIdx.x;
    part[2 * b] = s;
    part[2 * b + 1] = (double)k;
  }
}

// loss = sum / n_valid and inv[0] = 1 / n_valid (the mean's gradient factor)
__global__ void seg_ce_final_kernel(const double* __restrict__ part, long nblk, float* __restrict__ loss,
                                    float* __restrict__ inv) {
  __shared__ double s1[256], s2[256];
  double a = 0.0, b = 0.0;
  for (long i = threadIdx.x; i < nblk; i += 256) {
    a += part[2 * i];
    b += part[2 * i + 1];
  }
  s1[threadIdx.x] = a;
  s2[threadIdx.x] = b;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      s1[threadIdx.x] += s1[threadIdx.x + o];
      s2[threadIdx.x] += s2[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    // every pixel ignored: loss 0/0 = NaN and zero gradients, as torch's CE (ignore_index)
    loss[0] = (float)(s1[0] / s2[0]);
    inv[0] = s2[0] > 0.0 ? (float)(1.0 / s2[0]) : 0.f;
  }
}

template <int NC>
__global__ void seg_ce_cols_kernel(PtLoss a, const float* __restrict__ R, const float* __restrict__ inv) {
  const long total = (long)a.N * a.h * a.w * NC;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c = (int)(i % NC);
  const long p = i / NC;
  const int j = (int)(p % a.w), ii = (int)((p / a.w) % a.h), n = (int)(p / ((long)a.w * a.h));
  const int S = a.S;
  const float sy = align_corners_scale(a.h, S);
  const int ya = max(0, (int)floorf((float)(ii - 1) / sy) - 2), yb = min(S, (int)ceilf((float)(ii + 1) / sy) + 2);
  float s = 0.f;
  for (int Y = ya; Y < yb; ++Y) {
    const Lerp ly = lerp_coord(Y, a.h, sy);
    const float wy = (ly.i0 == ii ? ly.l0 : 0.f) + (ly.i1 == ii ? ly.l1 : 0.f);
    if (wy == 0.f) continue;
    const long o = (((long)n * S + Y) * (a.w + 1) + j) * NC + c;
    s = fmaf(wy, R[o] + a.Rr[o], s);
  }
  a.dlogits[p * NC + c] = s * inv[0];
}

template <int NC>
static int launch_seg_ce_nc(PtLoss a, float* R, double* part, float* inv, float* loss, hipStream_t st) {
  const dim3 g1(cdiv(a.w, 64), a.S, a.N);
  hipLaunchKernelGGL((seg_ce_rows_kernel<NC>), g1, dim3(64), 0, st, a, R, part);
  CWT_LAUNCH_CHECK();
  hipLaunchKernelGGL(seg_ce_final_kernel, dim3(1), dim3(256), 0, st, (const double*)part, (long)g1.x * g1.y * g1.z, loss,
                     inv);
  CWT_LAUNCH_CHECK();
  const long total = (long)a.N * a.h * a.w * NC;
  hipLaunchKernelGGL((seg_ce_cols_kernel<NC>), dim3(cdiv(total, 256)), dim3(256), 0, st, a, (const float*)R,
                     (const float*)inv);
  CWT_LAUNCH_CHECK();
  return 0;
}

size_t seg_ce_ws_bytes(int N, int S, int w, int nc) {
  return (size_t)2 * N * S * (w + 1) * nc * 4 + (size_t)2 * cdiv(w, 64) * S * N * 8 + 256;
}

int launch_seg_ce_smooth(PtLoss a, void* ws, size_t ws_bytes, float* loss, hipStream_t st) {
  if (seg_ce_ws_bytes(a.N, a.S, a.w, a.nc) > ws_bytes) return fail(CWT_ESTATE, "seg_ce: workspace too small");
  const size_t plane = (size_t)a.N * a.S * (a.w + 1) * a.nc;
  float* R = (float*)ws;
  a.Rr = R + plane;
  double* part = (double*)(a.Rr + plane);
  float* inv = (float*)(part + (size_t)2 * cdiv(a.w, 64) * a.S * a.N);
  CWT_HIP(hipMemsetAsync(R, 0, 2 * plane * 4, st));
  switch (a.nc) {
    case 16: return launch_seg_ce_nc<16>(a, R, part, inv, loss, st);
    case 61: return launch_seg_ce_nc<61>(a, R, part, inv, loss, st);
    case 2: return launch_seg_ce_nc<2>(a, R, part, inv, loss, st);
    default: return fail(CWT_EARG, "seg_ce: num_classes must be 2, 16 or 61");
  }
}

}  // namespace cwt

namespace cwt {

// ------------------------------------------------------------------------------------------
// Evaluation of the upsampled logits (pretrain.py:223-250 standard_validate and the logging
// block :123-131): per high-res pixel the bilinear (align_corners) logits, their argmax (first
// maximum, as torch's CPU argmax) and nn.CrossEntropyLoss(ignore_index=255) (plain one-hot);
// intersectionAndUnionGPU (util.py:280-308) counts per class: pixels with target 255 are
// excluded from every count.  Integer counts through LDS then global atomics (order-free,
// exact); the loss as per-block partials summed in fixed order.
// counts: [3][NC] unsigned (intersection, prediction, target); part: 2 doubles per block.
// ------------------------------------------------------------------------------------------
template <int NC>
__global__ __launch_bounds__(64) void seg_eval_kernel(PtLoss a, unsigned* __restrict__ counts, double* __restrict__ part) {
  __shared__ unsigned sc[3][NC];
  for (int i = threadIdx.x; i < 3 * NC; i += 64) (&sc[0][0])[i] = 0u;
  __syncthreads();
  const int n = blockIdx.z, Y = blockIdx.y;
  const int j = blockIdx.x * 64 + threadIdx.x;
  const int S = a.S, h = a.h, w = a.w;
  const float sy = align_corners_scale(h, S), sx = align_corners_scale(w, S);
  const Lerp ly = lerp_coord(Y, h, sy);
  double lsum = 0.0;
  unsigned cnt = 0;
  if (j < w) {
    const int xa = max(0, (int)floorf((float)j / sx) - 2), xb = min(S, (int)ceilf((float)(j + 1) / sx) + 2);
    const float* L0 = a.logits + (((long)n * h + ly.i0) * w) * NC;
    const float* L1 = a.logits + (((long)n * h + ly.i1) * w) * NC;
    const int64_t* tg = a.target + ((long)n * S + Y) * S;
    for (int X = xa; X < xb; ++X) {
      const Lerp lx = lerp_coord(X, w, sx);
      if (lx.i0 != j) continue;
      const int y = (int)tg[X];
      if (y == a.ignore) continue;
      float z[NC];
      float m = -INFINITY;
      int am = 0;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        z[c] = ly.l0 * (lx.l0 * L0[lx.i0 * NC + c] + lx.l1 * L0[lx.i1 * NC + c]) +
               ly.l1 * (lx.l0 * L1[lx.i0 * NC + c] + lx.l1 * L1[lx.i1 * NC + c]);
        if (z[c] > m) {
          m = z[c];
          am = c;
        }
      }
      float se = 0.f;
#pragma unroll
      for (int c = 0; c < NC; ++c) se += expf(z[c] - m);
      float zy = 0.f;
#pragma unroll
      for (int c = 0; c < NC; ++c) zy = (c == y) ? z[c] : zy;
      lsum += (double)(m + logf(se) - zy);
      ++cnt;
      atomicAdd(&sc[1][am], 1u);
      if (y >= 0 && y < NC) {
        atomicAdd(&sc[2][y], 1u);
        if (am == y) atomicAdd(&sc[0][y], 1u);
      }
    }
  }
  __shared__ double sl[64];
  __shared__ unsigned sk[64];
  sl[threadIdx.x] = lsum;
  sk[threadIdx.x] = cnt;
  __syncthreads();
  for (int i = threadIdx.x; i < 3 * NC; i += 64)
    if ((&sc[0][0])[i]) atomicAdd(&counts[i], (&sc[0][0])[i]);
  if (threadIdx.x == 0) {
    double s = 0.0;
    unsigned k = 0;
    for (int i = 0; i < 64; ++i) {
      s += sl[i];
      k += sk[i];
    }
    const long b = ((long)n * gridDim.y + Y) * gridDim.x + blockIdx.x;
    part[2 * b] = s;
    part[2 * b + 1] = (double)k;
  }
}

// out[0] = mean loss over the valid pixels, out[1] = their count; iu[3][nc] floats from the counts
// (intersection, union = prediction + target - intersection, target), as intersectionAndUnionGPU
__global__ void seg_eval_final_kernel(const double* __restrict__ part, long nblk, const unsigned* __restrict__ counts,
                                      int nc, float* __restrict__ out, float* __restrict__ iu) {
  __shared__ double s1[256], s2[256];
  double a = 0.0, b = 0.0;
  for (long i = threadIdx.x; i < nblk; i += 256) {
    a += part[2 * i];
    b += part[2 * i + 1];
  }
  s1[threadIdx.x] = a;
  s2[threadIdx.x] = b;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      s1[threadIdx.x] += s1[threadIdx.x + o];
      s2[threadIdx.x] += s2[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[0] = (float)(s1[0] / s2[0]);
    out[1] = (float)s2[0];
  }
  for (int c = threadIdx.x; c < nc; c += 256) {
    const float in = (float)counts[c], pr = (float)counts[nc + c], tg = (float)counts[2 * nc + c];
    iu[c] = in;
    iu[nc + c] = pr + tg - in;
    iu[2 * nc + c] = tg;
  }
}

template <int NC>
static int launch_seg_eval_nc(PtLoss a, unsigned* counts, double* part, float* out, float* iu, hipStream_t st) {
  const dim3 g(cdiv(a.w, 64), a.S, a.N);
  hipLaunchKernelGGL((seg_eval_kernel<NC>), g, dim3(64), 0, st, a, counts, part);
  CWT_LAUNCH_CHECK();
  hipLaunchKernelGGL(seg_eval_final_kernel, dim3(1), dim3(256), 0, st, (const double*)part, (long)g.x * g.y * g.z,
                     (const unsigned*)counts, NC, out, iu);
  CWT_LAUNCH_CHECK();
  return 0;
}

size_t seg_eval_ws_bytes(int N, int S, int w, int nc) { return (size_t)3 * nc * 4 + 256 + (size_t)2 * cdiv(w, 64) * S * N * 8; }

int launch_seg_eval(PtLoss a, void* ws, size_t ws_bytes, float* out, float* iu, hipStream_t st) {
  if (seg_eval_ws_bytes(a.N, a.S, a.w, a.nc) > ws_bytes) return fail(CWT_ESTATE, "seg_eval: workspace too small");
  unsigned* counts = (unsigned*)ws;
  double* part = (double*)((char*)ws + (((size_t)3 * a.nc * 4 + 255) & ~(size_t)255));
  CWT_HIP(hipMemsetAsync(counts, 0, (size_t)3 * a.nc * 4, st));
  switch (a.nc) {
    case 16: return launch_seg_eval_nc<16>(a, counts, part, out, iu, st);
    case 61: return launch_seg_eval_nc<61>(a, counts, part, out, iu, st);
    case 2: return launch_seg_eval_nc<2>(a, counts, part, out, iu, st);
    default: return fail(CWT_EARG, "seg_eval: num_classes must be 2, 16 or 61");
  }
}

}  // namespace cwt

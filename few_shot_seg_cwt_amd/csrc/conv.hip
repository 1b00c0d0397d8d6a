// Implicit-GEMM convolution, NHWC fp32, on the CDNA4 f32 matrix cores.
//
// Replaces the cuDNN launches behind every nn.Conv2d + nn.BatchNorm2d (+ residual add)
// (+ ReLU) of the frozen extractor: reference resnet.py:63-68,74-96,111-116,137 and
// pspnet.py:27-29,125-127 (SURVEY.md Appendix A lists every shape).
//
// GEMM view: out[m][co] = sum_k A[m][k] * B[k][co], m = (n, oh, ow), k = (ky, kx, ci)
// (tap-major, ci-minor), A gathered on the fly from the NHWC input (zero outside the
// padded image), B = weights pre-packed [Co][K] (k contiguous).
//
// Tiling: BM x BN block tile, 4 waves (2x2), each wave (BM/2)x(BN/2) built from 32x32
// v_mfma_f32_32x32x2_f32 tiles (f32 in / f32 acc: exact fmaf chains, 64 FLOP/clk/SIMD).
// K advances in BK = 32 slices, always inside one tap because Ci % 32 == 0.  Both operand
// tiles are stored row-major with k contiguous (128 B rows) in LDS, 16-B chunks XOR-
// swizzled by (row>>1)&7 so the ds_read_b128 fragment reads are bank-conflict free.
// Within each 8-k group, lane half h holds k = 8g+4h+{0..3} so one ds_read_b128 feeds four
// MFMAs (the k order inside a sum is free; A and B use the same permutation).
// Pipeline: registers prefetch K-slice t+1 from global while MFMAs consume slice t; two
// LDS buffers, one barrier per slice.
// Epilogue: y = acc*scale[co] + shift[co] (+ residual) (ReLU), written NHWC at a channel
// offset/stride so layer4 can write straight into the PPM concat buffer.  With split-K
// the raw partial sums go to a workspace and conv_splitk_epilogue applies the same math.
#include <algorithm>

#include "common.h"
#include "kernels.h"

namespace cwt {

// STAGE only names the instantiation (0 stem, 1-4 layer1-4, 5 PPM, 6 bottleneck) so that
// rocprofv3's per-kernel statistics break the conv stack down by stage.
// (256x128 tiles at one workgroup per CU were tried: they spill 60-76 VGPRs with the two
// register sets of the prefetch.)
template <int BM, int BN, int STAGE>
__global__ __launch_bounds__(256, 2) void conv_igemm_f32(ConvArgs a) {
  constexpr int BK = 32;
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int TM = WM / 32, TN = WN / 32;
  constexpr int A_LD = BM * 8 / 256;  // float4 chunks per thread per A slice
  constexpr int B_LD = BN * 8 / 256;
  constexpr int ROWS = BM + BN;
  __shared__ f32x4 smem[2][ROWS * 8];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = tid >> 6;
  const int wm = wv >> 1, wn = wv & 1;
  int mt, nt, ks;
  conv_tile_coords(mt, nt, ks);
  const int m0 = mt * BM;
  const int n0 = nt * BN;
  const int kt_begin = ks * a.kt_per_split;
  const int kt_end = min(a.ktiles, kt_begin + a.kt_per_split);

  // ---- per-thread gather geometry (constant over K) ----
  const int lc = tid & 7;   // 16-B chunk within a 128-B row
  const int lr = tid >> 3;  // 0..31
  int a_ih0[A_LD], a_iw0[A_LD], a_pix[A_LD];
  const int HoWo = a.Ho * a.Wo;
#pragma unroll
  for (int j = 0; j < A_LD; ++j) {
    int m = m0 + lr + 32 * j;
    if (m < a.M) {
      int n = m / HoWo;
      int rem = m - n * HoWo;
      int oh = rem / a.Wo;
      int ow = rem - oh * a.Wo;
      a_ih0[j] = oh * a.stride - a.pad;
      a_iw0[j] = ow * a.stride - a.pad;
      a_pix[j] = n * a.Hi * a.Wi;
    } else {
      a_ih0[j] = -(1 << 28);
      a_iw0[j] = 0;
      a_pix[j] = 0;
    }
  }
  const float* wbase = a.w + (long)(n0 + lr) * a.K + lc * 4;

  f32x4 ra[A_LD], rb[B_LD], ra2[A_LD], rb2[B_LD];  // two register sets (two slices in flight)
  auto load_slice = [&](int kt, f32x4(&ra)[A_LD], f32x4(&rb)[B_LD]) {
    const int k0 = kt * BK;
    const int taps = a.kh * a.kw;  // packed_k order: 32-channel block major, taps inner
    const int cb = kt / taps;
    const int tap = kt - cb * taps;
    const int ci0 = cb * BK;
    const int ky = tap / a.kw, kx = tap - (tap / a.kw) * a.kw;
    const int dy = ky * a.dil, dx = kx * a.dil;
#pragma unroll
    for (int j = 0; j < A_LD; ++j) {
      int ih = a_ih0[j] + dy, iw = a_iw0[j] + dx;
      if ((unsigned)ih < (unsigned)a.Hi && (unsigned)iw < (unsigned)a.Wi) {
        const float* p = a.x + (long)(a_pix[j] + ih * a.Wi + iw) * a.x_ld + ci0 + lc * 4;
        ra[j] = *(const f32x4*)p;
      } else {
        ra[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
#pragma unroll
    for (int j = 0; j < B_LD; ++j) rb[j] = *(const f32x4*)(wbase + (long)(32 * j) * a.K + k0);
  };
  auto store_slice = [&](int buf, const f32x4(&ra)[A_LD], const f32x4(&rb)[B_LD]) {
#pragma unroll
    for (int j = 0; j < A_LD; ++j) {
      int row = lr + 32 * j;
      smem[buf][row * 8 + (lc ^ ((row >> 1) & 7))] = ra[j];
    }
#pragma unroll
    for (int j = 0; j < B_LD; ++j) {
      int row = BM + lr + 32 * j;
      smem[buf][row * 8 + (lc ^ ((row >> 1) & 7))] = rb[j];
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int h = lane >> 5;
  const int l31 = lane & 31;

  // Register prefetch two K-slices ahead: two register sets used alternately (the loop is unrolled
  // by two so each set is static); the loads of slice t+2 go out before slice t's MFMAs and have
  // two slices of MFMA time (~3.4 us at 128 x 128) to land before they are stored to LDS.
  auto compute_slice = [&](int cur) {
    const f32x4* sb = smem[cur];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      f32x4 av[TM], bv[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        int row = wm * WM + i * 32 + l31;
        av[i] = sb[row * 8 + ((2 * g + h) ^ ((row >> 1) & 7))];
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        int row = BM + wn * WN + j * 32 + l31;
        bv[j] = sb[row * 8 + ((2 * g + h) ^ ((row >> 1) & 7))];
      }
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i][s], bv[j][s], acc[i][j], 0, 0, 0);
    }
  };
  if (kt_begin < kt_end) {
    load_slice(kt_begin, ra, rb);
    if (kt_begin + 1 < kt_end) load_slice(kt_begin + 1, ra2, rb2);
    store_slice(0, ra, rb);
    __syncthreads();
    for (int kt = kt_begin; kt < kt_end; kt += 2) {
      // LDS buffer 0 holds slice kt, set 2 slice kt+1, set 1 is free
      if (kt + 2 < kt_end) load_slice(kt + 2, ra, rb);
      compute_slice(0);
      if (kt + 1 < kt_end) store_slice(1, ra2, rb2);
      __syncthreads();
      if (kt + 1 >= kt_end) break;
      // LDS buffer 1 holds slice kt+1, set 1 slice kt+2, set 2 is free
      if (kt + 3 < kt_end) load_slice(kt + 3, ra2, rb2);
      compute_slice(1);
      if (kt + 2 < kt_end) store_slice(0, ra, rb);
      __syncthreads();
    }
  }

  // ---- epilogue ----
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int co = n0 + wn * WN + j * 32 + l31;
    float sc = 1.f, sh = 0.f;
    if (!a.part) {
      sc = a.scale[co];
      sh = a.shift[co];
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) conv_store_fragment(a, acc[i][j], m0 + wm * WM + i * 32, co, h, ks, sc, sh);
  }
}

// Sum split-K partials in fixed order (deterministic), then BN / residual / ReLU.
// NS = compile-time split count (0: runtime nsplit): every partial and the residual are
// loaded before the first add, then summed in split order (deterministic).
template <int NS>
__global__ void conv_splitk_epilogue(ConvArgs a, int nsplit) {
  const int c4n = a.Co >> 2;
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)a.M * c4n;
  if (idx >= total) return;
  int m = (int)(idx / c4n);
  int co = (int)(idx - (long)m * c4n) * 4;
  const long ps = (long)a.M * a.Co;
  const float* pp = a.part + (long)m * a.Co + co;
  f32x4 s;
  f32x4 r = {0.f, 0.f, 0.f, 0.f};
  if (a.res) r = *(const f32x4*)(a.res + (long)m * a.res_ld + co);
  if (NS > 0) {
    f32x4 pv[NS > 0 ? NS : 1];
#pragma unroll
    for (int k = 0; k < NS; ++k) pv[k] = *(const f32x4*)(pp + k * ps);
    s = pv[0];
#pragma unroll
    for (int k = 1; k < NS; ++k) s += pv[k];
  } else {
    s = *(const f32x4*)pp;
    for (int k = 1; k < nsplit; ++k) s += *(const f32x4*)(pp + k * ps);
  }
  f32x4 sc = *(const f32x4*)(a.scale + co);
  f32x4 sh = *(const f32x4*)(a.shift + co);
  f32x4 v;
#pragma unroll
  for (int q = 0; q < 4; ++q) v[q] = fmaf(s[q], sc[q], sh[q]);
  v += r;
  if (a.relu) {
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = fmaxf(v[q], 0.f);
  }
  *(f32x4*)(a.y + (long)m * a.y_ld + a.y_off + co) = v;
}

// Measured plans of the exact-fp32 conv (tools/conv_f32_sweep.py on the MI355X,
// tools/gen_plan_table.py --f32): {M, Co, K, bm, bn, nsplit}
struct MeasuredPlanF32 {
  int M, Co, K, bm, bn, nsplit;
};
static const MeasuredPlanF32 kMeasuredPlansF32[] = {
#include "conv_plans_f32.inc"
    {0, 0, 0, 0, 0, 0}};

// Choose tile + split-K for a conv so the grid covers the 256 CUs (SURVEY.md §8(d):
// at batch 1-6 images, M is only 3600-43200 pixels at layer2-4): the measured table first.
ConvPlan plan_conv(int M, int Co, int K) {
  ConvPlan p;
  {
    const int ktiles = K / 32;
    for (const MeasuredPlanF32& e : kMeasuredPlansF32)
      if (e.M == M && e.Co == Co && e.K == K && e.bn > 0 && Co % e.bn == 0) {
        p.bm = e.bm;
        p.bn = e.bn;
        p.kt_per_split = cdiv(ktiles, e.nsplit);
        p.nsplit = cdiv(ktiles, p.kt_per_split);
        return p;
      }
  }
  const int ktiles = K / 32;
  p.bn = (Co % 128 == 0) ? 128 : 64;
  p.bm = 128;
  long tiles = (long)cdiv(M, p.bm) * (Co / p.bn);
  if (tiles < 256) {
    p.bm = 64;
    p.bn = 64;
    tiles = (long)cdiv(M, p.bm) * (Co / p.bn);
  }
  int ks = 1;
  while (tiles * ks < 512 && ktiles / (ks * 2) >= 16) ks *= 2;
  p.kt_per_split = cdiv(ktiles, ks);
  p.nsplit = cdiv(ktiles, p.kt_per_split);
  return p;
}

template <int STAGE>
static void launch_tiles(const ConvArgs& a, const ConvPlan& p, dim3 grid, hipStream_t st) {
  if (p.bm == 128 && p.bn == 128)
    hipLaunchKernelGGL((conv_igemm_f32<128, 128, STAGE>), grid, dim3(256), 0, st, a);
  else if (p.bm == 128 && p.bn == 64)
    hipLaunchKernelGGL((conv_igemm_f32<128, 64, STAGE>), grid, dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((conv_igemm_f32<64, 64, STAGE>), grid, dim3(256), 0, st, a);
}

int launch_conv(ConvArgs a, const ConvPlan& p, int stage, float* part_ws, size_t part_ws_floats, hipStream_t st) {
  a.ktiles = a.K / 32;
  a.kt_per_split = p.kt_per_split;
  const int nsplit = p.nsplit;
  if (nsplit > 1) {
    if ((size_t)nsplit * a.M * a.Co > part_ws_floats) return fail(CWT_ESTATE, "split-K workspace too small");
    a.part = part_ws;
  } else {
    a.part = nullptr;
  }
  dim3 grid(cdiv(a.M, p.bm), a.Co / p.bn, nsplit);
  switch (stage) {
    case 0: launch_tiles<0>(a, p, grid, st); break;
    case 1: launch_tiles<1>(a, p, grid, st); break;
    case 2: launch_tiles<2>(a, p, grid, st); break;
    case 3: launch_tiles<3>(a, p, grid, st); break;
    case 4: launch_tiles<4>(a, p, grid, st); break;
    case 5: launch_tiles<5>(a, p, grid, st); break;
    default: launch_tiles<6>(a, p, grid, st); break;
  }
  CWT_LAUNCH_CHECK();
  if (nsplit > 1) return launch_splitk_epilogue(a, nsplit, st);
  return 0;
}

int launch_splitk_epilogue(const ConvArgs& a, int nsplit, hipStream_t st) {
  long total = (long)a.M * (a.Co / 4);
  const dim3 grid(cdiv(total, 256));
  switch (nsplit) {
    case 2: hipLaunchKernelGGL(conv_splitk_epilogue<2>, grid, dim3(256), 0, st, a, nsplit); break;
    case 4: hipLaunchKernelGGL(conv_splitk_epilogue<4>, grid, dim3(256), 0, st, a, nsplit); break;
    case 8: hipLaunchKernelGGL(conv_splitk_epilogue<8>, grid, dim3(256), 0, st, a, nsplit); break;
    default: hipLaunchKernelGGL(conv_splitk_epilogue<0>, grid, dim3(256), 0, st, a, nsplit); break;
  }
  CWT_LAUNCH_CHECK();
  return 0;
}

// [Co][taps][Ci] (tap-major) -> [Co][packed_k] (32-channel block major, taps inner).
__global__ void repack_cblock_kernel(const float* __restrict__ src, float* __restrict__ dst, int Co, int taps,
                                     int Ci) {
  const long K = (long)taps * Ci;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < (long)Co * K; i += (long)gridDim.x * blockDim.x) {
    const long co = i / K;
    const int r = (int)(i - co * K);
    const int tap = r / Ci, ci = r - tap * Ci;
    dst[co * K + packed_k(ci, tap, taps)] = src[i];
  }
}

int launch_repack_cblock(const float* src, float* dst, int Co, int taps, int Ci, hipStream_t st) {
  if (Ci % 32) return fail(CWT_EARG, "repack: Ci % 32 != 0");
  const long n = (long)Co * taps * Ci;
  hipLaunchKernelGGL(repack_cblock_kernel, dim3((unsigned)std::min<long>(4096, cdiv(n, 256))), dim3(256), 0, st, src,
                     dst, Co, taps, Ci);
  CWT_LAUNCH_CHECK();
  return 0;
}


}  // namespace cwt

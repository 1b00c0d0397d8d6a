// Implicit-GEMM convolution, NHWC, fp32 in/out, computed on the bf16 matrix cores as
// "bf16x3": every fp32 operand is split into hi = bf16(x) and lo = bf16(x - hi) and
//   a.b  ~=  a_hi.b_hi + a_hi.b_lo + a_lo.b_hi          (fp32 accumulation)
// dropping only a_lo.b_lo (~2^-16 |a||b|).  Three v_mfma_f32_32x32x16_bf16 (32 cycles each,
// 16 k) replace eight v_mfma_f32_32x32x2_f32 (64 cycles each, 2 k): 5.3x the fp32 MFMA rate
// per CU at ~1e-5 relative error per conv.  Measured end to end: episode
// logits within 2e-5 of the reference's fp32 CPU path, against the 1e-3 bar; plain bf16
// misses it (7e-3, hundreds of flipped pixels).
//
// Same GEMM view, tiling and epilogue as conv.hip (see there); differences:
//  * weights are pre-split once at load into w_hi / w_lo [Co][K] bf16;
//  * activations stay fp32 in HBM and are split while being staged to LDS
//    (v_cvt_pk_bf16_f32, round-to-nearest-even);
//  * LDS holds four bf16 regions per stage (A_hi, A_lo, B_hi, B_lo), rows of BK = 32
//    bf16 = 4 chunks of 16 B, chunk c stored at c ^ ((row >> 2) & 3): conflict-free for
//    the 16-lane groups of ds_read_b128;
//  * per 16-k sub-step a wave reads one 16-B fragment per operand per 32-row tile and
//    issues 3 MFMAs per 32x32 output tile.
#include "common.h"
#include "kernels.h"

namespace cwt {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

// Tile BM x BN, WAVES_M x WAVES_N waves (each WM x WN = TM x TN fragments of 32x32).
// 4-wave tiles (up to 128x128) keep one workgroup per SIMD quad; the 8-wave 256-row tiles
// halve the operand bytes per FLOP (a 128x128 tile asks ~42 B/clk/CU of L2->CU traffic at
// the bf16 MFMA rate, close to the per-CU load bandwidth).
template <int BM, int BN, int WAVES_M, int WAVES_N, int STAGE>
__global__ __launch_bounds__(WAVES_M * WAVES_N * 64) void conv_igemm_bf16x3(ConvArgs a) {
  constexpr int NT = WAVES_M * WAVES_N * 64;
  constexpr int BK = 32;
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  constexpr int TM = WM / 32, TN = WN / 32;
  constexpr int A_LD = BM * 8 / NT;  // fp32 float4 per thread per A slice
  constexpr int B_LD = BN * 4 / NT;  // 16-B bf16 chunks per thread per B slice (each of hi, lo)
  constexpr int A_PASS = NT / 8;     // A rows covered per load pass
  constexpr int B_PASS = NT / 4;     // B rows covered per load pass
  static_assert(A_LD >= 1 && B_LD >= 1 && TM >= 1 && TN >= 1, "tile too small for the thread count");
  // chunk (16 B) offsets of the four regions inside one stage
  constexpr int AHI = 0, ALO = BM * 4, BHI = BM * 8, BLO = BM * 8 + BN * 4;
  constexpr int STAGE_CHUNKS = BM * 8 + BN * 8;
  __shared__ bf16x8 smem[2 * STAGE_CHUNKS];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = tid >> 6;
  const int wm = wv / WAVES_N, wn = wv % WAVES_N;
  int mt, nt, ks;
  conv_tile_coords(mt, nt, ks);
  const int m0 = mt * BM;
  const int n0 = nt * BN;
  const int kt_begin = ks * a.kt_per_split;
  const int kt_end = min(a.ktiles, kt_begin + a.kt_per_split);

  // A gather geometry (constant over K): thread -> (row lr + A_PASS j, float4 lc).  Element
  // offsets are 32-bit (activations stay far below 2^31 floats); the per-tap shift is uniform.
  const int lc = tid & 7;
  const int lr = tid >> 3;
  int a_ih0[A_LD], a_iw0[A_LD], a_off0[A_LD];
  const int HoWo = a.Ho * a.Wo;
#pragma unroll
  for (int j = 0; j < A_LD; ++j) {
    int m = m0 + lr + A_PASS * j;
    if (m < a.M) {
      int n = m / HoWo;
      int rem = m - n * HoWo;
      int oh = rem / a.Wo;
      int ow = rem - oh * a.Wo;
      a_ih0[j] = oh * a.stride - a.pad;
      a_iw0[j] = ow * a.stride - a.pad;
      a_off0[j] = ((n * a.Hi + a_ih0[j]) * a.Wi + a_iw0[j]) * a.x_ld + lc * 4;
    } else {
      a_ih0[j] = -(1 << 28);
      a_iw0[j] = 0;
      a_off0[j] = 0;
    }
  }
  // B geometry: thread -> (row br + B_PASS j, chunk bc)
  const int bc = tid & 3;
  const int br = tid >> 2;
  const __bf16* whi = a.w_hi + (long)(n0 + br) * a.K + bc * 8;
  const __bf16* wlo = a.w_lo + (long)(n0 + br) * a.K + bc * 8;

  f32x4 ra[A_LD];
  bf16x8 rbh[B_LD], rbl[B_LD];
  // incremental tap / channel position of the K slice (packed_k order: 32-channel block
  // major, taps inner; avoids per-slice integer division)
  int cur_ci0 = 0, cur_ky = 0, cur_kx = 0;
  const int taps = a.kh * a.kw;
  auto seek = [&](int kt) {
    const int cb = kt / taps;
    const int tap = kt - cb * taps;
    cur_ci0 = cb * BK;
    cur_ky = tap / a.kw;
    cur_kx = tap - cur_ky * a.kw;
  };
  auto advance = [&]() {
    if (++cur_kx == a.kw) {
      cur_kx = 0;
      if (++cur_ky == a.kh) {
        cur_ky = 0;
        cur_ci0 += BK;
      }
    }
  };
  bool a_in[A_LD];
  auto load_slice = [&](int kt) {
    const int dy = cur_ky * a.dil, dx = cur_kx * a.dil;
    const int shift = (dy * a.Wi + dx) * a.x_ld + cur_ci0;  // uniform
#pragma unroll
    for (int j = 0; j < A_LD; ++j) {
      // unconditional load at a clamped (always valid) offset; out-of-image rows are zeroed
      // when staged, so no branch (and no wait) sits between the loads
      const int ih = a_ih0[j] + dy, iw = a_iw0[j] + dx;
      a_in[j] = (unsigned)ih < (unsigned)a.Hi && (unsigned)iw < (unsigned)a.Wi;
      ra[j] = *(const f32x4*)(a.x + (a_in[j] ? a_off0[j] + shift : lc * 4));
    }
    const int k0 = kt * BK;
#pragma unroll
    for (int j = 0; j < B_LD; ++j) {
      rbh[j] = *(const bf16x8*)(whi + (long)(B_PASS * j) * a.K + k0);
      rbl[j] = *(const bf16x8*)(wlo + (long)(B_PASS * j) * a.K + k0);
    }
  };
  auto store_slice = [&](int buf) {
    bf16x8* sb = smem + buf * STAGE_CHUNKS;
    bf16x4* sb4 = (bf16x4*)sb;
#pragma unroll
    for (int j = 0; j < A_LD; ++j) {
      const int row = lr + A_PASS * j;
      const int c = lc >> 1, half = lc & 1;
      const int pos = row * 4 + (c ^ ((row >> 2) & 3));
      bf16x4 hi, lo;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float v = a_in[j] ? ra[j][q] : 0.f;
        const __bf16 hb = (__bf16)v;
        hi[q] = hb;
        lo[q] = (__bf16)(v - (float)hb);
      }
      sb4[(AHI + pos) * 2 + half] = hi;
      sb4[(ALO + pos) * 2 + half] = lo;
    }
#pragma unroll
    for (int j = 0; j < B_LD; ++j) {
      const int row = br + B_PASS * j;
      const int pos = row * 4 + (bc ^ ((row >> 2) & 3));
      sb[BHI + pos] = rbh[j];
      sb[BLO + pos] = rbl[j];
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

  if (kt_begin < kt_end) {
    seek(kt_begin);
    load_slice(kt_begin);
    store_slice(0);
    __syncthreads();
    for (int kt = kt_begin; kt < kt_end; ++kt) {
      const int cur = (kt - kt_begin) & 1;
      const bool more = kt + 1 < kt_end;
      if (more) {
        advance();
        load_slice(kt + 1);
      }
      const bf16x8* sb = smem + cur * STAGE_CHUNKS;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int c = 2 * s + h;
        bf16x8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int row = wm * WM + i * 32 + l31;
          const int pos = row * 4 + (c ^ ((row >> 2) & 3));
          ah[i] = sb[AHI + pos];
          al[i] = sb[ALO + pos];
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int row = wn * WN + j * 32 + l31;
          const int pos = row * 4 + (c ^ ((row >> 2) & 3));
          bh[j] = sb[BHI + pos];
          bl[j] = sb[BLO + pos];
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
          }
      }
      if (more) store_slice(cur ^ 1);
      __syncthreads();
    }
  }

  // ---- epilogue (C/D layout of the 32x32 MFMA: col = lane&31, row = (r&3)+8(r>>2)+4h) ----
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

template <int STAGE>
static void launch_tiles_x3(const ConvArgs& a, const ConvPlan& p, dim3 grid, hipStream_t st) {
  if (p.bm == 256 && p.bn == 256)
    hipLaunchKernelGGL((conv_igemm_bf16x3<256, 256, 2, 4, STAGE>), grid, dim3(512), 0, st, a);
  else if (p.bm == 256 && p.bn == 128)
    hipLaunchKernelGGL((conv_igemm_bf16x3<256, 128, 4, 2, STAGE>), grid, dim3(512), 0, st, a);
  else if (p.bm == 128 && p.bn == 128)
    hipLaunchKernelGGL((conv_igemm_bf16x3<128, 128, 2, 2, STAGE>), grid, dim3(256), 0, st, a);
  else if (p.bm == 128 && p.bn == 64)
    hipLaunchKernelGGL((conv_igemm_bf16x3<128, 64, 2, 2, STAGE>), grid, dim3(256), 0, st, a);
  else if (p.bm == 64 && p.bn == 128)
    hipLaunchKernelGGL((conv_igemm_bf16x3<64, 128, 2, 2, STAGE>), grid, dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((conv_igemm_bf16x3<64, 64, 2, 2, STAGE>), grid, dim3(256), 0, st, a);
}

struct MeasuredPlan {
  int M, Co, K, bm, bn, nsplit;
};
static const MeasuredPlan kMeasuredPlans[] = {
#include "conv_plans.inc"
};

// The measured plan for this GEMM shape if the sweep found one (conv_plans.inc), else the
// largest tile that still yields >= kMinWG workgroups, splitting K (powers of two, at
// least 8 k-tiles of 32 per split) where the output alone is too small a grid.
ConvPlan plan_conv_x3(int M, int Co, int K) {
  constexpr long kMinWG = 200;
  const int ktiles = K / 32;
  for (const MeasuredPlan& e : kMeasuredPlans)
    if (e.M == M && e.Co == Co && e.K == K && Co % e.bn == 0) {
      ConvPlan p;
      p.bm = e.bm;
      p.bn = e.bn;
      p.kt_per_split = cdiv(ktiles, e.nsplit);
      p.nsplit = cdiv(ktiles, p.kt_per_split);
      return p;
    }
  static const int cand[6][2] = {{256, 256}, {256, 128}, {128, 128}, {128, 64}, {64, 128}, {64, 64}};
  ConvPlan best;  // if no tile reaches kMinWG: the smallest one that divides Co, most splits
  for (auto& c : cand) {
    if (Co % c[1] != 0) continue;
    const long tiles = (long)cdiv(M, c[0]) * (Co / c[1]);
    int ks = 1;
    while (tiles * ks < kMinWG && ktiles / (ks * 2) >= 8) ks *= 2;
    ConvPlan p;
    p.bm = c[0];
    p.bn = c[1];
    p.kt_per_split = cdiv(ktiles, ks);
    p.nsplit = cdiv(ktiles, p.kt_per_split);
    if (tiles * p.nsplit >= kMinWG) return p;
    best = p;
  }
  return best;
}

int launch_conv_x3(ConvArgs a, const ConvPlan& p, int stage, float* part_ws, size_t part_ws_floats,
                   hipStream_t st) {
  if (!a.w_hi || !a.w_lo) return fail(CWT_ESTATE, "bf16x3 conv needs split weights");
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
    case 0: launch_tiles_x3<0>(a, p, grid, st); break;
    case 1: launch_tiles_x3<1>(a, p, grid, st); break;
    case 2: launch_tiles_x3<2>(a, p, grid, st); break;
    case 3: launch_tiles_x3<3>(a, p, grid, st); break;
    case 4: launch_tiles_x3<4>(a, p, grid, st); break;
    case 5: launch_tiles_x3<5>(a, p, grid, st); break;
    default: launch_tiles_x3<6>(a, p, grid, st); break;
  }
  CWT_LAUNCH_CHECK();
  if (nsplit > 1) return launch_splitk_epilogue(a, nsplit, st);
  return 0;
}

}  // namespace cwt

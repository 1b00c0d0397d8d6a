// Implicit-GEMM convolution on split activations ("x3s"): bf16x3 arithmetic (every fp32
// operand x = hi + lo with hi = bf16_rne(x), lo = bf16_rne(x - hi); a.b = a_lo.b_hi +
// a_hi.b_lo + a_hi.b_hi, three bf16 MFMAs with fp32 accumulation, only a_lo.b_lo ~ 2^-16
// dropped) with BOTH operands stored pre-split in HBM, so the main loop moves bytes
// HBM/L2 -> LDS by LDS-DMA (global_load_lds_dwordx4) and never touches them in VGPRs.
//
// Split layout ("S-layout") of an activation map with C channels, and of the packed weights:
//   [row][C/32][64 bf16]: per 32-channel block, 32 x hi = bf16_rne(v) then 32 x lo =
//   bf16_rne(v - hi).  One 128-B line holds one block of one pixel (or of one output
//   channel's K-slice for the weights, rows = Co, blocks in packed_k order).
// hi + lo carries 16 significant bits, which is all the bf16x3 MFMAs see of an fp32 operand
// anyway: storing the split instead of fp32 changes only what residual adds and the byte
// kernels see (hi + lo, a 2^-17 relative rounding of the fp32 value).  Same bytes as fp32.
//
// Main loop (one barrier per 32-deep K-tile, NSTG-deep LDS ring):
//   wait own LDS-DMA of tile t (counted vmcnt, later tiles stay in flight) -> barrier ->
//   issue LDS-DMA of tile t+NSTG-1 into the slot tile t-1 just vacated -> fragments of
//   tile t by ds_read_b128 -> 3 x v_mfma_f32_16x16x32_bf16 per 16x16 fragment pair.
// LDS image: rows of 128 B (A rows then B rows per stage), 16-B chunk c of row r stored in
// slot c ^ ((r >> 1) & 7) (the swizzle goes on the LDS-DMA SOURCE address, the image
// itself is lane-linear): conflict-free for the 16x16x32 fragment reads (4 lane groups of
// 16 hit 16 distinct 16-B bank slots; checked exhaustively).
// Out-of-image taps (zero padding) and rows past M load from a zero line.
// Epilogue: fragments -> per-wave LDS tile -> row-contiguous 8-channel groups per lane:
// BN scale/shift, residual (fp32 or S-layout), ReLU, stored as fp32 NHWC (channel
// offset/stride) and/or S-layout, or the raw split-K partials (fp32 [ks][M][Co]).
//
// PREC = 1 (conv_igemm_b16, the bf16 conv stack of BASELINE config #5): the same kernel over
// PLAIN bf16 operands.  Activations are NHWC bf16 ([row][C], i.e. the S-layout with
// 64-channel blocks and no lo half) and the weights [Co][K] bf16 with K ordered
// (64-channel block, tap, channel): a 128-B LDS row holds 64 consecutive k of one pixel/tap,
// so a K-tile is 64 deep and its two 32-deep halves (chunks 0-3 and 4-7 of the row, where
// PREC 3 keeps hi and lo) take one MFMA each.  fp32 accumulation; BN, residual and ReLU in
// fp32; outputs rounded to bf16 (fp32 for the last conv, whose output is the feature map).
#include "conv_body.h"

namespace cwt {
// STAGE only names the instantiation (rocprofv3 reports the conv stack by stage).
template <int BM, int BN, int WAVES_M, int WAVES_N, int NSTG, int STAGE, int PF = 0>
__global__ __launch_bounds__(WAVES_M* WAVES_N * 64) void conv_igemm_x3s(ConvSArgs a) {
  conv_s_body<BM, BN, WAVES_M, WAVES_N, NSTG, 3, (PF | 8)>(a);
}
template <int BM, int BN, int WAVES_M, int WAVES_N, int NSTG, int STAGE, int PF = 0>
__global__ __launch_bounds__(WAVES_M* WAVES_N * 64) void conv_igemm_b16(ConvSArgs a) {
  conv_s_body<BM, BN, WAVES_M, WAVES_N, NSTG, 1, (PF | 8)>(a);
}
// Exact fp32 on the same LDS-DMA body: fp32 NHWC activations and the fp32 packed weights are
// byte-for-byte the S-layout's geometry (one 128-B line = 32 fp32 channels of one pixel, or 32 k
// of one packed weight row), so only the fragment arithmetic differs (v_mfma_f32_16x16x4_f32,
// an fmaf chain per output: the reference's fp32 products without the bf16x3 split).
template <int BM, int BN, int WAVES_M, int WAVES_N, int NSTG, int STAGE, int PF = 0>
__global__ __launch_bounds__(WAVES_M* WAVES_N * 64) void conv_igemm_f32d(ConvSArgs a) {
  conv_s_body<BM, BN, WAVES_M, WAVES_N, NSTG, 0, (PF | 8)>(a);
}

// Split-K reduction (fixed order, deterministic) + the same epilogue math.
template <int NS, int PREC>
__global__ void conv_s_splitk_epilogue(ConvSArgs a, int nsplit) {
  const int g8 = a.Co >> 3;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)a.M * g8) return;
  const int m = (int)(idx / g8);
  const int co = (int)(idx - (long)m * g8) * 8;
  const long ps = (long)a.M * a.Co;
  const float* pp = a.part + (long)m * a.Co + co;
  float v[8];
  {
    const f32x4 p0 = *(const f32x4*)pp, p1 = *(const f32x4*)(pp + 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[i] = p0[i];
      v[4 + i] = p1[i];
    }
  }
  const int ns = NS > 0 ? NS : nsplit;
#pragma unroll
  for (int k = 1; k < (NS > 0 ? NS : 64); ++k) {
    if (k >= ns) break;
    const f32x4 p0 = *(const f32x4*)(pp + k * ps), p1 = *(const f32x4*)(pp + k * ps + 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[i] += p0[i];
      v[4 + i] += p1[i];
    }
  }
  float sc[8], sh[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    sc[i] = a.scale[co + i];
    sh[i] = a.shift[co + i];
  }
  store_out8<PREC>(a, m, co, v, sc, sh, load_res8<PREC>(a, m, co));
}

// fp32 [P][C] (pixel stride ld) -> S-layout [P][C/32][64]
__global__ void split_act_kernel(const float* x, long P, int C, int ld, __bf16* out) {
  const int g8 = C >> 3;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= P * g8) return;
  const long p = idx / g8;
  const int c = (int)(idx - p * g8) * 8;
  const f32x4 v0 = *(const f32x4*)(x + p * ld + c), v1 = *(const f32x4*)(x + p * ld + c + 4);
  const float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
  bf16x8 hi, lo;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    hi[i] = (__bf16)v[i];
    lo[i] = (__bf16)(v[i] - (float)hi[i]);
  }
  __bf16* sp = out + (p * (C >> 5) + (c >> 5)) * 64 + (c & 31);
  *(bf16x8*)sp = hi;
  *(bf16x8*)(sp + 32) = lo;
}

// S-layout -> fp32 (hi + lo), pixel stride ld
__global__ void unsplit_act_kernel(const __bf16* s, long P, int C, float* out, int ld) {
  const int g8 = C >> 3;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= P * g8) return;
  const long p = idx / g8;
  const int c = (int)(idx - p * g8) * 8;
  const __bf16* sp = s + (p * (C >> 5) + (c >> 5)) * 64 + (c & 31);
  const bf16x8 hi = *(const bf16x8*)sp, lo = *(const bf16x8*)(sp + 32);
  f32x4 v0, v1;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v0[i] = (float)hi[i] + (float)lo[i];
    v1[i] = (float)hi[4 + i] + (float)lo[4 + i];
  }
  *(f32x4*)(out + p * ld + c) = v0;
  *(f32x4*)(out + p * ld + c + 4) = v1;
}

// plain bf16 -> fp32 (the bf16 stack's activations)
__global__ void widen_bf16_kernel(const __bf16* x, long n, float* y) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) y[i] = (float)x[i];
}

int launch_widen_bf16(const __bf16* x, long n, float* y, hipStream_t st) {
  hipLaunchKernelGGL(widen_bf16_kernel, dim3((unsigned)std::min<long>(65536, (n + 255) / 256)), dim3(256), 0, st, x, n, y);
  CWT_LAUNCH_CHECK();
  return 0;
}

int launch_split_act(const float* x, long P, int C, int ld, __bf16* out, hipStream_t st) {
  if (C % 32) return fail(CWT_EARG, "split_act: C % 32");
  const long n = P * (C / 8);
  hipLaunchKernelGGL(split_act_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, x, P, C, ld, out);
  CWT_LAUNCH_CHECK();
  return 0;
}

int launch_unsplit_act(const __bf16* s, long P, int C, float* out, int ld, hipStream_t st) {
  if (C % 32) return fail(CWT_EARG, "unsplit_act: C % 32");
  const long n = P * (C / 8);
  hipLaunchKernelGGL(unsplit_act_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, s, P, C, out, ld);
  CWT_LAUNCH_CHECK();
  return 0;
}

// plan.var: 0 = the base loop; 1 = fragment prefetch (PF), same waves; 2 = PF with 8 waves
// (two per SIMD) on the 128- and 64-row tiles; 4 = 128x128 with a 2-stage ring (64 KB: two
// workgroups per CU).  Deeper rings (one workgroup per CU, 4-5 tiles in flight) measured no
// faster: a workgroup's LDS-DMA intake, not its bytes in flight, is the limit.  256x256 has no PF form: its second fragment
// set does not fit the 256 VGPRs of a wave at two waves per SIMD.
#define CWT_TILE_LAUNCH(KERNEL)                                                                                  \
  template <int STAGE>                                                                                       \
  static void launch_tiles_##KERNEL(const ConvSArgs& a, const ConvPlan& p, dim3 grid, hipStream_t st) {      \
    const int v = p.var;                                                                                     \
    if (v >= 8) { /* timing study (cwt_debug_conv_s only): 8/9 base 64x64 w/o MFMA / w/o DMA,            */ \
      /* 10/11 the 8-wave prefetch 128x128 w/o MFMA / w/o DMA                                              */ \
      if (v == 8) hipLaunchKernelGGL((KERNEL<64, 64, 2, 2, 4, 0, 2>), grid, dim3(256), 0, st, a);           \
      else if (v == 9) hipLaunchKernelGGL((KERNEL<64, 64, 2, 2, 4, 0, 4>), grid, dim3(256), 0, st, a);      \
      else if (v == 10) hipLaunchKernelGGL((KERNEL<128, 128, 2, 4, 3, 0, 3>), grid, dim3(512), 0, st, a);   \
      else hipLaunchKernelGGL((KERNEL<128, 128, 2, 4, 3, 0, 5>), grid, dim3(512), 0, st, a);                \
      return;                                                                                                \
    }                                                                                                        \
    if (p.bm == 256 && p.bn == 256) {                                                                        \
      hipLaunchKernelGGL((KERNEL<256, 256, 2, 4, 2, STAGE, 0>), grid, dim3(512), 0, st, a); /* PF: no VGPRs */ \
    } else if (p.bm == 256 && p.bn == 128) {                                                                 \
      if (v) hipLaunchKernelGGL((KERNEL<256, 128, 4, 2, 3, STAGE, 1>), grid, dim3(512), 0, st, a);           \
      else hipLaunchKernelGGL((KERNEL<256, 128, 4, 2, 3, STAGE, 0>), grid, dim3(512), 0, st, a);             \
    } else if (p.bm == 128 && p.bn == 256) {                                                                 \
      if (v) hipLaunchKernelGGL((KERNEL<128, 256, 2, 4, 3, STAGE, 1>), grid, dim3(512), 0, st, a);           \
      else hipLaunchKernelGGL((KERNEL<128, 256, 2, 4, 3, STAGE, 0>), grid, dim3(512), 0, st, a);             \
    } else if (p.bm == 128 && p.bn == 128) {                                                                 \
      if (v == 4) hipLaunchKernelGGL((KERNEL<128, 128, 2, 2, 2, STAGE, 0>), grid, dim3(256), 0, st, a);      \
      else if (v == 2) hipLaunchKernelGGL((KERNEL<128, 128, 2, 4, 3, STAGE, 1>), grid, dim3(512), 0, st, a); \
      else if (v) hipLaunchKernelGGL((KERNEL<128, 128, 2, 2, 3, STAGE, 1>), grid, dim3(256), 0, st, a);      \
      else hipLaunchKernelGGL((KERNEL<128, 128, 2, 2, 3, STAGE, 0>), grid, dim3(256), 0, st, a);             \
    } else if (p.bm == 128 && p.bn == 64) {                                                                  \
      if (v == 2) hipLaunchKernelGGL((KERNEL<128, 64, 4, 2, 3, STAGE, 1>), grid, dim3(512), 0, st, a);  \
      else if (v) hipLaunchKernelGGL((KERNEL<128, 64, 2, 2, 3, STAGE, 1>), grid, dim3(256), 0, st, a);       \
      else hipLaunchKernelGGL((KERNEL<128, 64, 2, 2, 3, STAGE, 0>), grid, dim3(256), 0, st, a);              \
    } else if (p.bm == 64 && p.bn == 128) {                                                                  \
      if (v == 2) hipLaunchKernelGGL((KERNEL<64, 128, 2, 4, 3, STAGE, 1>), grid, dim3(512), 0, st, a);  \
      else if (v) hipLaunchKernelGGL((KERNEL<64, 128, 2, 2, 3, STAGE, 1>), grid, dim3(256), 0, st, a);       \
      else hipLaunchKernelGGL((KERNEL<64, 128, 2, 2, 3, STAGE, 0>), grid, dim3(256), 0, st, a);              \
    } else {                                                                                                 \
      if (v == 2) hipLaunchKernelGGL((KERNEL<64, 64, 2, 4, 4, STAGE, 1>), grid, dim3(512), 0, st, a);   \
      else if (v) hipLaunchKernelGGL((KERNEL<64, 64, 2, 2, 4, STAGE, 1>), grid, dim3(256), 0, st, a);        \
      else hipLaunchKernelGGL((KERNEL<64, 64, 2, 2, 4, STAGE, 0>), grid, dim3(256), 0, st, a);               \
    }                                                                                                        \
  }
CWT_TILE_LAUNCH(conv_igemm_x3s)
CWT_TILE_LAUNCH(conv_igemm_b16)
CWT_TILE_LAUNCH(conv_igemm_f32d)
#undef CWT_TILE_LAUNCH

struct MeasuredPlanS {
  int M, Co, K, bm, bn, nsplit, var;  // var: main-loop variant (launch_tiles_*; 0 where a line omits it)
};
static const MeasuredPlanS kMeasuredPlansS[] = {
#include "conv_plans_x3s.inc"
};

// The measured plan for this GEMM shape if the sweep found one (conv_plans_x3s.inc, made by
// tools/gen_plan_table.py --x3s from tools/conv_s_sweep.py on the MI355X), else the largest
// tile giving >= kMinWG workgroups, splitting K by powers of two (>= 8 K-tiles per split)
// where the output grid is too small.
ConvPlan plan_heuristic_s(int M, int Co, int ktiles) {
  constexpr long kMinWG = 200;
  static const int cand[7][2] = {{256, 256}, {256, 128}, {128, 256}, {128, 128}, {128, 64}, {64, 128}, {64, 64}};
  ConvPlan best;
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

ConvPlan plan_conv_x3s(int M, int Co, int K) {
  const int ktiles = K / 32;
  for (const MeasuredPlanS& e : kMeasuredPlansS)
    if (e.M == M && e.Co == Co && e.K == K && Co % e.bn == 0) {
      ConvPlan p;
      p.bm = e.bm;
      p.bn = e.bn;
      p.var = e.var;
      p.kt_per_split = cdiv(ktiles, e.nsplit);
      p.nsplit = cdiv(ktiles, p.kt_per_split);
      return p;
    }
  return plan_heuristic_s(M, Co, ktiles);
}

static const MeasuredPlanS kMeasuredPlansB16[] = {
#include "conv_plans_b16.inc"
};

// Plain bf16: 64-deep K-tiles; its own measured table (conv_plans_b16.inc, tools/conv_s_sweep.py
// --prec 1), else the heuristic.
ConvPlan plan_conv_b16(int M, int Co, int K) {
  const int ktiles = K / 64;
  for (const MeasuredPlanS& e : kMeasuredPlansB16)
    if (e.M == M && e.Co == Co && e.K == K && Co % e.bn == 0) {
      ConvPlan p;
      p.bm = e.bm;
      p.bn = e.bn;
      p.var = e.var;
      p.kt_per_split = cdiv(ktiles, e.nsplit);
      p.nsplit = cdiv(ktiles, p.kt_per_split);
      return p;
    }
  return plan_heuristic_s(M, Co, ktiles);
}

static const MeasuredPlanS kMeasuredPlansF32D[] = {
#include "conv_plans_f32d.inc"
    {0, 0, 0, 0, 0, 0, 0}};

// Exact fp32 on the LDS-DMA body: 32-deep K-tiles; its own measured table
// (conv_plans_f32d.inc, tools/conv_s_sweep.py --prec 0), else the heuristic.
ConvPlan plan_conv_f32d(int M, int Co, int K) {
  const int ktiles = K / 32;
  for (const MeasuredPlanS& e : kMeasuredPlansF32D)
    if (e.M == M && e.Co == Co && e.K == K && e.bn > 0 && Co % e.bn == 0) {
      ConvPlan p;
      p.bm = e.bm;
      p.bn = e.bn;
      p.var = e.var;
      p.kt_per_split = cdiv(ktiles, e.nsplit);
      p.nsplit = cdiv(ktiles, p.kt_per_split);
      return p;
    }
  return plan_heuristic_s(M, Co, ktiles);
}

template <int PREC>
static void launch_splitk_s(const ConvSArgs& a, int nsplit, hipStream_t st) {
  const long n = (long)a.M * (a.Co / 8);
  const dim3 g((unsigned)((n + 255) / 256)), b(256);
  switch (nsplit) {
    case 2: hipLaunchKernelGGL((conv_s_splitk_epilogue<2, PREC>), g, b, 0, st, a, nsplit); break;
    case 3: hipLaunchKernelGGL((conv_s_splitk_epilogue<3, PREC>), g, b, 0, st, a, nsplit); break;
    case 4: hipLaunchKernelGGL((conv_s_splitk_epilogue<4, PREC>), g, b, 0, st, a, nsplit); break;
    case 8: hipLaunchKernelGGL((conv_s_splitk_epilogue<8, PREC>), g, b, 0, st, a, nsplit); break;
    default: hipLaunchKernelGGL((conv_s_splitk_epilogue<0, PREC>), g, b, 0, st, a, nsplit); break;
  }
}

// prec 3: bf16x3 over S-layout operands; prec 1: plain bf16 (NHWC bf16 activations, weights in
// 64-channel-block order, plan_conv_b16)
int launch_conv_x3s(ConvSArgs a, const ConvPlan& p, int stage, float* part_ws, size_t part_ws_floats,
                    hipStream_t st, int prec) {
  if (prec != 0 && prec != 1 && prec != 3 && prec != 6)
    return fail(CWT_EARG, "conv precision must be 3 (bf16x3), 1 (bf16), 0 (exact fp32) or 6 (bf16x6)");
  const bool batched = prec == 6 && a.batch > 1;
  if ((prec == 0 || prec == 6) && (a.ys || a.res_s || (!a.y && !batched)))
    return fail(CWT_EARG, "fp32-operand conv: fp32 output and residual only");
  if (batched && (p.nsplit != 1 || !a.part || a.kh != 1 || a.kw != 1))
    return fail(CWT_EARG, "batched x6 GEMMs: 1x1, no split-K, raw output to part");
  if (prec == 6 && !a.ws_lo) return fail(CWT_ESTATE, "x6 conv: the weights' lo plane is missing");
  if (!a.xs || !a.ws || !a.zero) return fail(CWT_ESTATE, "S-layout conv needs its input, weights and a zero line");
  const int kb = prec == 1 ? 64 : 32;
  if (a.Ci % kb || a.Co % 64 || a.Co % p.bn)
    return fail(CWT_EARG, prec == 1 ? "bf16 conv: need Ci % 64 == 0, Co % 64 == 0"
                                    : "x3s conv: need Ci % 32 == 0, Co % 64 == 0");
  a.ktiles = a.K / kb;
  a.ktiles_total = a.ktiles;
  a.kt_per_split = p.kt_per_split;
  const int nsplit = p.nsplit;
  if (nsplit < 1 || (long)p.kt_per_split * nsplit < a.ktiles) return fail(CWT_EARG, "conv plan does not cover K");
  ConvSArgs main = a;
  if (batched) {
    // main.part: the caller's [batch][M][Co] output
  } else if (nsplit > 1) {
    if ((size_t)nsplit * a.M * a.Co > part_ws_floats) return fail(CWT_ESTATE, "split-K workspace too small");
    main.part = part_ws;
  } else {
    main.part = nullptr;
  }
  dim3 grid(cdiv(a.M, p.bm), a.Co / p.bn, nsplit * (batched ? a.batch : 1));
  if (prec == 6) {
    launch_tiles_x6(stage, main, p, grid, st);
  } else if (prec == 0) {
    switch (stage) {
      case 0: launch_tiles_conv_igemm_f32d<0>(main, p, grid, st); break;
      case 1: launch_tiles_conv_igemm_f32d<1>(main, p, grid, st); break;
      case 2: launch_tiles_conv_igemm_f32d<2>(main, p, grid, st); break;
      case 3: launch_tiles_conv_igemm_f32d<3>(main, p, grid, st); break;
      case 4: launch_tiles_conv_igemm_f32d<4>(main, p, grid, st); break;
      case 5: launch_tiles_conv_igemm_f32d<5>(main, p, grid, st); break;
      default: launch_tiles_conv_igemm_f32d<6>(main, p, grid, st); break;
    }
  } else if (prec == 1) {
    switch (stage) {
      case 0: launch_tiles_conv_igemm_b16<0>(main, p, grid, st); break;
      case 1: launch_tiles_conv_igemm_b16<1>(main, p, grid, st); break;
      case 2: launch_tiles_conv_igemm_b16<2>(main, p, grid, st); break;
      case 3: launch_tiles_conv_igemm_b16<3>(main, p, grid, st); break;
      case 4: launch_tiles_conv_igemm_b16<4>(main, p, grid, st); break;
      case 5: launch_tiles_conv_igemm_b16<5>(main, p, grid, st); break;
      default: launch_tiles_conv_igemm_b16<6>(main, p, grid, st); break;
    }
  } else {
    switch (stage) {
      case 0: launch_tiles_conv_igemm_x3s<0>(main, p, grid, st); break;
      case 1: launch_tiles_conv_igemm_x3s<1>(main, p, grid, st); break;
      case 2: launch_tiles_conv_igemm_x3s<2>(main, p, grid, st); break;
      case 3: launch_tiles_conv_igemm_x3s<3>(main, p, grid, st); break;
      case 4: launch_tiles_conv_igemm_x3s<4>(main, p, grid, st); break;
      case 5: launch_tiles_conv_igemm_x3s<5>(main, p, grid, st); break;
      default: launch_tiles_conv_igemm_x3s<6>(main, p, grid, st); break;
    }
  }
  CWT_LAUNCH_CHECK();
  if (nsplit > 1 && !batched) {
    main.part = part_ws;
    if (prec == 1)
      launch_splitk_s<1>(main, nsplit, st);
    else if (prec == 0 || prec == 6)
      launch_splitk_s<0>(main, nsplit, st);
    else
      launch_splitk_s<3>(main, nsplit, st);
    CWT_LAUNCH_CHECK();
  }
  return 0;
}

}  // namespace cwt

// fp32 width on the bf16 matrix cores (conv_igemm_x6, PREC 6 of the shared body, conv_body.h):
// the kernels, their tile / wave-layout forms, the measured plan tables and the weights' split.
#include "conv_body.h"

namespace cwt {

// fp32 width on the bf16 matrix cores: conv_igemm_f32d's activations split three ways in registers,
// the weights pre-split (conv_body.h, PREC 6)
template <int BM, int BN, int WAVES_M, int WAVES_N, int NSTG, int STAGE, int PF = 0>
__global__ __launch_bounds__(WAVES_M* WAVES_N * 64) void conv_igemm_x6(ConvSArgs a) {
  // a stage also holds the weights' lo plane: rings that would overflow the 160 KB of LDS lose a stage
  constexpr int STG = (BM + BN) * 128 + BN * 64;
  constexpr int NS = NSTG * STG <= 163840 ? NSTG : 163840 / STG;
  static_assert(NS >= 2, "x6: a two-stage ring must fit in LDS");
  conv_s_body<BM, BN, WAVES_M, WAVES_N, NS, 6, (PF | 8)>(a);
}

// fp32 packed weights [R][K] (K % 32 == 0) -> the x6 kernel's two weight planes: the S-layout
// line [R][K/32][32 hi | 32 mid] and the lo plane [R][K/32][32 lo] (hi = bf16_rne(w), mid =
// bf16_rne(w - hi), lo = w - hi - mid, exact)
__global__ void split_w3_kernel(const float* w, long n8, int K, __bf16* ws, __bf16* wl) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n8) return;
  const long e = idx * 8;  // 8 consecutive k of one row
  const long r = e / K;
  const int k = (int)(e - r * K);
  const f32x4 v0 = *(const f32x4*)(w + e), v1 = *(const f32x4*)(w + e + 4);
  bf16x8 h, m, l;
  split3_bf16(v0, v1, h, m, l);
  __bf16* sp = ws + (r * (K >> 5) + (k >> 5)) * 64 + (k & 31);
  *(bf16x8*)sp = h;
  *(bf16x8*)(sp + 32) = m;
  *(bf16x8*)(wl + (r * (K >> 5) + (k >> 5)) * 32 + (k & 31)) = l;
}

int launch_split_w3(const float* w, long R, int K, __bf16* ws, __bf16* wl, hipStream_t st) {
  if (K % 32) return fail(CWT_EARG, "split_w3: K % 32");
  const long n8 = R * K / 8;
  hipLaunchKernelGGL(split_w3_kernel, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0, st, w, n8, K, ws, wl);
  CWT_LAUNCH_CHECK();
  return 0;
}

// Timing study (cwt_debug_occupy): each workgroup holds a whole CU -- 1024 threads and all 160 KB of
// its LDS -- and sleeps on the 100 MHz realtime clock for `ticks`, so a conv timed meanwhile on
// another stream gets the CUs the pipeline's resident inner loop leaves it.  Bounded by `ticks`.
__global__ __launch_bounds__(1024) void occupy_kernel(long ticks) {
  extern __shared__ char occ_lds[];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) occ_lds[0] = 0;
  while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)ticks) __builtin_amdgcn_s_sleep(127);
}

int launch_occupy(int nwg, int us, hipStream_t st) {
  constexpr int kLds = 160 * 1024;
  static const hipError_t attr =
      hipFuncSetAttribute((const void*)occupy_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, kLds);
  if (attr != hipSuccess) return fail(CWT_ESTATE, "occupy: 160 KB of dynamic LDS refused");
  hipLaunchKernelGGL(occupy_kernel, dim3(nwg), dim3(1024), kLds, st, (long)us * 100);
  CWT_LAUNCH_CHECK();
  return 0;
}

// Tile and wave-layout forms (plan.var).  The main loop's VALU is the A split (~44 instructions per
// 8 fp32 values, per A fragment per K-tile) against 6 MFMAs per fragment pair, so a wave that holds
// more output columns (larger WN) amortises each split over more MFMAs: var 3 lays the waves out
// WN = 128 wide (FN = 8: ~0.9 VALU per MFMA against ~1.8 at WN = 64; the 16x16x32 MFMA leaves 8 of
// its 16 cycles to vector issue, PMC VALU / MFMA 3-4 in the WN = 64 forms, profiles/r5).
//   256x256: 0 = 2x4 waves, 3 = 4x2 (WN 128);  256x128: 0 = 4x2, 1 = prefetch, 3 = 8x1 (WN 128);
//   128x256: 0 = 2x4, 1 = prefetch, 3 = 4x2 (WN 128);  128x128: 0 = 2x2, 1 = prefetch, 2 = prefetch
//   2x4, 4 = 2x2 on a 2-stage ring, 3 = 4x1 (WN 128), 5 = 4x1 on a 2-stage ring (two per CU);
//   128x64, 64x128, 64x64: 0, 1, 2 as the other kernels; 64x128 also 3 = 4x1 (WN 128), 5 = 4x1 on a
//   2-stage ring; round 6, for the Co = 64 layers (stem conv2, layer1 conv1 / conv2), where the 2x2
//   forms split every A fragment twice: 128x64 3 = 4x1 (WN 64), 5 = the same on a 2-stage ring, 64x64
//   3 = 4x1 (WN 64).  var 8-11: the timing-study kernels;
//   12 / 13: var 5 (128x128) / var 3 (256x256) without the A split (timing study: wrong numbers);
//   14 / 15: var 5 without operand DMA / without MFMAs (timing study: wrong numbers); 16 without
//   both, 17 without both and without the epilogue (the launch, prologue and barriers alone).
template <int STAGE>
static void launch_tiles_x6_stage(const ConvSArgs& a, const ConvPlan& p, dim3 grid, hipStream_t st) {
  const int v = p.var;
#define X6(BM_, BN_, WM_, WN_, NS_, PF_) \
  hipLaunchKernelGGL((conv_igemm_x6<BM_, BN_, WM_, WN_, NS_, STAGE, PF_>), grid, dim3(WM_ * WN_ * 64), 0, st, a)
  if (v >= 8) {
    if (v == 12) X6(128, 128, 4, 1, 2, 16);  // timing study: var 5 without the A split
    else if (v == 14) X6(128, 128, 4, 1, 2, 4);   // timing study: var 5 without operand DMA
    else if (v == 15) X6(128, 128, 4, 1, 2, 2);   // timing study: var 5 without MFMAs
    else if (v == 16) X6(128, 128, 4, 1, 2, 6);   // timing study: var 5 without operand DMA and MFMAs
    else if (v == 17) X6(128, 128, 4, 1, 2, 38);  // timing study: ... and without the epilogue
    else if (v == 18) X6(128, 128, 4, 1, 2, 64);  // timing study: the launch alone (every workgroup returns)
    else if (v == 13) X6(256, 256, 4, 2, 2, 16);  // timing study: 256x256 var 3 without the A split
    else if (v == 8) X6(64, 64, 2, 2, 4, 2);
    else if (v == 9) X6(64, 64, 2, 2, 4, 4);
    else if (v == 10) X6(128, 128, 2, 4, 3, 3);
    else X6(128, 128, 2, 4, 3, 5);
    return;
  }
  if (p.bm == 256 && p.bn == 256) {
    if (v == 3) X6(256, 256, 4, 2, 2, 0);
    else X6(256, 256, 2, 4, 2, 0);
  } else if (p.bm == 256 && p.bn == 128) {
    if (v == 3) X6(256, 128, 8, 1, 2, 0);
    else if (v) X6(256, 128, 4, 2, 3, 1);
    else X6(256, 128, 4, 2, 3, 0);
  } else if (p.bm == 128 && p.bn == 256) {
    if (v == 3) X6(128, 256, 4, 2, 2, 0);
    else if (v) X6(128, 256, 2, 4, 3, 1);
    else X6(128, 256, 2, 4, 3, 0);
  } else if (p.bm == 128 && p.bn == 128) {
    if (v == 5) X6(128, 128, 4, 1, 2, 0);
    else if (v == 4) X6(128, 128, 2, 2, 2, 0);
    else if (v == 3) X6(128, 128, 4, 1, 3, 0);
    else if (v == 2) X6(128, 128, 2, 4, 3, 1);
    else if (v) X6(128, 128, 2, 2, 3, 1);
    else X6(128, 128, 2, 2, 3, 0);
  } else if (p.bm == 128 && p.bn == 64) {
    if (v == 3) X6(128, 64, 4, 1, 3, 0);       // WN = 64: the A split once per row block (Co = 64 layers)
    else if (v == 5) X6(128, 64, 4, 1, 2, 0);  // ... on a two-stage ring
    else if (v == 2) X6(128, 64, 4, 2, 3, 1);
    else if (v) X6(128, 64, 2, 2, 3, 1);
    else X6(128, 64, 2, 2, 3, 0);
  } else if (p.bm == 64 && p.bn == 128) {
    if (v == 3) X6(64, 128, 4, 1, 3, 0);  // WN = 128: one A fragment per wave, no split-K needed at Co = 256
    else if (v == 5) X6(64, 128, 4, 1, 2, 0);
    else if (v == 2) X6(64, 128, 2, 4, 3, 1);
    else if (v) X6(64, 128, 2, 2, 3, 1);
    else X6(64, 128, 2, 2, 3, 0);
  } else {
    if (v == 3) X6(64, 64, 4, 1, 4, 0);  // WN = 64
    else if (v == 2) X6(64, 64, 2, 4, 4, 1);
    else if (v) X6(64, 64, 2, 2, 4, 1);
    else X6(64, 64, 2, 2, 4, 0);
  }
#undef X6
}

// STAGE names the instantiation for rocprofv3 (0 stem .. 6 bottleneck as the other kernels; 7 / 8
// the F(2x2) / F(4x4) Winograd forms' batched GEMMs, so their counters are not averaged with the
// direct convs')
void launch_tiles_x6(int stage, const ConvSArgs& a, const ConvPlan& p, dim3 grid, hipStream_t st) {
  switch (stage) {
    case 0: launch_tiles_x6_stage<0>(a, p, grid, st); break;
    case 1: launch_tiles_x6_stage<1>(a, p, grid, st); break;
    case 2: launch_tiles_x6_stage<2>(a, p, grid, st); break;
    case 3: launch_tiles_x6_stage<3>(a, p, grid, st); break;
    case 4: launch_tiles_x6_stage<4>(a, p, grid, st); break;
    case 5: launch_tiles_x6_stage<5>(a, p, grid, st); break;
    case 6: launch_tiles_x6_stage<6>(a, p, grid, st); break;
    case 7: launch_tiles_x6_stage<7>(a, p, grid, st); break;
    default: launch_tiles_x6_stage<8>(a, p, grid, st); break;
  }
}

// batch: 0 for a direct conv's GEMM, else the Winograd form's GEMM count (16 or 36), M its tiles
struct MeasuredPlanS6 {
  int M, Co, K, bm, bn, nsplit, var, batch;
};

static const MeasuredPlanS6 kMeasuredPlansX6[] = {
#include "conv_plans_x6.inc"
    {0, 0, 0, 0, 0, 0, 0, 0}};

// fp32 width on the bf16 matrix cores (conv_igemm_x6): 32-deep K-tiles over f32d's operands; its
// own measured table (conv_plans_x6.inc, tools/conv_s_sweep.py --prec 6), else the heuristic.
ConvPlan plan_conv_x6(int M, int Co, int K) {
  const int ktiles = K / 32;
  for (const MeasuredPlanS6& e : kMeasuredPlansX6)
    if (e.batch == 0 && e.M == M && e.Co == Co && e.K == K && e.bn > 0 && Co % e.bn == 0) {
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

// The Winograd forms' batched GEMMs [M = tiles][K = Ci] x [Ci][Co] (batch 16 or 36): the
// measured table (entries carrying the batch), else the largest tile giving >= 200 workgroups
// over the whole batch, no split-K
ConvPlan plan_conv_x6_batched(int M, int Co, int K, int batch) {
  const int ktiles = K / 32;
  for (const MeasuredPlanS6& e : kMeasuredPlansX6)
    if (e.batch == batch && e.M == M && e.Co == Co && e.K == K && e.bn > 0 && Co % e.bn == 0 && e.nsplit == 1) {
      ConvPlan p;
      p.bm = e.bm;
      p.bn = e.bn;
      p.var = e.var;
      p.kt_per_split = ktiles;
      p.nsplit = 1;
      return p;
    }
  static const int cand[7][2] = {{256, 256}, {256, 128}, {128, 256}, {128, 128}, {128, 64}, {64, 128}, {64, 64}};
  ConvPlan best;
  for (auto& c : cand) {
    if (Co % c[1] != 0) continue;
    ConvPlan p;
    p.bm = c[0];
    p.bn = c[1];
    p.kt_per_split = ktiles;
    p.nsplit = 1;
    best = p;
    if ((long)cdiv(M, c[0]) * (Co / c[1]) * batch >= 200) return p;
  }
  return best;
}

}  // namespace cwt

// MatchNet's 4-D matching head and the MMN head around it (reference
// src/model/match.py:21-163, src/model/conv4d.py:11-62, src/model/mmn.py:11-71,
// src/model/msm/msm_func.py:50-104): the run_match_model chain of corr_forward,
//   MutualMatching -> NeighConsensus (symmetric, three CenterPivotConv4d + ReLU) ->
//   MutualMatching -> softmax(temp * corr2d) -> v . attn^T,
// over a correlation of NA = hA*wA query positions by NB = hB*wB support positions.
//
// Layout: a 4-D tensor x[B][C][hA][wA][hB][wB] (torch) is held channels-last,
// [B][a][b][C] with a = (ha, wa), b = (hb, wb) row-major: the C <= 10 channels of one (a, b)
// pair are one contiguous run, the b positions of one a a contiguous [hB][wB][C] image.
//
// CenterPivotConv4d (stride 1, kernel 3, padding 1) is two 2-D convolutions summed: conv1 over
// the a plane for every fixed b, conv2 over the b plane for every fixed a (conv4d.py:40-62).
// NeighConsensus in symmetric mode is conv(x) + conv(x^T)^T (match.py:75-80); the transposed
// branch is the same layer stack with the two convolutions' roles swapped (conv1 over b, conv2
// over a), so neither branch moves the 4-D tensor: cp4d_layer_kernel takes the a-plane and
// b-plane weights as arguments.
//
// Arithmetic: exact fp32 everywhere (VALU fmaf for the tiny-channel 4-D convs, the f32 MFMA
// GEMM of heads.hip for v . attn^T); MutualMatching uses the reference's operation order
// (corr * ((corr / (max_B + eps)) * (corr / (max_A + eps)))).
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace cwt {

// ---- MutualMatching (match.py:34-53), per channel of x[B][NA][NB][C] (C = 1 or 2) ----
// row maxima (over b for each a) and per-row-block partial column maxima; a thread reads the C
// channels of a pair as one vector (both channels of a 128-B line in the same block)
constexpr int MM_RB = 16;  // rows of a per block (the scalar form)
constexpr int MM_RBV = 8;  // rows per block of the vector forms (450 workgroups at 60^2)
// PLANAR: x is the torch layout [B][C][NA][NB] (channel planes) instead of channels-last
template <int C, int RB = MM_RBV, bool PLANAR = false>
__global__ __launch_bounds__(256) void mm_rowcol_kernel(const float* __restrict__ x, int NA, int NB,
                                                        float* __restrict__ rowmax, float* __restrict__ colpart,
                                                        const float* __restrict__ x2 = nullptr) {
  // grid: (cdiv(NA, RB), B); rowmax [B*C][NA], colpart [B*C][cdiv(NA,RB)][NB]
  typedef float vec_t __attribute__((ext_vector_type(C)));
  const int b = blockIdx.y;
  const int a0 = blockIdx.x * RB;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const vec_t* xb = (const vec_t*)(x + (long)b * NA * NB * C);
  __shared__ float rm[4][RB][C];
  float rmax[RB][C];
#pragma unroll
  for (int r = 0; r < RB; ++r)
#pragma unroll
    for (int c = 0; c < C; ++c) rmax[r][c] = -INFINITY;
  for (int j = t; j < NB; j += 256) {
    float cm[C];
#pragma unroll
    for (int c = 0; c < C; ++c) cm[c] = -INFINITY;
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const int a = a0 + r;
      if (a < NA) {
        vec_t v;
        if (PLANAR) {
#pragma unroll
          for (int c = 0; c < C; ++c) {
            const float pv = x[((long)(b * C + c) * NA + a) * NB + j];
            if (C == 1) v[0] = pv; else v[c] = pv;
          }
        } else {
          v = xb[(long)a * NB + j];
          if (C == 1 && x2) v[0] = v[0] + x2[(long)b * NA * NB + (long)a * NB + j];  // the symmetric branches' sum
        }
#pragma unroll
        for (int c = 0; c < C; ++c) {
          const float vc = C == 1 ? v[0] : v[c];
          cm[c] = fmaxf(cm[c], vc);
          rmax[r][c] = fmaxf(rmax[r][c], vc);
        }
      }
    }
#pragma unroll
    for (int c = 0; c < C; ++c) colpart[((long)(b * C + c) * gridDim.x + blockIdx.x) * NB + j] = cm[c];
  }
#pragma unroll
  for (int r = 0; r < RB; ++r)
#pragma unroll
    for (int c = 0; c < C; ++c) {
      float v = rmax[r][c];
      for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
      if (lane == 0) rm[wv][r][c] = v;
    }
  __syncthreads();
  if (t < RB * C) {
    const int r = t / C, c = t % C;
    if (a0 + r < NA)
      rowmax[(long)(b * C + c) * NA + a0 + r] = fmaxf(fmaxf(rm[0][r][c], rm[1][r][c]), fmaxf(rm[2][r][c], rm[3][r][c]));
  }
}

// column maxima from the row blocks' partials: block = 64 columns x 4 slices of the row blocks
// (the one-column-per-thread form ran 225 dependent loads per thread on 30 workgroups)
__global__ __launch_bounds__(256) void mm_colmax_kernel(const float* __restrict__ colpart, int nrb, int NB,
                                                        float* __restrict__ colmax) {
  __shared__ float part[4][64];
  const int bc = blockIdx.y;
  const int jl = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + jl;
  float m = -INFINITY;
  if (j < NB)
    for (int rb = sl; rb < nrb; rb += 4) m = fmaxf(m, colpart[((long)bc * nrb + rb) * NB + j]);
  part[sl][jl] = m;
  __syncthreads();
  if (sl == 0 && j < NB) colmax[(long)bc * NB + j] = fmaxf(fmaxf(part[0][jl], part[1][jl]), fmaxf(part[2][jl], part[3][jl]));
}

// y = x * ((x / (rowmax + eps)) * (x / (colmax + eps))); x, y [B][NA][NB][C] (y may alias x).
// grid (NA, B): block (a, b) walks the row's NB pairs (C channels each as one vector)
template <int C, bool PLANAR = false>  // PLANAR: x channel planes [B][C][NA][NB], y channels-last
__global__ __launch_bounds__(256) void mm_apply_kernel(const float* x, int NA, int NB,
                                                       const float* __restrict__ rowmax,
                                                       const float* __restrict__ colmax, float* y,
                                                       const float* __restrict__ x2 = nullptr) {
  typedef float vec_t __attribute__((ext_vector_type(C)));
  const float eps = 1e-5f;
  const int a = blockIdx.x, b = blockIdx.y;
  const long row = ((long)b * NA + a) * NB;
  const vec_t* xr = (const vec_t*)x + row;
  vec_t* yr = (vec_t*)y + row;
  float ra[C];
#pragma unroll
  for (int c = 0; c < C; ++c) ra[c] = rowmax[(long)(b * C + c) * NA + a] + eps;
  for (int j = threadIdx.x; j < NB; j += 256) {
    vec_t v;
    if (PLANAR) {
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const float pv = x[((long)(b * C + c) * NA + a) * NB + j];
        if (C == 1) v[0] = pv; else v[c] = pv;
      }
    } else {
      v = xr[j];
      if (C == 1 && x2) v[0] = v[0] + x2[row + j];
    }
    vec_t o;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const float vc = C == 1 ? v[0] : v[c];
      const float vb = vc / (colmax[(long)(b * C + c) * NB + j] + eps);  // corr4d_B: max over the A positions
      const float va = vc / ra[c];                                       // corr4d_A: max over the B positions
      if (C == 1) o[0] = vc * (va * vb); else o[c] = vc * (va * vb);
    }
    yr[j] = o;
  }
}

// any C (cwt_mutual_matching takes up to 64): the scalar forms
__global__ __launch_bounds__(256) void mm_apply_any_kernel(const float* x, long total, int NA, int NB, int C,
                                                       const float* __restrict__ rowmax,
                                                       const float* __restrict__ colmax, float* y) {
  const float eps = 1e-5f;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int c = (int)(i % C);
    const long p = i / C;
    const int j = (int)(p % NB);
    const long ab = p / NB;
    const int a = (int)(ab % NA), b = (int)(ab / NA);
    const int bc = b * C + c;
    const float v = x[i];
    const float vb = v / (colmax[(long)bc * NB + j] + eps);  // corr4d_B: max over the A positions
    const float va = v / (rowmax[(long)bc * NA + a] + eps);  // corr4d_A: max over the B positions
    y[i] = v * (va * vb);
  }
}
__global__ __launch_bounds__(256) void mm_rowcol_any_kernel(const float* __restrict__ x, int NA, int NB, int C,
                                                        float* __restrict__ rowmax, float* __restrict__ colpart) {
  // grid: (cdiv(NA, MM_RB), B * C); rowmax [B*C][NA], colpart [B*C][cdiv(NA,MM_RB)][NB]
  const int bc = blockIdx.y, b = bc / C, c = bc - b * C;
  const int a0 = blockIdx.x * MM_RB;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const float* xb = x + (long)b * NA * NB * C + c;
  __shared__ float rm[4][MM_RB];
  float rmax[MM_RB];
#pragma unroll
  for (int r = 0; r < MM_RB; ++r) rmax[r] = -INFINITY;
  for (int j = t; j < NB; j += 256) {
    float cm = -INFINITY;
#pragma unroll
    for (int r = 0; r < MM_RB; ++r) {
      const int a = a0 + r;
      if (a < NA) {
        const float v = xb[((long)a * NB + j) * C];
        cm = fmaxf(cm, v);
        rmax[r] = fmaxf(rmax[r], v);
      }
    }
    colpart[((long)bc * gridDim.x + blockIdx.x) * NB + j] = cm;
  }
#pragma unroll
  for (int r = 0; r < MM_RB; ++r) {
    float v = rmax[r];
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    if (lane == 0) rm[wv][r] = v;
  }
  __syncthreads();
  if (t < MM_RB && a0 + t < NA)
    rowmax[(long)bc * NA + a0 + t] = fmaxf(fmaxf(rm[0][t], rm[1][t]), fmaxf(rm[2][t], rm[3][t]));
}

// ---- one CenterPivotConv4d layer (+ ReLU) on x[B][NA][NB][CIN] -> y[B][NA][NB][COUT] ----
// y[a][b][o] = relu( sum_{c,ky,kx} Wa[o][c][ky][kx] x[(ha+ky-1, wa+kx-1)][b][c] + ba[o]
//                  + sum_{c,ky,kx} Wb[o][c][ky][kx] x[a][(hb+ky-1, wb+kx-1)][c] + bb[o] )
// (zero padding).  Workgroup tile: an a patch of TAH x TAW positions by a b patch of TBH x TBW;
// its cross-shaped input (a patch + halo at the tile's b positions, b patch + halo at its a
// positions) is staged in LDS; thread = one (a, b) pair, all COUT outputs.
constexpr int CP_TAH = 2, CP_TAW = 8, CP_TBH = 2, CP_TBW = 8;
constexpr int CP_NA = CP_TAH * CP_TAW, CP_NB = CP_TBH * CP_TBW;             // 16 x 16 = 256 pairs
constexpr int CP_HA = (CP_TAH + 2) * (CP_TAW + 2), CP_HB = (CP_TBH + 2) * (CP_TBW + 2);  // 40 halo positions
// MODE 1 (backward, match_bwd.hip): the input gradient of a layer -- the same cross-shaped
// convolution of the output gradient with each filter transposed (in / out channels exchanged)
// and flipped (tap 8 - t), no bias, no ReLU; accum adds into y (the symmetric branches' sum).
template <int CIN, int COUT, int MODE>
__global__ __launch_bounds__(256) void cp4d_layer_kernel(const float* __restrict__ x, int hA, int wA, int hB, int wB,
                                                         const float* __restrict__ Wa, const float* __restrict__ ba,
                                                         const float* __restrict__ Wb, const float* __restrict__ bb,
                                                         float* __restrict__ y, int accum) {
  // a halo box x b tile, one float of padding per a-halo position (the wave's two a rows of a
  // 32-lane group then fall on disjoint banks); b halo box at the tile's a positions
  __shared__ float xa[CP_HA][CP_NB * CIN + 1];
  __shared__ float xb[CP_NA][CP_HB][CIN];
  // weights tap-major with the outputs innermost ([side][tap][c][o], o padded to a multiple of
  // 4): one broadcast ds_read_b128 gives four outputs' weights for an input value
  constexpr int CO4 = (COUT + 3) & ~3;
  __shared__ __attribute__((aligned(16))) float wl[2][9][CIN][CO4];
  const int NA = hA * wA, NB = hB * wB;
  const int ntb = (wB + CP_TBW - 1) / CP_TBW;
  const int ta = blockIdx.y, tb = blockIdx.x;  // a tile, b tile
  const int ntaw = (wA + CP_TAW - 1) / CP_TAW;
  const int ha0 = (ta / ntaw) * CP_TAH, wa0 = (ta % ntaw) * CP_TAW;
  const int hb0 = (tb / ntb) * CP_TBH, wb0 = (tb % ntb) * CP_TBW;
  const long xoff = (long)blockIdx.z * NA * NB * CIN;
  const int t = threadIdx.x;
  for (int i = threadIdx.x; i < 2 * 9 * CIN * CO4; i += 256) {
    const int o = i % CO4, r = i / CO4;
    const int c = r % CIN, r2 = r / CIN;
    const int tap = r2 % 9, side = r2 / 9;
    const float* W = side ? Wb : Wa;
    (&wl[0][0][0][0])[i] = o >= COUT ? 0.f : MODE == 0 ? W[(o * CIN + c) * 9 + tap] : W[(c * COUT + o) * 9 + 8 - tap];
  }
  // both boxes: every load of the thread issued before the first LDS store (one round of
  // memory latency per workgroup instead of one per element)
  constexpr int EA = CP_HA * CP_NB * CIN, EB = CP_NA * CP_HB * CIN;
  constexpr int IA = (EA + 255) / 256, IB = (EB + 255) / 256;
  float ra[IA], rb[IB];
#pragma unroll
  for (int k = 0; k < IA; ++k) {  // a halo box at the tile's b positions
    const int i = t + 256 * k;
    const int c = i % CIN, p = i / CIN;
    const int bi = p % CP_NB, ai = p / CP_NB;
    const int ha = ha0 - 1 + ai / (CP_TAW + 2), wa = wa0 - 1 + ai % (CP_TAW + 2);
    const int hb = hb0 + bi / CP_TBW, wb = wb0 + bi % CP_TBW;
    const bool in = i < EA && (unsigned)ha < (unsigned)hA && (unsigned)wa < (unsigned)wA && hb < hB && wb < wB;
    ra[k] = in ? x[xoff + (((long)(ha * wA + wa) * NB) + hb * wB + wb) * CIN + c] : 0.f;
  }
#pragma unroll
  for (int k = 0; k < IB; ++k) {  // b halo box at the tile's a positions
    const int i = t + 256 * k;
    const int c = i % CIN, p = i / CIN;
    const int bi = p % CP_HB, ai = p / CP_HB;
    const int ha = ha0 + ai / CP_TAW, wa = wa0 + ai % CP_TAW;
    const int hb = hb0 - 1 + bi / (CP_TBW + 2), wb = wb0 - 1 + bi % (CP_TBW + 2);
    const bool in = i < EB && ha < hA && wa < wA && (unsigned)hb < (unsigned)hB && (unsigned)wb < (unsigned)wB;
    rb[k] = in ? x[xoff + (((long)(ha * wA + wa) * NB) + hb * wB + wb) * CIN + c] : 0.f;
  }
#pragma unroll
  for (int k = 0; k < IA; ++k) {
    const int i = t + 256 * k;
    if (i < EA) {
      const int c = i % CIN, p = i / CIN;
      xa[p / CP_NB][(p % CP_NB) * CIN + c] = ra[k];
    }
  }
#pragma unroll
  for (int k = 0; k < IB; ++k) {
    const int i = t + 256 * k;
    if (i < EB) (&xb[0][0][0])[i] = rb[k];
  }
  __syncthreads();
  const int ai = t / CP_NB, bi = t % CP_NB;  // this thread's pair within the tile
  const int ha = ha0 + ai / CP_TAW, wa = wa0 + ai % CP_TAW;
  const int hb = hb0 + bi / CP_TBW, wb = wb0 + bi % CP_TBW;
  float acc[COUT];
#pragma unroll
  for (int o = 0; o < COUT; ++o) acc[o] = MODE == 0 ? ba[o] + bb[o] : 0.f;
  const int aiy = ai / CP_TAW, aix = ai % CP_TAW, biy = bi / CP_TBW, bix = bi % CP_TBW;
#pragma unroll 1
  for (int tap = 0; tap < 9; ++tap) {  // one tap's inputs and weights live at a time
      const int ky = tap / 3, kx = tap - 3 * (tap / 3);
      const float* pa = &xa[(aiy + ky) * (CP_TAW + 2) + aix + kx][bi * CIN];
      const float* pb = xb[ai][(biy + ky) * (CP_TBW + 2) + bix + kx];
      float va[CIN], vb[CIN];
#pragma unroll
      for (int c = 0; c < CIN; ++c) {
        va[c] = pa[c];
        vb[c] = pb[c];
      }
#pragma unroll
      for (int c = 0; c < CIN; ++c) {
        const float* w0 = wl[0][tap][c];
        const float* w1 = wl[1][tap][c];
#pragma unroll
        for (int o4 = 0; o4 < CO4; o4 += 4) {
          const f32x4 a4 = *(const f32x4*)(w0 + o4), b4 = *(const f32x4*)(w1 + o4);
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (o4 + q < COUT) {
              acc[o4 + q] = fmaf(a4[q], va[c], acc[o4 + q]);
              acc[o4 + q] = fmaf(b4[q], vb[c], acc[o4 + q]);
            }
        }
        if (c & 1) __builtin_amdgcn_sched_barrier(0);  // bounds the weight reads in flight (registers)
      }
    }
  if (ha < hA && wa < wA && hb < hB && wb < wB) {
    float* yp = y + (long)blockIdx.z * NA * NB * COUT + ((long)(ha * wA + wa) * NB + hb * wB + wb) * COUT;
#pragma unroll
    for (int o = 0; o < COUT; ++o) yp[o] = MODE == 0 ? fmaxf(acc[o], 0.f) : accum ? yp[o] + acc[o] : acc[o];
  }
}

// ---- the same layer on the f32 matrix cores (COUT = 10) and a register-blocked VALU form for
// COUT = 1 (round 4; the scalar kernel above measured 16 % of the fp32 VALU peak at 60^2: bound
// by its broadcast LDS weight reads, one per two FMAs, and by 4-B staging loads) ----
// Tile: a 4 x 4 patch of a positions by a 4 x 4 patch of b positions (256 pairs); staged in LDS
// as the a halo box (6 x 6) at the tile's 16 b positions and the tile's 16 a positions at the b
// halo box, CIN floats per position (dense; 2 floats of padding at the end).
constexpr int CM_T = 4, CM_H = CM_T + 2, CM_NH = CM_H * CM_H, CM_NT = CM_T * CM_T;  // 6 x 6 halo, 16 tile
template <int CIN>
struct CmLds {
  static constexpr int EA = CM_NH * CM_NT * CIN, EB = CM_NT * CM_NH * CIN;  // floats
};

// xa[ah][bt][c]: a halo position ah (6 x 6 around the a tile), tile b position bt; xb[at][bh][c]:
// tile a position at, b halo position bh.  CIN even: 8-B loads (a position is CIN / 2 of them,
// 8-B aligned); every load of the thread is issued before the first LDS store; positions off the
// map read 0.
template <int CIN>
__device__ __forceinline__ void cm_stage(const float* __restrict__ x, int hA, int wA, int hB, int wB, int ha0, int wa0,
                                         int hb0, int wb0, long xoff, float* xa, float* xb) {
  const int NB = hB * wB;
  constexpr int V = (CIN % 2 == 0) ? 2 : 1;  // floats per load
  constexpr int VP = CIN / V;                // loads per position
  constexpr int LA = CM_NH * CM_NT * VP, LB = CM_NT * CM_NH * VP;
  constexpr int IA = (LA + 255) / 256, IB = (LB + 255) / 256;
  typedef float vec_t __attribute__((ext_vector_type(V)));
  const int t = threadIdx.x;
  vec_t ra[IA], rb[IB];
#pragma unroll
  for (int k = 0; k < IA; ++k) {
    const int i = t + 256 * k;
    const int q = i % VP, p = i / VP;
    const int bt = p % CM_NT, ah = p / CM_NT;
    const int ha = ha0 - 1 + ah / CM_H, wa = wa0 - 1 + ah % CM_H;
    const int hb = hb0 + bt / CM_T, wb = wb0 + bt % CM_T;
    const bool in = i < LA && (unsigned)ha < (unsigned)hA && (unsigned)wa < (unsigned)wA && hb < hB && wb < wB;
    ra[k] = in ? *(const vec_t*)(x + xoff + (((long)(ha * wA + wa) * NB) + hb * wB + wb) * CIN + q * V) : vec_t(0.f);
  }
#pragma unroll
  for (int k = 0; k < IB; ++k) {
    const int i = t + 256 * k;
    const int q = i % VP, p = i / VP;
    const int bh = p % CM_NH, at = p / CM_NH;
    const int ha = ha0 + at / CM_T, wa = wa0 + at % CM_T;
    const int hb = hb0 - 1 + bh / CM_H, wb = wb0 - 1 + bh % CM_H;
    const bool in = i < LB && ha < hA && wa < wA && (unsigned)hb < (unsigned)hB && (unsigned)wb < (unsigned)wB;
    rb[k] = in ? *(const vec_t*)(x + xoff + (((long)(ha * wA + wa) * NB) + hb * wB + wb) * CIN + q * V) : vec_t(0.f);
  }
#pragma unroll
  for (int k = 0; k < IA; ++k) {
    const int i = t + 256 * k;
    if (i < LA) *(vec_t*)(xa + i * V) = ra[k];
  }
#pragma unroll
  for (int k = 0; k < IB; ++k) {
    const int i = t + 256 * k;
    if (i < LB) *(vec_t*)(xb + i * V) = rb[k];
  }
}

// COUT = 10 on v_mfma_f32_16x16x4_f32 (fp32 products, fp32 sums: an fmaf chain per output).
// Output rows of one MFMA group: the 16 tile b positions of ONE tile a position (group G = the a
// position); columns: the 10 output channels (16 wide, 6 unused).  K = (tap, channel) dense,
// 9 CIN rows padded to a multiple of 4 (zero weights): MFMA m, lane group g = lane / 16 takes
// k = 4 m + g, read at the lane's per-k LDS offset.  Both 2-D convolutions (a plane, b plane)
// accumulate into the same accumulators.  4 waves x 4 groups = the tile's 256 pairs.
// MODE 1: the input gradient of a layer with 10 input channels (the backward, launch_cp4d_dgrad):
// transposed, flipped filters (W[(c COUT + o) 9 + 8 - tap]), no bias, no ReLU, y accumulated when
// accum != 0.
template <int CIN, int MODE = 0>
__global__ __launch_bounds__(256) void cp4d_mfma_kernel(const float* __restrict__ x, int hA, int wA, int hB, int wB,
                                                        const float* __restrict__ Wa, const float* __restrict__ ba,
                                                        const float* __restrict__ Wb, const float* __restrict__ bb,
                                                        float* __restrict__ y, int accum = 0) {
  constexpr int COUT = 10;
  constexpr int KT = 9 * CIN;        // K rows per branch
  constexpr int NM = (KT + 3) / 4;   // MFMAs per branch and group
  __shared__ __attribute__((aligned(16))) float xa[CmLds<CIN>::EA + 2];
  __shared__ __attribute__((aligned(16))) float xb[CmLds<CIN>::EB + 2];
  const int NA = hA * wA, NB = hB * wB;
  const int ntb = (wB + CM_T - 1) / CM_T, nta = (wA + CM_T - 1) / CM_T;
  const int ta = blockIdx.y, tb = blockIdx.x;
  const int ha0 = (ta / nta) * CM_T, wa0 = (ta % nta) * CM_T;
  const int hb0 = (tb / ntb) * CM_T, wb0 = (tb % ntb) * CM_T;
  const long xoff = (long)blockIdx.z * NA * NB * CIN;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int r = lane & 15, g4 = lane >> 4;
  cm_stage<CIN>(x, hA, wA, hB, wB, ha0, wa0, hb0, wb0, xoff, xa, xb);
  // this lane's weights (B operand: column r = output channel, k = 4 m + g4) and the LDS offsets
  // of its k's (tap, channel) in the two staged boxes
  float wra[NM], wrb[NM];
  int offa[NM], offb[NM];
#pragma unroll
  for (int m = 0; m < NM; ++m) {
    const int k = 4 * m + g4;
    const bool kin = k < KT;
    const int tap = kin ? k / CIN : 0, c = kin ? k % CIN : 0;
    const int ky = tap / 3, kx = tap - 3 * (tap / 3);
    const bool live = kin && r < COUT;
    const int wi = MODE == 0 ? (r * CIN + c) * 9 + tap : (c * COUT + r) * 9 + 8 - tap;
    wra[m] = live ? Wa[wi] : 0.f;
    wrb[m] = live ? Wb[wi] : 0.f;
    offa[m] = (ky * CM_H + kx) * CM_NT * CIN + c;
    offb[m] = (ky * CM_H + kx) * CIN + c;
  }
  // row r of group G: a tile position G (ay, ax), b tile position r (by, bx)
  const int by = r / CM_T, bx = r % CM_T;
  const int base_b = (by * CM_H + bx) * CIN;
  __syncthreads();
  f32x4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int m = 0; m < NM; ++m) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int G = wv * 4 + j, ay = G / CM_T, ax = G % CM_T;
      const float va = xa[((ay * CM_H + ax) * CM_NT + r) * CIN + offa[m]];
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(va, wra[m], acc[j], 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int G = wv * 4 + j;
      const float vb = xb[G * CM_NH * CIN + base_b + offb[m]];
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(vb, wrb[m], acc[j], 0, 0, 0);
    }
  }
  // D: lane (col o = r, rows 4 g4 + i) -> pair (a = G, b = 4 g4 + i), channel o
  if (r < COUT) {
    const float bias = MODE == 0 ? ba[r] + bb[r] : 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int G = wv * 4 + j;
      const int ha = ha0 + G / CM_T, wa = wa0 + G % CM_T;
      if (ha >= hA || wa >= wA) continue;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int bt = 4 * g4 + i;
        const int hb = hb0 + bt / CM_T, wb = wb0 + bt % CM_T;
        if (hb < hB && wb < wB) {
          float* yp = y + (long)blockIdx.z * NA * NB * COUT + ((long)(ha * wA + wa) * NB + hb * wB + wb) * COUT + r;
          *yp = MODE == 0 ? fmaxf(acc[j][i] + bias, 0.f) : accum ? *yp + acc[j][i] : acc[j][i];
        }
      }
    }
  }
}

// Weight and bias gradients of one CenterPivotConv4d layer (the backward, match_bwd.hip) on the
// same matrix cores: dW[(side, tap, c)][o] = sum over pairs p of X_side,tap[p][c] G[p][o] is the
// transpose of the forward GEMM -- rows the 18 CIN (side, tap, channel) entries plus one row of
// ones (whose result is the bias gradient sum_p G[p][o]), columns the COUT output channels, K the
// pairs.  Workgroups stride over the forward's 4x4 (a) by 4x4 (b) tiles, staged as cm_stage does,
// with the tile's (ReLU-masked) output gradient beside them; MFMA k-step s takes pairs 4 s .. 4 s
// + 3 (lane group g4 = pair within the step), wave w the row blocks w, w + 4, ...; the sums stay
// in the accumulators across tiles and land in part[workgroup] ([(side, tap, o)][c], then the
// bias), summed in workgroup order by cp4d_wgrad_reduce_kernel.
template <int CIN, int COUT>
__global__ __launch_bounds__(256) void cp4d_wgrad_mfma_kernel(const float* __restrict__ x, const float* __restrict__ gm,
                                                              int B, int hA, int wA, int hB, int wB,
                                                              float* __restrict__ part) {
  constexpr int KE = 18 * CIN;              // (side, tap, c) rows; row KE = ones (the bias)
  constexpr int MB = (KE + 1 + 15) / 16;    // 16-row blocks
  constexpr int MW = (MB + 3) / 4;          // blocks per wave
  constexpr int EA = CmLds<CIN>::EA, EB = CmLds<CIN>::EB;
  constexpr int NE = 18 * COUT;
  __shared__ __attribute__((aligned(16))) float xs[EA + EB + 2];
  __shared__ float gl[CM_NT * CM_NT][COUT];
  float* xa = xs;
  float* xb = xs + EA;
  const int NA = hA * wA, NB = hB * wB;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int i16 = lane & 15, g4 = lane >> 4;
  // this lane's A rows: kind 0 data (LDS offset off[], box b[]), 1 the ones row, 2 padding
  int off[MW], kind[MW];
  bool inb[MW];
#pragma unroll
  for (int mw = 0; mw < MW; ++mw) {
    const int kk = 16 * (wv + 4 * mw) + i16;
    kind[mw] = kk < KE ? 0 : kk == KE ? 1 : 2;
    const int k2 = kk < KE ? kk : 0;
    const int side = k2 / (9 * CIN), tap = (k2 / CIN) % 9, c = k2 % CIN;
    const int ky = tap / 3, kx = tap - 3 * (tap / 3);
    inb[mw] = side != 0;
    off[mw] = side == 0 ? (ky * CM_H + kx) * CM_NT * CIN + c : EA + (ky * CM_H + kx) * CIN + c;
  }
  f32x4 acc[MW];
#pragma unroll
  for (int mw = 0; mw < MW; ++mw) acc[mw] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int ntbw = (wB + CM_T - 1) / CM_T, ntaw = (wA + CM_T - 1) / CM_T;
  const long ntb = (long)((hB + CM_T - 1) / CM_T) * ntbw, nta = (long)((hA + CM_T - 1) / CM_T) * ntaw;
  const long ntiles = (long)B * nta * ntb;
  for (long tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const long tb = tile % ntb, rest = tile / ntb;
    const long ta = rest % nta, bz = rest / nta;
    const int ha0 = (int)(ta / ntaw) * CM_T, wa0 = (int)(ta % ntaw) * CM_T;
    const int hb0 = (int)(tb / ntbw) * CM_T, wb0 = (int)(tb % ntbw) * CM_T;
    __syncthreads();  // the previous tile's LDS reads are done
    cm_stage<CIN>(x, hA, wA, hB, wB, ha0, wa0, hb0, wb0, bz * NA * NB * CIN, xa, xb);
    for (int e = t; e < CM_NT * CM_NT * COUT; e += 256) {
      const int o = e % COUT, p = e / COUT;
      const int at = p / CM_NT, bt = p % CM_NT;
      const int ha = ha0 + at / CM_T, wa = wa0 + at % CM_T, hb = hb0 + bt / CM_T, wb = wb0 + bt % CM_T;
      const bool in = ha < hA && wa < wA && hb < hB && wb < wB;
      (&gl[0][0])[e] = in ? gm[(bz * NA * NB + (long)(ha * wA + wa) * NB + hb * wB + wb) * COUT + o] : 0.f;
    }
    __syncthreads();
#pragma unroll 4
    for (int st = 0; st < CM_NT * CM_NT / 4; ++st) {
      const int p = 4 * st + g4, at = p / CM_NT, bt = p % CM_NT;
      const int terma = (((at / CM_T) * CM_H + at % CM_T) * CM_NT + bt) * CIN;
      const int termb = (at * CM_NH + (bt / CM_T) * CM_H + bt % CM_T) * CIN;
      const float bv = i16 < COUT ? gl[p][i16 < COUT ? i16 : 0] : 0.f;
#pragma unroll
      for (int mw = 0; mw < MW; ++mw) {
        if (wv + 4 * mw >= MB) continue;
        const float av = kind[mw] == 0 ? xs[(inb[mw] ? termb : terma) + off[mw]] : kind[mw] == 1 ? 1.f : 0.f;
        acc[mw] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[mw], 0, 0, 0);
      }
    }
  }
  // D: lane (column o = i16, rows 4 g4 + r of block m)
  float* pw = part + (long)blockIdx.x * (NE * CIN + COUT);
  if (i16 < COUT) {
#pragma unroll
    for (int mw = 0; mw < MW; ++mw) {
      const int m = wv + 4 * mw;
      if (m >= MB) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int kk = 16 * m + 4 * g4 + r;
        if (kk < KE) {
          const int side = kk / (9 * CIN), tap = (kk / CIN) % 9, c = kk % CIN;
          pw[((side * 9 + tap) * COUT + i16) * CIN + c] = acc[mw][r];
        } else if (kk == KE) {
          pw[NE * CIN + i16] = acc[mw][r];
        }
      }
    }
  }
}

int launch_cp4d_wgrad_mfma(const float* x, const float* gm, int B, int hA, int wA, int hB, int wB, int cin, int cout,
                           int G, float* part, hipStream_t st) {
#define CWT_WGM(CI, CO)                                                                                            \
  if (cin == CI && cout == CO) {                                                                                   \
    hipLaunchKernelGGL((cp4d_wgrad_mfma_kernel<CI, CO>), dim3(G), dim3(256), 0, st, x, gm, B, hA, wA, hB, wB, part); \
    CWT_LAUNCH_CHECK();                                                                                            \
    return 0;                                                                                                      \
  }
  CWT_WGM(1, 10)
  CWT_WGM(2, 10)
  CWT_WGM(10, 10)
  CWT_WGM(10, 1)
#undef CWT_WGM
  return fail(CWT_EARG, "cp4d wgrad: channels (1|2 -> 10, 10 -> 10, 10 -> 1) only");
}

// COUT = 1 (the consensus stack's last layer, CIN = 10): a thread per (a, b) pair of the same
// staged tile, its channels read 2 at a time (ds_read_b64), the 2 x 9 x CIN weights in LDS read
// as wave-uniform broadcasts, two independent partial sums per thread.
template <int CIN>
__global__ __launch_bounds__(256) void cp4d_c1_kernel(const float* __restrict__ x, int hA, int wA, int hB, int wB,
                                                      const float* __restrict__ Wa, const float* __restrict__ ba,
                                                      const float* __restrict__ Wb, const float* __restrict__ bb,
                                                      float* __restrict__ y) {
  static_assert(CIN % 2 == 0, "pairs of channels");
  __shared__ __attribute__((aligned(16))) float xa[CmLds<CIN>::EA + 2];
  __shared__ __attribute__((aligned(16))) float xb[CmLds<CIN>::EB + 2];
  __shared__ __attribute__((aligned(16))) float wl[2][9][CIN];
  const int NA = hA * wA, NB = hB * wB;
  const int ntb = (wB + CM_T - 1) / CM_T, nta = (wA + CM_T - 1) / CM_T;
  const int ta = blockIdx.y, tb = blockIdx.x;
  const int ha0 = (ta / nta) * CM_T, wa0 = (ta % nta) * CM_T;
  const int hb0 = (tb / ntb) * CM_T, wb0 = (tb % ntb) * CM_T;
  const long xoff = (long)blockIdx.z * NA * NB * CIN;
  const int t = threadIdx.x;
  if (t < 2 * 9 * CIN) {
    const int c = t % CIN, tap = (t / CIN) % 9, side = t / (9 * CIN);
    (&wl[0][0][0])[t] = (side ? Wb : Wa)[c * 9 + tap];
  }
  cm_stage<CIN>(x, hA, wA, hB, wB, ha0, wa0, hb0, wb0, xoff, xa, xb);
  __syncthreads();
  const int at = t / CM_NT, bt = t % CM_NT;
  const int ay = at / CM_T, ax = at % CM_T, by = bt / CM_T, bx = bt % CM_T;
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  float s0 = 0.f, s1 = 0.f;
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int ky = tap / 3, kx = tap % 3;
    const float* pa = &xa[(((ay + ky) * CM_H + ax + kx) * CM_NT + bt) * CIN];
    const float* pb = &xb[(at * CM_NH + (by + ky) * CM_H + bx + kx) * CIN];
#pragma unroll
    for (int c2 = 0; c2 < CIN / 2; ++c2) {
      const f32x2 va = *(const f32x2*)(pa + 2 * c2), vb = *(const f32x2*)(pb + 2 * c2);
      const f32x2 wa = *(const f32x2*)&wl[0][tap][2 * c2], wb = *(const f32x2*)&wl[1][tap][2 * c2];
      s0 = fmaf(wa[0], va[0], s0);
      s1 = fmaf(wa[1], va[1], s1);
      s0 = fmaf(wb[0], vb[0], s0);
      s1 = fmaf(wb[1], vb[1], s1);
    }
  }
  const int ha = ha0 + ay, wa = wa0 + ax, hb = hb0 + by, wb = wb0 + bx;
  if (ha < hA && wa < wA && hb < hB && wb < wB)
    y[(long)blockIdx.z * NA * NB + (long)(ha * wA + wa) * NB + hb * wB + wb] = fmaxf((s0 + s1) + (ba[0] + bb[0]), 0.f);
}

// ---- persistent forms (round 4, second pass): the tile kernels above spent ~85 % of a wave's
// life outside the matrix pipe (PMC: SQ_VALU_MFMA_BUSY 40 % of the 10 -> 10 layer's time, a wave
// living 41 k cycles for 5.9 k of MFMA) -- each workgroup staged its tile, then loaded its weights
// (46 scattered loads per lane), then computed, with nothing to overlap the loads but the two
// other workgroups on the CU.  Here a workgroup stays resident over tiles t, t + G, t + 2G, ...:
// weights and per-lane LDS offsets are formed once, and the next tile's staging loads are issued
// into registers right after the current tile is stored to LDS, so they fly under its MFMAs.
// Same staged layout, same per-output fmaf chains (the K order below only changes which MFMA
// carries which (tap, channel) row: the f32 MFMA accumulates one product at a time, in K order,
// so the sums differ from the tile kernels' only in that order).
template <int CIN>
struct CmRegs {
  static constexpr int V = (CIN % 2 == 0) ? 2 : 1, VP = CIN / V;
  static constexpr int LA = CM_NH * CM_NT * VP, LB = CM_NT * CM_NH * VP;
  static constexpr int IA = (LA + 255) / 256, IB = (LB + 255) / 256;
  typedef float vec_t __attribute__((ext_vector_type(V)));
  vec_t ra[IA], rb[IB];
};

// tile t of the grid of (a tile, b tile, batch) -> its origin and input offset
struct CmTile {
  int ha0, wa0, hb0, wb0, z;
};
__device__ __forceinline__ CmTile cm_tile(int t, int nta, int ntb, int NTA, int NTB) {
  const int per = NTA * NTB;
  const int z = t / per, r = t - z * per;
  const int ta = r / NTB, tb = r - ta * NTB;
  return CmTile{(ta / nta) * CM_T, (ta % nta) * CM_T, (tb / ntb) * CM_T, (tb % ntb) * CM_T, z};
}

// Tile schedule of the persistent kernels.  order 0: workgroup w takes tiles w, w + G, ... of
// the (batch, a tile, b tile) order, b fastest.  order 1: the same order cut into 8 contiguous
// ranges, one per XCD (workgroup w runs on XCD w % 8 when G % 8 == 0), so the tiles that share
// staged data share an L2.  order 2: as 1, with the tiles visited by rows of b tiles, a tiles
// fastest within a row (the b-halo strip of a row is then streamed once per a tile, the a halo
// slides along wa inside one L2).
struct CmSched {
  int cur, end, step;
};
__device__ __forceinline__ CmSched cm_sched(int ntiles, int order) {
  if (order == 0 || (gridDim.x & 7)) return CmSched{(int)blockIdx.x, ntiles, (int)gridDim.x};
  const int xcd = blockIdx.x & 7, per = (ntiles + 7) / 8;
  return CmSched{xcd * per + (int)(blockIdx.x >> 3), min(ntiles, (xcd + 1) * per), (int)(gridDim.x >> 3)};
}
__device__ __forceinline__ int cm_order(int l, int order, int NTA, int NTB, int nbb) {
  if (order < 2) return l;
  const int per = NTA * NTB, z = l / per, r = l - z * per;
  const int full = (NTB / nbb) * nbb;
  int ta, tb;
  if (r < NTA * full) {
    const int blk = r / (NTA * nbb), rem = r - blk * NTA * nbb;
    ta = rem / nbb;
    tb = blk * nbb + rem % nbb;
  } else {
    const int r2 = r - NTA * full, nl = NTB - full;
    ta = r2 / nl;
    tb = full + r2 % nl;
  }
  return z * per + ta * NTB + tb;
}

template <int CIN>
__device__ __forceinline__ void cm_load(CmRegs<CIN>& R, const float* __restrict__ x, int hA, int wA, int hB, int wB,
                                        const CmTile& T) {
  using Rg = CmRegs<CIN>;
  typedef typename Rg::vec_t vec_t;
  constexpr int V = Rg::V, VP = Rg::VP;
  const int NB = hB * wB;
  const float* xz = x + (long)T.z * hA * wA * NB * CIN;
  const int t = threadIdx.x;
#pragma unroll
  for (int k = 0; k < Rg::IA; ++k) {
    int i = t + 256 * k;
    asm volatile("" : "+v"(i));  // re-derive the indices per tile: hoisted, 24 loads' worth held ~120 VGPRs
    const int q = i % VP, p = i / VP;
    const int bt = p % CM_NT, ah = p / CM_NT;
    const int ha = T.ha0 - 1 + ah / CM_H, wa = T.wa0 - 1 + ah % CM_H;
    const int hb = T.hb0 + bt / CM_T, wb = T.wb0 + bt % CM_T;
    const bool in = i < Rg::LA && (unsigned)ha < (unsigned)hA && (unsigned)wa < (unsigned)wA && hb < hB && wb < wB;
    R.ra[k] = in ? *(const vec_t*)(xz + (((long)(ha * wA + wa) * NB) + hb * wB + wb) * CIN + q * V) : vec_t(0.f);
  }
#pragma unroll
  for (int k = 0; k < Rg::IB; ++k) {
    int i = t + 256 * k;
    asm volatile("" : "+v"(i));
    const int q = i % VP, p = i / VP;
    const int bh = p % CM_NH, at = p / CM_NH;
    const int ha = T.ha0 + at / CM_T, wa = T.wa0 + at % CM_T;
    const int hb = T.hb0 - 1 + bh / CM_H, wb = T.wb0 - 1 + bh % CM_H;
    const bool in = i < Rg::LB && ha < hA && wa < wA && (unsigned)hb < (unsigned)hB && (unsigned)wb < (unsigned)wB;
    R.rb[k] = in ? *(const vec_t*)(xz + (((long)(ha * wA + wa) * NB) + hb * wB + wb) * CIN + q * V) : vec_t(0.f);
  }
}

template <int CIN>
__device__ __forceinline__ void cm_store(const CmRegs<CIN>& R, float* xa, float* xb) {
  using Rg = CmRegs<CIN>;
  typedef typename Rg::vec_t vec_t;
  const int t = threadIdx.x;
#pragma unroll
  for (int k = 0; k < Rg::IA; ++k) {
    const int i = t + 256 * k;
    if (i < Rg::LA) *(vec_t*)(xa + i * Rg::V) = R.ra[k];
  }
#pragma unroll
  for (int k = 0; k < Rg::IB; ++k) {
    const int i = t + 256 * k;
    if (i < Rg::LB) *(vec_t*)(xb + i * Rg::V) = R.rb[k];
  }
}

// K order of the persistent MFMA kernel (per branch): first the F = CIN / 4 full channel quads
// of every tap (MFMA m < 9 F: tap m / F, channels 4 (m % F) + g4 -- the four lane groups share the
// tap, so the LDS offset is the lane's base + an immediate), then the R = CIN % 4 leftover
// channels of PER = 4 / R taps per MFMA (lane group g4: tap i PER + g4 / R, channel 4F + g4 % R;
// offsets formed once into registers).  CIN = 10: 18 + 5 = 23 MFMAs (92 rows, as before).
template <int CIN>
struct CmK {
  static constexpr int F = CIN / 4, R = CIN % 4;
  static constexpr int PER = R ? 4 / R : 1;
  static constexpr int NFULL = 9 * F;
  // F even: the full quads of a tap go in MFMA pairs (2p, 2p + 1) whose lane group g4 takes the
  // ADJACENT channels 8 q + 2 g4 and 8 q + 2 g4 + 1 -- one ds_read_b64 feeds both MFMAs
  static constexpr bool PAIR = F % 2 == 0 && F > 0;
  static constexpr int NMIX = R ? (9 + PER - 1) / PER : 0;
  static constexpr int NM = NFULL + NMIX;
};
__device__ __forceinline__ constexpr int cm_toff(int tap) { return (tap / 3) * CM_H + tap % 3; }  // halo position

template <int CIN>
__global__ __launch_bounds__(256) void cp4d_mfma_persist_kernel(const float* __restrict__ x, int hA, int wA, int hB,
                                                                int wB, int ntiles, const float* __restrict__ Wa,
                                                                const float* __restrict__ ba,
                                                                const float* __restrict__ Wb,
                                                                const float* __restrict__ bb, float* __restrict__ y,
                                                                int dbg, int order) {
  constexpr int COUT = 10;
  using K = CmK<CIN>;
  constexpr int NM = K::NM, NMIX = K::NMIX;
  __shared__ __attribute__((aligned(16))) float xa[CmLds<CIN>::EA + 2];
  __shared__ __attribute__((aligned(16))) float xb[CmLds<CIN>::EB + 2];
  const int NA = hA * wA, NB = hB * wB;
  const int ntb = (wB + CM_T - 1) / CM_T, nta = (wA + CM_T - 1) / CM_T;
  const int NTB = ntb * ((hB + CM_T - 1) / CM_T), NTA = nta * ((hA + CM_T - 1) / CM_T);
  const int t = threadIdx.x, lane = t & 63, wv = __builtin_amdgcn_readfirstlane(t >> 6);
  const int r = lane & 15, g4 = lane >> 4;
  CmSched sc = cm_sched(ntiles, order);
  if (sc.cur >= sc.end) return;
  int tile = cm_order(sc.cur, order, NTA, NTB, ntb);
  CmRegs<CIN> R;
  cm_load<CIN>(R, x, hA, wA, hB, wB, cm_tile(tile, nta, ntb, NTA, NTB));
  // weights (B operand: column r = output channel) in this K order, and the mixed MFMAs' offsets
  float wra[NM], wrb[NM];
  int mixa[NMIX > 0 ? NMIX : 1], mixb[NMIX > 0 ? NMIX : 1];
#pragma unroll
  for (int m = 0; m < NM; ++m) {
    int tap, c;
    bool kin;
    if (m < K::NFULL && K::PAIR) {
      const int pp = m / 2, h = m % 2;
      tap = pp / (K::F / 2);
      c = 8 * (pp % (K::F / 2)) + 2 * g4 + h;
      kin = true;
    } else if (m < K::NFULL) {
      tap = m / K::F;
      c = 4 * (m % K::F) + g4;
      kin = true;
    } else {
      const int i = m - K::NFULL;
      tap = i * K::PER + g4 / (K::R ? K::R : 1);
      c = 4 * K::F + g4 % (K::R ? K::R : 1);
      kin = g4 / (K::R ? K::R : 1) < K::PER && tap < 9;
      if (!kin) tap = c = 0;
      mixa[i] = cm_toff(tap) * CM_NT * CIN + c;
      mixb[i] = cm_toff(tap) * CIN + c;
    }
    const bool live = kin && r < COUT;
    wra[m] = live ? Wa[(r * CIN + c) * 9 + tap] : 0.f;
    wrb[m] = live ? Wb[(r * CIN + c) * 9 + tap] : 0.f;
  }
  const float bias = r < COUT ? ba[r] + bb[r] : 0.f;
  // row r of group j: a tile position (wv, j), b tile position r = (by, bx)
  const int by = r / CM_T, bx = r % CM_T;
  const float* pa = xa + (wv * CM_H * CM_NT + r) * CIN;                // + j CM_NT CIN + offsets
  const float* pb = xb + (wv * CM_T * CM_NH + by * CM_H + bx) * CIN;   // + j CM_NH CIN + offsets
  for (;;) {
    const CmTile T = cm_tile(tile, nta, ntb, NTA, NTB);
    sc.cur += sc.step;
    const bool more = sc.cur < sc.end;
    tile = cm_order(more ? sc.cur : 0, order, NTA, NTB, ntb);
    __syncthreads();  // the previous tile's LDS reads are done
    cm_store<CIN>(R, xa, xb);
    __syncthreads();
    if (more && !(dbg & 2)) cm_load<CIN>(R, x, hA, wA, hB, wB, cm_tile(tile, nta, ntb, NTA, NTB));
    f32x4 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    typedef float f32x2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int m = 0; m < (K::PAIR ? K::NFULL : 0); m += 2) {
      if (dbg & 1) break;
      const int pp = m / 2, tap = pp / (K::F / 2), q8 = 8 * (pp % (K::F / 2)) + 2 * g4;
      const int oa = cm_toff(tap) * CM_NT * CIN + q8, ob = cm_toff(tap) * CIN + q8;
      f32x2 va[4], vb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        va[j] = *(const f32x2*)(pa + j * CM_NT * CIN + oa);
        vb[j] = *(const f32x2*)(pb + j * CM_NH * CIN + ob);
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(va[j][h], wra[m + h], acc[j], 0, 0, 0);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(vb[j][h], wrb[m + h], acc[j], 0, 0, 0);
      }
    }
#pragma unroll
    for (int m = K::PAIR ? K::NFULL : 0; m < NM; ++m) {
      if (dbg & 1) break;  // timing study: staging only (CWT_CP4D_DBG=1); 2: compute only
      int oa, ob;
      if (m < K::NFULL) {
        oa = cm_toff(m / K::F) * CM_NT * CIN + 4 * (m % K::F) + g4;
        ob = cm_toff(m / K::F) * CIN + 4 * (m % K::F) + g4;
      } else {
        oa = mixa[m - K::NFULL];
        ob = mixb[m - K::NFULL];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(pa[j * CM_NT * CIN + oa], wra[m], acc[j], 0, 0, 0);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(pb[j * CM_NH * CIN + ob], wrb[m], acc[j], 0, 0, 0);
    }
    // D: lane (col o = r, rows 4 g4 + i) -> pair (a = (wv, j), b = 4 g4 + i), channel o
    if (r < COUT) {
      float* yz = y + (long)T.z * NA * NB * COUT;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ha = T.ha0 + wv, wa = T.wa0 + j;
        if (ha >= hA || wa >= wA) continue;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int hb = T.hb0 + g4, wb = T.wb0 + i;
          if (hb < hB && wb < wB) yz[((long)(ha * wA + wa) * NB + hb * wB + wb) * COUT + r] = fmaxf(acc[j][i] + bias, 0.f);
        }
      }
    }
    if (!more) break;
  }
}

// COUT = 1, persistent: cp4d_c1_kernel's per-pair arithmetic over the same staged tiles
template <int CIN>
__global__ __launch_bounds__(256) void cp4d_c1_persist_kernel(const float* __restrict__ x, int hA, int wA, int hB,
                                                              int wB, int ntiles, const float* __restrict__ Wa,
                                                              const float* __restrict__ ba,
                                                              const float* __restrict__ Wb,
                                                              const float* __restrict__ bb, float* __restrict__ y,
                                                              int dbg, int order) {
  static_assert(CIN % 2 == 0, "pairs of channels");
  __shared__ __attribute__((aligned(16))) float xa[CmLds<CIN>::EA + 2];
  __shared__ __attribute__((aligned(16))) float xb[CmLds<CIN>::EB + 2];
  __shared__ __attribute__((aligned(16))) float wl[2][9][CIN];
  const int NA = hA * wA, NB = hB * wB;
  const int ntb = (wB + CM_T - 1) / CM_T, nta = (wA + CM_T - 1) / CM_T;
  const int NTB = ntb * ((hB + CM_T - 1) / CM_T), NTA = nta * ((hA + CM_T - 1) / CM_T);
  const int t = threadIdx.x;
  CmSched sc = cm_sched(ntiles, order);
  if (sc.cur >= sc.end) return;
  int tile = cm_order(sc.cur, order, NTA, NTB, ntb);
  CmRegs<CIN> R;
  cm_load<CIN>(R, x, hA, wA, hB, wB, cm_tile(tile, nta, ntb, NTA, NTB));
  if (t < 2 * 9 * CIN) {
    const int c = t % CIN, tap = (t / CIN) % 9, side = t / (9 * CIN);
    (&wl[0][0][0])[t] = (side ? Wb : Wa)[c * 9 + tap];
  }
  const float bias = ba[0] + bb[0];
  const int at = t / CM_NT, bt = t % CM_NT;
  const int ay = at / CM_T, ax = at % CM_T, by = bt / CM_T, bx = bt % CM_T;
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  for (;;) {
    const CmTile T = cm_tile(tile, nta, ntb, NTA, NTB);
    sc.cur += sc.step;
    const bool more = sc.cur < sc.end;
    tile = cm_order(more ? sc.cur : 0, order, NTA, NTB, ntb);
    __syncthreads();
    cm_store<CIN>(R, xa, xb);
    __syncthreads();
    if (more && !(dbg & 2)) cm_load<CIN>(R, x, hA, wA, hB, wB, cm_tile(tile, nta, ntb, NTA, NTB));
    float s0 = 0.f, s1 = 0.f;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      if (dbg & 1) break;
      const int ky = tap / 3, kx = tap % 3;
      const float* pa = &xa[(((ay + ky) * CM_H + ax + kx) * CM_NT + bt) * CIN];
      const float* pb = &xb[(at * CM_NH + (by + ky) * CM_H + bx + kx) * CIN];
#pragma unroll
      for (int c2 = 0; c2 < CIN / 2; ++c2) {
        const f32x2 va = *(const f32x2*)(pa + 2 * c2), vb = *(const f32x2*)(pb + 2 * c2);
        const f32x2 wa = *(const f32x2*)&wl[0][tap][2 * c2], wb = *(const f32x2*)&wl[1][tap][2 * c2];
        s0 = fmaf(wa[0], va[0], s0);
        s1 = fmaf(wa[1], va[1], s1);
        s0 = fmaf(wb[0], vb[0], s0);
        s1 = fmaf(wb[1], vb[1], s1);
      }
    }
    const int ha = T.ha0 + ay, wa = T.wa0 + ax, hb = T.hb0 + by, wb = T.wb0 + bx;
    if (ha < hA && wa < wA && hb < hB && wb < wB)
      y[(long)T.z * NA * NB + (long)(ha * wA + wa) * NB + hb * wB + wb] = fmaxf((s0 + s1) + bias, 0.f);
    if (!more) break;
  }
}

// ---- rolling-window form (round 4, third pass): the tile kernels above stage a cross-shaped
// box per 4x4-by-4x4 tile and so read every input 4.5 times (2.33 GB per 10 -> 10 layer at 60^2,
// 2.0 GB of it past the L2s: staging-bound).  Here a workgroup owns a 4 x 12 tile of
// b positions and a strip of 4 a rows, and walks the strip's a columns left to right: the window
// holds the 6 a rows (strip + halo) x 3 a columns of the b box (the tile + its 1-position ring,
// 6 x 14), so each step loads ONE new a column -- the a-plane convolution reads an input
// (4 + 2) / 4 times, the b-plane convolution only the ring around the tile (the tile itself is
// already in the window): ~2.2 reads per input.  The new column's loads are issued into
// registers before the current column's MFMAs and stored after them.  MFMA layout and K order
// as cp4d_mfma_persist_kernel (rows: 16 b positions of one a position; columns: the 10 outputs;
// CmK's K order); wave w takes a row w of the strip, its three groups the tile's 48 b positions.
// MODE 1: the input gradient (launch_cp4d_dgrad), as cp4d_mfma_kernel's MODE 1.
constexpr int RL_BH = 4, RL_BW = 12, RL_XH = RL_BH + 2, RL_XW = RL_BW + 2;
constexpr int RL_NT = RL_BH * RL_BW, RL_NX = RL_XH * RL_XW, RL_RA = 4, RL_ROWS = RL_RA + 2;
static_assert(RL_NT == 48, "three 16-row MFMA groups per a position");

// four column slots per a row (one barrier per step: the column stored in step wa is read from
// step wa + 1 on, into the slot last read in step wa - 1; three slots need a second barrier and
// measured 3 % slower)
template <int CIN>
struct RlWin {
  static constexpr int NS = 4;
  static constexpr int V = (CIN % 2 == 0) ? 2 : 1, VP = CIN / V;
  static constexpr int SLOT = RL_NX * CIN;        // floats of one (a row, column slot): the b box
  static constexpr int ROW = NS * SLOT;           // NS column slots per a row
  static constexpr int FLOATS = RL_ROWS * ROW;
  static constexpr int L = RL_ROWS * RL_NX * VP;  // loads per window column
  static constexpr int IL = (L + 255) / 256;
  static constexpr int LDS = FLOATS + (IL * 256 - L) * V + 4;  // + a dummy tail for the spare lanes
  typedef float vec_t __attribute__((ext_vector_type(V)));
};
constexpr int RL_OOR = 0x40000000;  // a buffer offset past every num_records: loads read 0, stores drop

// The window column's loads, branch-free: a buffer resource based at the column (num_records 0
// off the map), per-lane byte offsets out of range where the position is off the map or unused.
template <int CIN, int V, int IL, typename vec_t>
__device__ __forceinline__ void rl_load(vec_t (&rg)[IL], const int (&goff)[IL], const float* xz, int col, int wA,
                                        int NA, int NB) {
  const bool colin = (unsigned)col < (unsigned)wA;
  const float* base = xz + (colin ? (long)col * NB * CIN : 0L);
  const int nrec = colin ? (int)((long)(NA - col) * NB * CIN * 4) : 0;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, nrec, 0x00020000);
#pragma unroll
  for (int k = 0; k < IL; ++k) {
    if constexpr (V == 2) {
      typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
      const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rs, goff[k], 0, 0);
      rg[k] = __builtin_bit_cast(vec_t, v);
    } else {
      rg[k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, goff[k], 0, 0));
    }
  }
}

template <int CIN, int MODE, int PF>
__global__ __launch_bounds__(256) void cp4d_roll_kernel(const float* __restrict__ x, int hA, int wA, int hB, int wB,
                                                        int nsa, int wc, const float* __restrict__ Wa,
                                                        const float* __restrict__ ba, const float* __restrict__ Wb,
                                                        const float* __restrict__ bb, float* __restrict__ y,
                                                        int accum, int dbg) {
  constexpr int COUT = 10;
  using K = CmK<CIN>;
  using Wn = RlWin<CIN>;
  typedef typename Wn::vec_t vec_t;
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  constexpr int NM = K::NM, NMIX = K::NMIX, V = Wn::V, VP = Wn::VP;
  __shared__ __attribute__((aligned(16))) float win[Wn::LDS];
  const int NA = hA * wA, NB = hB * wB;
  const int ntbw = (wB + RL_BW - 1) / RL_BW;
  const int hb0 = ((int)blockIdx.x / ntbw) * RL_BH, wb0 = ((int)blockIdx.x % ntbw) * RL_BW;
  const int c0 = blockIdx.y * wc, c1 = min(wA, c0 + wc);
  const int z = blockIdx.z / nsa, ha0 = (blockIdx.z % nsa) * RL_RA;
  const float* xz = x + (long)z * NA * NB * CIN;
  float* yz = y + (long)z * NA * NB * COUT;
  const int t = threadIdx.x, lane = t & 63, wv = __builtin_amdgcn_readfirstlane(t >> 6);
  const int r = lane & 15, g4 = lane >> 4;
  // this thread's share of a window column: global offset at a column 0 (+ col NB CIN), -1 when
  // off the map or not needed (the ring of the two halo rows), and its LDS offset in a slot
  int goff[Wn::IL], loff[Wn::IL];
#pragma unroll
  for (int k = 0; k < Wn::IL; ++k) {
    const int i = t + 256 * k;
    const int q = i % VP, p = i / VP;
    const int pos = p % RL_NX, row = p / RL_NX;
    const int py = pos / RL_XW, px = pos % RL_XW;
    const int ha = ha0 - 1 + row, hb = hb0 - 1 + py, wb = wb0 - 1 + px;
    const bool ring = py == 0 || py == RL_XH - 1 || px == 0 || px == RL_XW - 1;
    const bool in = i < Wn::L && (!ring || (row >= 1 && row <= RL_RA)) && (unsigned)ha < (unsigned)hA &&
                    (unsigned)hb < (unsigned)hB && (unsigned)wb < (unsigned)wB;
    goff[k] = in ? (((ha * wA) * NB + hb * wB + wb) * CIN + q * V) * 4 : RL_OOR;
    loff[k] = i < Wn::L ? row * Wn::ROW + pos * CIN + q * V : Wn::FLOATS + (i - Wn::L) * V;
  }
  vec_t rg[Wn::IL];
  auto load = [&](int col) { rl_load<CIN, Wn::V, Wn::IL>(rg, goff, xz, col, wA, NA, NB); };
  auto store = [&](int slot) {
#pragma unroll
    for (int k = 0; k < Wn::IL; ++k) *(vec_t*)(win + (k < Wn::IL - 1 || loff[k] < Wn::FLOATS ? slot * Wn::SLOT : 0) + loff[k]) = rg[k];
  };
  load(c0 - 1);
  // weights (B operand: column r = output channel) in CmK's K order; the mixed MFMAs' offsets:
  // a plane (ky ROW + c) * 4 + kx (the column slot picked per step), b plane the box offset
  float wra[NM], wrb[NM];
  int mixa[NMIX > 0 ? NMIX : 1], mixb[NMIX > 0 ? NMIX : 1];
#pragma unroll
  for (int m = 0; m < NM; ++m) {
    int tap, c;
    bool kin;
    if (m < K::NFULL && K::PAIR) {
      const int pp = m / 2, h = m % 2;
      tap = pp / (K::F / 2);
      c = 8 * (pp % (K::F / 2)) + 2 * g4 + h;
      kin = true;
    } else if (m < K::NFULL) {
      tap = m / K::F;
      c = 4 * (m % K::F) + g4;
      kin = true;
    } else {
      const int i = m - K::NFULL;
      tap = i * K::PER + g4 / (K::R ? K::R : 1);
      c = 4 * K::F + g4 % (K::R ? K::R : 1);
      kin = g4 / (K::R ? K::R : 1) < K::PER && tap < 9;
      if (!kin) tap = c = 0;
      mixa[i] = ((tap / 3) * Wn::ROW + c) * 4 + tap % 3;
      mixb[i] = ((tap / 3 - 1) * RL_XW + tap % 3 - 1) * CIN + c;
    }
    const bool live = kin && r < COUT;
    const int wi = MODE == 0 ? (r * CIN + c) * 9 + tap : (c * COUT + r) * 9 + 8 - tap;
    wra[m] = live ? Wa[wi] : 0.f;
    wrb[m] = live ? Wb[wi] : 0.f;
  }
  const float bias = (MODE == 0 && r < COUT) ? ba[r] + bb[r] : 0.f;
  // group j's row r: tile b position 16 j + 4 (r % 4) + r / 4 -> its box position (times CIN); the
  // D rows 4 g4 + i of a lane are then the positions 16 j + 4 i + g4, so each of its stores covers
  // 4 consecutive b positions (160 contiguous bytes) instead of 4 positions 4 apart
  int pbj[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int tp = 16 * j + 4 * (r & 3) + (r >> 2);  // D row 4 g4 + i <-> tile position 16 j + 4 i + g4
    pbj[j] = ((tp / RL_BW + 1) * RL_XW + tp % RL_BW + 1) * CIN;
  }
  const float* wwin = win + wv * Wn::ROW;  // a row wv of the strip: window rows wv .. wv + 2
  const int ha = ha0 + wv;
  int yoff[3][4];  // byte offsets of this lane's outputs from column wa's base
#pragma unroll
  for (int j = 0; j < 3; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int tp = 16 * j + 4 * i + g4;  // one store instruction: 4 consecutive b positions x 10 outputs
      const int hb = hb0 + tp / RL_BW, wb = wb0 + tp % RL_BW;
      yoff[j][i] = (r < COUT && ha < hA && hb < hB && wb < wB) ? ((ha * wA * NB + hb * wB + wb) * COUT + r) * 4 : RL_OOR;
    }
  vec_t rg2[Wn::IL];
  auto load2 = [&](int col) { rl_load<CIN, Wn::V, Wn::IL>(rg2, goff, xz, col, wA, NA, NB); };
  auto store2 = [&](int slot) {
#pragma unroll
    for (int k = 0; k < Wn::IL; ++k) *(vec_t*)(win + (k < Wn::IL - 1 || loff[k] < Wn::FLOATS ? slot * Wn::SLOT : 0) + loff[k]) = rg2[k];
  };
  // step wa: publish column wa + 1 (barrier), store column wa + 2 into the slot of column wa - 2,
  // issue the loads of column wa + 1 + PF (PF = 2: two register sets, even / odd steps), compute
  // column wa from the slots of columns wa - 1, wa, wa + 1
  auto step = [&](int wa, auto&& st, auto&& ld) {
    const int s = (wa - c0) & 3;  // slot of column wa - 1
    __syncthreads();
    if (wa + 2 <= c1) st((s + 3) & 3);
    if (wa + 2 + PF <= c1 && !(dbg & 2)) ld(wa + 2 + PF);  // dbg (timing study): 2 no loads, 1 no arithmetic
    const int cb0 = s * Wn::SLOT, cb1 = ((s + 1) & 3) * Wn::SLOT, cb2 = ((s + 2) & 3) * Wn::SLOT;
    f32x4 acc[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int m = 0; m < (K::PAIR ? K::NFULL : 0); m += 2) {
      if (dbg & 1) break;
      const int pp = m / 2, tap = pp / (K::F / 2), q8 = 8 * (pp % (K::F / 2)) + 2 * g4;
      const int ky = tap / 3, kx = tap % 3;
      const int oa = ky * Wn::ROW + (kx == 0 ? cb0 : kx == 1 ? cb1 : cb2) + q8;
      const int ob = Wn::ROW + cb1 + ((ky - 1) * RL_XW + kx - 1) * CIN + q8;
      f32x2 va[3], vb[3];
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        va[j] = *(const f32x2*)(wwin + oa + pbj[j]);
        vb[j] = *(const f32x2*)(wwin + ob + pbj[j]);
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int j = 0; j < 3; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(va[j][h], wra[m + h], acc[j], 0, 0, 0);
#pragma unroll
        for (int j = 0; j < 3; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(vb[j][h], wrb[m + h], acc[j], 0, 0, 0);
      }
    }
#pragma unroll
    for (int m = K::PAIR ? K::NFULL : 0; m < NM; ++m) {
      if (dbg & 1) break;
      int oa, ob;
      if (m < K::NFULL) {
        const int tap = m / K::F, ky = tap / 3, kx = tap % 3, c = 4 * (m % K::F) + g4;
        oa = ky * Wn::ROW + (kx == 0 ? cb0 : kx == 1 ? cb1 : cb2) + c;
        ob = Wn::ROW + cb1 + ((ky - 1) * RL_XW + kx - 1) * CIN + c;
      } else {
        const int ma = mixa[m - K::NFULL], kx = ma & 3;
        oa = (ma >> 2) + (kx == 0 ? cb0 : kx == 1 ? cb1 : cb2);
        ob = Wn::ROW + cb1 + mixb[m - K::NFULL];
      }
#pragma unroll
      for (int j = 0; j < 3; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(wwin[oa + pbj[j]], wra[m], acc[j], 0, 0, 0);
#pragma unroll
      for (int j = 0; j < 3; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(wwin[ob + pbj[j]], wrb[m], acc[j], 0, 0, 0);
    }
    // D: lane (col o = r, rows 4 g4 + i) -> pair (a = (ha, wa), b = tile position 16 j + 4 g4 + i),
    // stored through a resource based at column wa (off-map pairs and dead columns: offset RL_OOR)
    {
      const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(yz + (long)wa * NB * COUT), (short)0, (int)((long)(NA - wa) * NB * COUT * 4), 0x00020000);
#pragma unroll
      for (int j = 0; j < 3; ++j) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float v = MODE == 0 ? fmaxf(acc[j][i] + bias, 0.f) : acc[j][i];
          if (MODE == 1 && accum)
            v += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ry, yoff[j][i], 0, 0));
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), ry, yoff[j][i], 0, 0);
        }
      }
    }
  };
  store(0);
  load(c0);
  store(1);
  load(c0 + 1);
  store(2);
  if (c0 + 2 <= c1) load(c0 + 2);
  if (PF == 2 && c0 + 3 <= c1) load2(c0 + 3);
  for (int wa = c0; wa < c1; wa += PF) {
    step(wa, store, load);
    if (PF == 2 && wa + 1 < c1) step(wa + 1, store2, load2);
  }
}

// COUT = 1 on the same rolling window (VALU: cp4d_c1_kernel's per-pair fmaf chains, the two
// branches' even / odd channels in two partial sums); thread t < 192 takes strip row t / 48 and
// tile b position t % 48; the filters are wave-uniform scalar loads (broadcast from LDS they made
// the kernel LDS-bound: 497 against 355 us at 60^2).
template <int CIN, int PF>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void cp4d_c1_roll_kernel(const float* __restrict__ x, int hA, int wA, int hB, int wB,
                                                           int nsa, int wc, const float* __restrict__ Wa,
                                                           const float* __restrict__ ba,
                                                           const float* __restrict__ Wb,
                                                           const float* __restrict__ bb, float* __restrict__ y,
                                                           int dbg) {
  static_assert(CIN % 2 == 0, "pairs of channels");
  using Wn = RlWin<CIN>;
  typedef typename Wn::vec_t vec_t;
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  constexpr int V = Wn::V, VP = Wn::VP;
  __shared__ __attribute__((aligned(16))) float win[Wn::LDS];
  const int NA = hA * wA, NB = hB * wB;
  const int ntbw = (wB + RL_BW - 1) / RL_BW;
  const int hb0 = ((int)blockIdx.x / ntbw) * RL_BH, wb0 = ((int)blockIdx.x % ntbw) * RL_BW;
  const int c0 = blockIdx.y * wc, c1 = min(wA, c0 + wc);
  const int z = blockIdx.z / nsa, ha0 = (blockIdx.z % nsa) * RL_RA;
  const float* xz = x + (long)z * NA * NB * CIN;
  float* yz = y + (long)z * NA * NB;
  const int t = threadIdx.x;
  int goff[Wn::IL], loff[Wn::IL];
#pragma unroll
  for (int k = 0; k < Wn::IL; ++k) {
    const int i = t + 256 * k;
    const int q = i % VP, p = i / VP;
    const int pos = p % RL_NX, row = p / RL_NX;
    const int py = pos / RL_XW, px = pos % RL_XW;
    const int ha = ha0 - 1 + row, hb = hb0 - 1 + py, wb = wb0 - 1 + px;
    const bool ring = py == 0 || py == RL_XH - 1 || px == 0 || px == RL_XW - 1;
    const bool in = i < Wn::L && (!ring || (row >= 1 && row <= RL_RA)) && (unsigned)ha < (unsigned)hA &&
                    (unsigned)hb < (unsigned)hB && (unsigned)wb < (unsigned)wB;
    goff[k] = in ? (((ha * wA) * NB + hb * wB + wb) * CIN + q * V) * 4 : RL_OOR;
    loff[k] = i < Wn::L ? row * Wn::ROW + pos * CIN + q * V : Wn::FLOATS + (i - Wn::L) * V;
  }
  vec_t rg[Wn::IL];
  auto load = [&](int col) { rl_load<CIN, Wn::V, Wn::IL>(rg, goff, xz, col, wA, NA, NB); };
  auto store = [&](int slot) {
#pragma unroll
    for (int k = 0; k < Wn::IL; ++k) *(vec_t*)(win + (k < Wn::IL - 1 || loff[k] < Wn::FLOATS ? slot * Wn::SLOT : 0) + loff[k]) = rg[k];
  };
  load(c0 - 1);
  const float bias = ba[0] + bb[0];
  const bool act = t < RL_RA * RL_NT;
  const int ai = act ? t / RL_NT : 0, tp = act ? t % RL_NT : 0;
  const int pb = ((tp / RL_BW + 1) * RL_XW + tp % RL_BW + 1) * CIN;
  const int ha = ha0 + ai, hb = hb0 + tp / RL_BW, wb = wb0 + tp % RL_BW;
  const bool outp = act && ha < hA && hb < hB && wb < wB;
  const int yoff = outp ? (ha * wA * NB + hb * wB + wb) * 4 : RL_OOR;  // from column wa's base
  const float* wwin = win + ai * Wn::ROW + pb;
  vec_t rg2[Wn::IL];
  auto load2 = [&](int col) { rl_load<CIN, Wn::V, Wn::IL>(rg2, goff, xz, col, wA, NA, NB); };
  auto store2 = [&](int slot) {
#pragma unroll
    for (int k = 0; k < Wn::IL; ++k) *(vec_t*)(win + (k < Wn::IL - 1 || loff[k] < Wn::FLOATS ? slot * Wn::SLOT : 0) + loff[k]) = rg2[k];
  };
  auto step = [&](int wa, auto&& st, auto&& ld) {  // as cp4d_roll_kernel's
    const int s = (wa - c0) & 3;
    __syncthreads();
    if (wa + 2 <= c1) st((s + 3) & 3);
    if (wa + 2 + PF <= c1 && !(dbg & 2)) ld(wa + 2 + PF);  // dbg (timing study): 2 no loads, 1 no arithmetic
    const int cb[3] = {s * Wn::SLOT, ((s + 1) & 3) * Wn::SLOT, ((s + 2) & 3) * Wn::SLOT};
    int wz = 0;
    asm volatile("" : "+s"(wz));  // the filters re-read per step as scalar loads (hoisted: 180 registers)
    const float* wga = Wa + wz;
    const float* wgb = Wb + wz;
    float s0 = 0.f, s1 = 0.f;
#pragma unroll 3
    for (int tap = 0; tap < 9; ++tap) {
      if (dbg & 1) break;
      const int ky = tap / 3, kx = tap % 3;
      const float* pa = wwin + ky * Wn::ROW + (kx == 0 ? cb[0] : kx == 1 ? cb[1] : cb[2]);
      const float* pbb = wwin + Wn::ROW + cb[1] + ((ky - 1) * RL_XW + kx - 1) * CIN;
#pragma unroll
      for (int c2 = 0; c2 < CIN / 2; ++c2) {
        const f32x2 va = *(const f32x2*)(pa + 2 * c2), vb = *(const f32x2*)(pbb + 2 * c2);
        const f32x2 w0 = {wga[(2 * c2) * 9 + tap], wga[(2 * c2 + 1) * 9 + tap]};
        const f32x2 w1 = {wgb[(2 * c2) * 9 + tap], wgb[(2 * c2 + 1) * 9 + tap]};
        s0 = fmaf(w0[0], va[0], s0);
        s1 = fmaf(w0[1], va[1], s1);
        s0 = fmaf(w1[0], vb[0], s0);
        s1 = fmaf(w1[1], vb[1], s1);
      }
    }
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(yz + (long)wa * NB), (short)0, (int)((long)(NA - wa) * NB * 4), 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, fmaxf((s0 + s1) + bias, 0.f)), ry, yoff, 0, 0);
  };
  store(0);
  load(c0);
  store(1);
  load(c0 + 1);
  store(2);
  if (c0 + 2 <= c1) load(c0 + 2);
  if (PF == 2 && c0 + 3 <= c1) load2(c0 + 3);
#pragma unroll 1
  for (int wa = c0; wa < c1; wa += PF) {
    step(wa, store, load);
    if (PF == 2 && wa + 1 < c1) step(wa + 1, store2, load2);
  }
}

// the rolling-window launch (cp4d_roll_kernel); returns 1 when the shape is not taken (index range)
// mode 0: COUT = 10 forward, 1: COUT = 10 input gradient, 2: COUT = 1 forward
static int launch_cp4d_roll(const float* x, int B, int hA, int wA, int hB, int wB, int cin, int mode, const float* Wa,
                            const float* ba, const float* Wb, const float* bb, float* y, int accum, hipStream_t st) {
  if ((long)hA * wA * hB * wB * 10 * 4 > RL_OOR) return 1;  // byte offsets within one batch entry below RL_OOR
  static const int wc_env = getenv("CWT_CP4D_WC") ? atoi(getenv("CWT_CP4D_WC")) : 30;
  const int wc = std::max(1, std::min(wA, wc_env));
  static const int dbg = getenv("CWT_CP4D_RDBG") ? atoi(getenv("CWT_CP4D_RDBG")) : 0;  // timing study only
  static const int pf = getenv("CWT_CP4D_PF") && atoi(getenv("CWT_CP4D_PF")) == 1 ? 1 : 2;  // prefetch depth
  const int nsa = cdiv(hA, RL_RA);
  const dim3 grid(cdiv(hB, RL_BH) * cdiv(wB, RL_BW), cdiv(wA, wc), B * nsa);
#define CWT_RL(CI, MD)                                                                                       \
  if (cin == CI && mode == MD) {                                                                             \
    if (pf == 1)                                                                                             \
      hipLaunchKernelGGL((cp4d_roll_kernel<CI, MD, 1>), grid, dim3(256), 0, st, x, hA, wA, hB, wB, nsa, wc, Wa, ba, \
                         Wb, bb, y, accum, dbg);                                                             \
    else                                                                                                     \
      hipLaunchKernelGGL((cp4d_roll_kernel<CI, MD, 2>), grid, dim3(256), 0, st, x, hA, wA, hB, wB, nsa, wc, Wa, ba, \
                         Wb, bb, y, accum, dbg);                                                             \
    CWT_LAUNCH_CHECK();                                                                                      \
    return 0;                                                                                                \
  }
  CWT_RL(1, 0)
  CWT_RL(2, 0)
  CWT_RL(10, 0)
  CWT_RL(1, 1)
  CWT_RL(10, 1)
#undef CWT_RL
  if (cin == 10 && mode == 2) {  // COUT = 1
    if (pf == 1)
      hipLaunchKernelGGL((cp4d_c1_roll_kernel<10, 1>), grid, dim3(256), 0, st, x, hA, wA, hB, wB, nsa, wc, Wa, ba, Wb,
                         bb, y, dbg);
    else
      hipLaunchKernelGGL((cp4d_c1_roll_kernel<10, 2>), grid, dim3(256), 0, st, x, hA, wA, hB, wB, nsa, wc, Wa, ba, Wb,
                         bb, y, dbg);
    CWT_LAUNCH_CHECK();
    return 0;
  }
  return 1;
}
// CWT_CP4D_ROLL: 0 never, 1 the COUT = 10 layers only, 2 (default) also COUT = 1 (its VALU form
// with the filters from scalar loads: 355 against the tile kernel's 482 us at 60^2)
static int cp4d_roll_mode() {
  static const int m = getenv("CWT_CP4D_ROLL") ? atoi(getenv("CWT_CP4D_ROLL")) : 2;
  return m;
}

// x [B][C][P] (channel planes) -> y [B][P][C] (channels last)
__global__ void to_channels_last_kernel(const float* __restrict__ x, int B, int C, long P, float* __restrict__ y) {
  const long total = (long)B * C * P;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int c = (int)(i % C);
    const long p = (i / C) % P;
    const long b = i / ((long)C * P);
    y[i] = x[(b * C + c) * P + p];
  }
}

// y += x (element count n)
__global__ void add_inplace_kernel(float* __restrict__ y, const float* __restrict__ x, long n) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) y[i] += x[i];
}

// softmax(temp * corr2d) over b, one workgroup per row a, written with row stride ldp (the pad
// columns zero): P[B][NA][ldp]
__global__ __launch_bounds__(256) void match_softmax_kernel(const float* __restrict__ corr, int NA, int NB, float temp,
                                                            int ldp, float* __restrict__ P) {
  const long row = blockIdx.x;  // b * NA + a
  const float* cr = corr + row * NB;
  float* pr = P + row * ldp;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  __shared__ float red[4];
  float m = -INFINITY;
  for (int j = t; j < NB; j += 256) m = fmaxf(m, cr[j] * temp);
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if (lane == 0) red[wv] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float s = 0.f;
  for (int j = t; j < NB; j += 256) s += __expf(cr[j] * temp - m);
  s = wave_sum_dpp(s);
  if (lane == 0) red[wv] = s;
  __syncthreads();
  const float inv = 1.f / ((red[0] + red[1]) + (red[2] + red[3]));
  for (int j = t; j < ldp; j += 256) pr[j] = j < NB ? __expf(cr[j] * temp - m) * inv : 0.f;
}

// v tokens [B][NB][C] -> vT [B][C][ldp] (pad columns zero)
__global__ __launch_bounds__(256) void match_vt_kernel(const float* __restrict__ v, int NB, int C, int ldp,
                                                       float* __restrict__ vt) {
  __shared__ float tile[32][33];
  const int b = blockIdx.z;
  const int j0 = blockIdx.x * 32, c0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  for (int r = ty; r < 32; r += 8) {
    const int j = j0 + r, c = c0 + tx;
    tile[r][tx] = (j < NB && c < C) ? v[((long)b * NB + j) * C + c] : 0.f;
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    const int c = c0 + r, j = j0 + tx;
    if (c < C && j < ldp) vt[((long)b * C + c) * ldp + j] = tile[tx][r];
  }
}

// ---- Conv4d ('cv4', src/model/conv4d.py:64-138) + ReLU, one NeighConsensus layer ----
// x, y channels last [B][hA wA][hB wB][C].  W is the reference's pre-permuted filter
// [k0][co][ci][k1][k2][k3] (Conv4d permutes it in its constructor), kernel 3, zero padding 1:
// y(i,j,k,l) = relu(bias + sum W[d0][co][ci][d1][d2][d3] x(i+d0-1, j+d1-1, k+d2-1, l+d3-1)), the
// per-slice conv3d sum of conv_4d.  swap = 1 applies the filter with (d0,d1) and (d2,d3)
// exchanged: conv(x^T)^T of the symmetric mode as one pass.  One thread per output position,
// every output channel; the filter tap-major in LDS (uniform broadcast reads).  fp32 VALU.
template <int CIN, int COUT>
__global__ __launch_bounds__(256) void cv4d_layer_kernel(const float* __restrict__ x, int B, int hA, int wA, int hB,
                                                         int wB, const float* __restrict__ W,
                                                         const float* __restrict__ bias, int swap,
                                                         float* __restrict__ y) {
  __shared__ float wl[81][CIN][COUT];
  for (int e = threadIdx.x; e < 81 * CIN * COUT; e += 256) {
    // e walks the stored layout [d0][co][ci][d1][d2][d3]
    const int d3 = e % 3, d2 = (e / 3) % 3, d1 = (e / 9) % 3;
    const int ci = (e / 27) % CIN, co = (e / (27 * CIN)) % COUT, d0 = e / (27 * CIN * COUT);
    const int tap = swap ? ((d2 * 3 + d3) * 3 + d0) * 3 + d1 : ((d0 * 3 + d1) * 3 + d2) * 3 + d3;
    wl[tap][ci][co] = W[e];
  }
  __syncthreads();
  const long NB = (long)hB * wB, P = (long)hA * wA * NB, total = (long)B * P;
  for (long q = (long)blockIdx.x * blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    const int b = (int)(q / P);
    const long pos = q - (long)b * P;
    const int l = (int)(pos % wB), k = (int)((pos / wB) % hB);
    const long pa = pos / NB;
    const int j = (int)(pa % wA), i = (int)(pa / wA);
    float acc[COUT];
#pragma unroll
    for (int co = 0; co < COUT; ++co) acc[co] = bias[co];
    for (int d0 = 0; d0 < 3; ++d0) {
      const int ii = i + d0 - 1;
      if ((unsigned)ii >= (unsigned)hA) continue;
      for (int d1 = 0; d1 < 3; ++d1) {
        const int jj = j + d1 - 1;
        if ((unsigned)jj >= (unsigned)wA) continue;
        for (int d2 = 0; d2 < 3; ++d2) {
          const int kk = k + d2 - 1;
          if ((unsigned)kk >= (unsigned)hB) continue;
#pragma unroll
          for (int d3 = 0; d3 < 3; ++d3) {
            const int ll = l + d3 - 1;
            if ((unsigned)ll >= (unsigned)wB) continue;
            const float* xp = x + ((long)b * P + ((long)ii * wA + jj) * NB + (long)kk * wB + ll) * CIN;
            const int tap = ((d0 * 3 + d1) * 3 + d2) * 3 + d3;
#pragma unroll
            for (int ci = 0; ci < CIN; ++ci) {
              const float xv = xp[ci];
#pragma unroll
              for (int co = 0; co < COUT; ++co) acc[co] = fmaf(wl[tap][ci][co], xv, acc[co]);
            }
          }
        }
      }
    }
    float* yp = y + q * COUT;
#pragma unroll
    for (int co = 0; co < COUT; ++co) yp[co] = fmaxf(acc[co], 0.f);
  }
}

// ---- Spatial context descriptor (src/model/base/spatial_context.py:13-65) ----
// x tokens [B][h][w][C]; g [B][h w][ldg]: g[o] = <x(p), x(p + offset o)> over the k x k window
// (zero outside the map), then featureL2Norm: g / sqrt(sum g^2 + 1e-6); columns k^2 .. ldg-1 zero.
// One workgroup per pixel: the pixel's feature in LDS, each wave one window offset at a time
// (lanes over channels, coalesced), the window in LDS for the norm.
constexpr int SCE_MAXK2 = 32 * 32;
__global__ __launch_bounds__(256) void sce_descriptor_kernel(const float* __restrict__ x, int h, int w, int C, int k,
                                                             int ldg, float* __restrict__ g) {
  extern __shared__ float sm_sce[];  // q [C], win [k*k]
  float* q = sm_sce;
  float* win = sm_sce + C;
  const long pix = blockIdx.x;  // b * h * w + y * w + xx
  const long hw = (long)h * w;
  const int b = (int)(pix / hw);
  const int yy = (int)((pix % hw) / w), xx = (int)(pix % w);
  const float* xb = x + (long)b * hw * C;
  for (int c = threadIdx.x; c < C; c += 256) q[c] = xb[((long)yy * w + xx) * C + c];
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, pad = k / 2, k2 = k * k;
  for (int o = wv; o < k2; o += 4) {
    const int ny = yy + o / k - pad, nx = xx + o % k - pad;
    float s = 0.f;
    if ((unsigned)ny < (unsigned)h && (unsigned)nx < (unsigned)w) {
      const float* xn = xb + ((long)ny * w + nx) * C;
      for (int c = lane; c < C; c += 64) s = fmaf(q[c], xn[c], s);
      s = wave_sum_dpp(s);
    }
    if (lane == 0) win[o] = s;
  }
  __syncthreads();
  float ss = 0.f;
  for (int o = threadIdx.x; o < k2; o += 256) ss = fmaf(win[o], win[o], ss);
  ss = wave_sum_dpp(ss);
  __shared__ float red[4];
  if (lane == 0) red[wv] = ss;
  __syncthreads();
  const float inv = 1.f / sqrtf(((red[0] + red[1]) + (red[2] + red[3])) + 1e-6f);
  float* gp = g + pix * ldg;
  for (int o = threadIdx.x; o < ldg; o += 256) gp[o] = o < k2 ? win[o] * inv : 0.f;
}

// ---- MMN agg 'sum' (mmn.py:62-63): y[b][p] = sum over l of x[b][l][p], l in order ----
__global__ void channel_sum_kernel(const float* __restrict__ x, int B, int L, long P, float* __restrict__ y) {
  const long total = (long)B * P;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int b = (int)(e / P);
    const long p = e - (long)b * P;
    const float* xb = x + (long)b * L * P + p;
    float s = xb[0];
    for (int l = 1; l < L; ++l) s += xb[(long)l * P];
    y[e] = s;
  }
}

// ---- MatchNet's support masks (match.py:117-126, run_cyc match.py:165-182) ----
// ig_mask [B][NB] (uint8, nullable): corr2d[b][a][j] = 1e-4 where ig_mask[b][j] (every query a).
// The cycle mask: k2q[j] = argmax over a of corr2d[a][j], q2k[a] = argmax over j of corr2d[a][j]
// (after the ig mask; first index on ties, as torch's max on the CPU), inconsistent[j] =
// s_mask[j] != s_mask[q2k[k2q[j]]], and corr2d += inconsistent[j] * -1000 (Dropout(0.1) of the
// mask is the identity in eval mode).
__device__ __forceinline__ float masked_corr(const float* cr, const uint8_t* ig, int j) {
  return (ig && ig[j]) ? 1e-4f : cr[j];
}

__device__ __forceinline__ void argmax_merge(float& v, int& i, float v2, int i2) {
  if (v2 > v || (v2 == v && i2 < i)) {
    v = v2;
    i = i2;
  }
}

// q2k: one workgroup per row (b, a)
__global__ __launch_bounds__(256) void match_row_argmax_kernel(const float* __restrict__ corr, const uint8_t* ig,
                                                               int NA, int NB, int* __restrict__ q2k) {
  const long row = blockIdx.x;  // b * NA + a
  const int b = (int)(row / NA);
  const float* cr = corr + row * NB;
  const uint8_t* igb = ig ? ig + (long)b * NB : nullptr;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  float v = -INFINITY;
  int idx = 0x7fffffff;
  for (int j = t; j < NB; j += 256) argmax_merge(v, idx, masked_corr(cr, igb, j), j);
  for (int o = 32; o > 0; o >>= 1) argmax_merge(v, idx, __shfl_xor(v, o, 64), __shfl_xor(idx, o, 64));
  __shared__ float rv[4];
  __shared__ int ri[4];
  if (lane == 0) {
    rv[wv] = v;
    ri[wv] = idx;
  }
  __syncthreads();
  if (t == 0) {
    for (int w = 1; w < 4; ++w) argmax_merge(v, idx, rv[w], ri[w]);
    q2k[row] = (idx >= 0 && idx < NB) ? idx : 0;  // an all-NaN row: keep the index in range
  }
}

// k2q partials: workgroup (column block of 64, row chunk, b); 4 waves stride the chunk's rows,
// lanes own columns; partial (value, index) per (b, chunk, column)
constexpr int MATCH_COL_CHUNKS = 16;
__global__ __launch_bounds__(256) void match_col_argmax_kernel(const float* __restrict__ corr, const uint8_t* ig,
                                                               int NA, int NB, float* __restrict__ pv,
                                                               int* __restrict__ pi) {
  const int b = blockIdx.z, chunk = blockIdx.y;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + lane;
  const int per = (NA + MATCH_COL_CHUNKS - 1) / MATCH_COL_CHUNKS;
  const int a0 = chunk * per, a1 = min(NA, a0 + per);
  float v = -INFINITY;
  int idx = 0x7fffffff;
  const bool masked = ig && j < NB && ig[(long)b * NB + j];
  if (j < NB)
    for (int a = a0 + wv; a < a1; a += 4) argmax_merge(v, idx, masked ? 1e-4f : corr[((long)b * NA + a) * NB + j], a);
  __shared__ float rv[4][64];
  __shared__ int ri[4][64];
  rv[wv][lane] = v;
  ri[wv][lane] = idx;
  __syncthreads();
  if (wv == 0 && j < NB) {
    for (int w = 1; w < 4; ++w) argmax_merge(v, idx, rv[w][lane], ri[w][lane]);
    const long o = ((long)b * MATCH_COL_CHUNKS + chunk) * NB + j;
    pv[o] = v;
    pi[o] = idx;
  }
}

// inconsistent[b][j] from the chunk partials, q2k and s_mask
__global__ void match_cyc_kernel(const float* __restrict__ pv, const int* __restrict__ pi, const int* __restrict__ q2k,
                                 const int64_t* __restrict__ s_mask, int B, int NA, int NB, float* __restrict__ incons) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long)B * NB) return;
  const int b = (int)(e / NB), j = (int)(e - (long)b * NB);
  float v = -INFINITY;
  int k2q = 0x7fffffff;
  for (int c = 0; c < MATCH_COL_CHUNKS; ++c) {
    const long o = ((long)b * MATCH_COL_CHUNKS + c) * NB + j;
    argmax_merge(v, k2q, pv[o], pi[o]);
  }
  if (k2q < 0 || k2q >= NA) k2q = 0;  // an all-NaN column: torch would return some index; keep it in range
  const int r = q2k[(long)b * NA + k2q];
  incons[e] = s_mask[(long)b * NB + j] != s_mask[(long)b * NB + r] ? 1.f : 0.f;
}

__global__ void match_mask_apply_kernel(float* __restrict__ corr, const uint8_t* ig, const float* incons, int B, int NA,
                                        int NB) {
  const long total = (long)B * NA * NB;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int j = (int)(e % NB);
    const int b = (int)(e / ((long)NA * NB));
    float v = corr[e];
    if (ig && ig[(long)b * NB + j]) v = 1e-4f;
    if (incons) v = v + incons[(long)b * NB + j] * -1000.f;
    corr[e] = v;
  }
}

// Train-mode Dropout(0.1) of the cycle mask (match.py:97 ass_drop, applied in run_cyc
// match.py:181): inconsistent[b][j] *= dropout_scale(p, seed, stream 5, b NB + j) -- kept entries
// become 1 / (1 - p), as nn.Dropout scales them; the mask is constant under autograd (argmax
// indices), so no gradient passes through it.
__global__ void match_cyc_dropout_kernel(float* __restrict__ incons, long n, float p, unsigned long long seed) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) incons[i] *= dropout_scale(p, seed, 5u, (unsigned long long)i);
}

// d corr2d[b][i][j] = 0 where ig_mask[b][j]: the masked entries were overwritten with the constant
// 1e-4 (match.py:117-119), so nothing flows back through them
__global__ void match_zero_ig_cols_kernel(float* __restrict__ g, const uint8_t* __restrict__ ig, int B, int NA, int NB) {
  const long total = (long)B * NA * NB;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int j = (int)(e % NB);
    const int b = (int)(e / ((long)NA * NB));
    if (ig[(long)b * NB + j]) g[e] = 0.f;
  }
}

int launch_match_zero_ig_cols(float* g, const uint8_t* ig, int B, int NA, int NB, hipStream_t st) {
  const long total = (long)B * NA * NB;
  hipLaunchKernelGGL(match_zero_ig_cols_kernel, dim3((unsigned)std::min<long>(65536, cdiv(total, 256))), dim3(256), 0, st,
                     g, ig, B, NA, NB);
  CWT_LAUNCH_CHECK();
  return 0;
}

// ---- WeightAverage (src/model/msm/msm_func.py:50-104), R = 3 ----
// tpg [N][P][3co]: theta | phi | g of every pixel (1x1 convs as one GEMM, biases not yet
// added); per pixel: cos_r = CosineSimilarity(phi(x_r), theta(x)) over its 3x3 replicate-padded
// neighbourhood r (torch: dot / (max(|phi|, 1e-8) max(|theta|, 1e-8))), softmax over the 9,
// wavg = sum_r softmax_r g(x_r).  One workgroup per pixel, co / 256 channels per thread.
template <int CPT>
__global__ __launch_bounds__(256) void wa_attn_kernel(const float* __restrict__ tpg, int h, int w, int co,
                                                      const float* __restrict__ bt, const float* __restrict__ bp,
                                                      const float* __restrict__ bg, float* __restrict__ wavg) {
  const long P = (long)h * w;
  const long pix = blockIdx.x;  // n * P + p
  const long n = pix / P;
  const int p = (int)(pix - n * P), y = p / w, x = p - y * w;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const long ld = 3L * co;
  __shared__ float red[4][19];
  __shared__ float sm[9];
  float th[CPT];
  const float* tp = tpg + pix * ld;
#pragma unroll
  for (int k = 0; k < CPT; ++k) th[k] = tp[t + 256 * k] + bt[t + 256 * k];
  float part[19];
  part[18] = 0.f;
#pragma unroll
  for (int k = 0; k < CPT; ++k) part[18] = fmaf(th[k], th[k], part[18]);
#pragma unroll
  for (int r = 0; r < 9; ++r) {
    const int yy = min(max(y + r / 3 - 1, 0), h - 1), xx = min(max(x + r % 3 - 1, 0), w - 1);
    const float* q = tpg + (n * P + (long)yy * w + xx) * ld + co;
    float d = 0.f, nn = 0.f;
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const float ph = q[t + 256 * k] + bp[t + 256 * k];
      d = fmaf(ph, th[k], d);
      nn = fmaf(ph, ph, nn);
    }
    part[r] = d;
    part[9 + r] = nn;
  }
#pragma unroll
  for (int i = 0; i < 19; ++i) {
    const float v = wave_sum_dpp(part[i]);
    if (lane == 0) red[wv][i] = v;
  }
  __syncthreads();
  if (t == 0) {
    float tot[19];
#pragma unroll
    for (int i = 0; i < 19; ++i) tot[i] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
    const float tn = fmaxf(sqrtf(tot[18]), 1e-8f);
    float cs[9], m = -INFINITY;
#pragma unroll
    for (int r = 0; r < 9; ++r) {
      cs[r] = tot[r] / (fmaxf(sqrtf(tot[9 + r]), 1e-8f) * tn);
      m = fmaxf(m, cs[r]);
    }
    float se = 0.f;
#pragma unroll
    for (int r = 0; r < 9; ++r) {
      cs[r] = expf(cs[r] - m);
      se += cs[r];
    }
#pragma unroll
    for (int r = 0; r < 9; ++r) sm[r] = cs[r] / se;
  }
  __syncthreads();
  float acc[CPT];
#pragma unroll
  for (int k = 0; k < CPT; ++k) acc[k] = 0.f;
#pragma unroll
  for (int r = 0; r < 9; ++r) {
    const int yy = min(max(y + r / 3 - 1, 0), h - 1), xx = min(max(x + r % 3 - 1, 0), w - 1);
    const float* q = tpg + (n * P + (long)yy * w + xx) * ld + 2 * co;
    const float a = sm[r];
#pragma unroll
    for (int k = 0; k < CPT; ++k) acc[k] = fmaf(a, q[t + 256 * k] + bg[t + 256 * k], acc[k]);
  }
#pragma unroll
  for (int k = 0; k < CPT; ++k) wavg[pix * co + t + 256 * k] = acc[k];
}

// out = x + (back + b): conv_back's bias and WeightAverage's residual (msm_func.py:99-104)
__global__ void wa_residual_kernel(const float* __restrict__ x, const float* __restrict__ back,
                                   const float* __restrict__ b, long n, int C, float* __restrict__ out) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    out[i] = x[i] + (back[i] + b[i % C]);
}

// MMN.forward's tail (mmn.py:65-67): att_mean = mean over the B support rows of att_fq;
// fq = f_q * (1 - att_wt) + att_mean * att_wt.  Tokens [B][P][C] / [P][C].
__global__ void mmn_blend_kernel(const float* __restrict__ fq_in, const float* __restrict__ att, int B, long n,
                                 float att_wt, float* __restrict__ att_mean, float* __restrict__ fq_out) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += att[(long)b * n + i];
    const float m = s / (float)B;
    att_mean[i] = m;
    fq_out[i] = fq_in[i] * (1.f - att_wt) + m * att_wt;
  }
}

int launch_wa_attn(const float* tpg, int N, int h, int w, int co, const float* bt, const float* bp, const float* bg,
                   float* wavg, hipStream_t st) {
  const dim3 grid((unsigned)((long)N * h * w));
  if (co == 256) hipLaunchKernelGGL((wa_attn_kernel<1>), grid, dim3(256), 0, st, tpg, h, w, co, bt, bp, bg, wavg);
  else if (co == 512) hipLaunchKernelGGL((wa_attn_kernel<2>), grid, dim3(256), 0, st, tpg, h, w, co, bt, bp, bg, wavg);
  else if (co == 1024) hipLaunchKernelGGL((wa_attn_kernel<4>), grid, dim3(256), 0, st, tpg, h, w, co, bt, bp, bg, wavg);
  else return fail(CWT_EARG, "WeightAverage: c_in / 2 must be 256, 512 or 1024");
  CWT_LAUNCH_CHECK();
  return 0;
}

int launch_wa_residual(const float* x, const float* back, const float* b, long n, int C, float* out, hipStream_t st) {
  hipLaunchKernelGGL(wa_residual_kernel, dim3((unsigned)std::min<long>(65536, cdiv(n, 256))), dim3(256), 0, st, x,
                     back, b, n, C, out);
  CWT_LAUNCH_CHECK();
  return 0;
}

int launch_mmn_blend(const float* fq_in, const float* att, int B, long n, float att_wt, float* att_mean, float* fq_out,
                     hipStream_t st) {
  hipLaunchKernelGGL(mmn_blend_kernel, dim3((unsigned)std::min<long>(65536, cdiv(n, 256))), dim3(256), 0, st, fq_in,
                     att, B, n, att_wt, att_mean, fq_out);
  CWT_LAUNCH_CHECK();
  return 0;
}

// the same on the torch layout x [B][2][NA][NB] (channel planes), y channels-last [B][NA][NB][2]: the
// transposition folded into the two passes over x (MatchNet's in_channel 2 correlation)
int launch_mutual_matching_planar2(const float* x, int B, int NA, int NB, float* y, float* rowmax, float* colpart,
                                   float* colmax, hipStream_t st) {
  const int nrbv = cdiv(NA, MM_RBV);
  hipLaunchKernelGGL((mm_rowcol_kernel<2, MM_RBV, true>), dim3(nrbv, B), dim3(256), 0, st, x, NA, NB, rowmax, colpart);
  CWT_LAUNCH_CHECK();
  hipLaunchKernelGGL(mm_colmax_kernel, dim3(cdiv(NB, 64), B * 2), dim3(256), 0, st, (const float*)colpart, nrbv, NB,
                     colmax);
  CWT_LAUNCH_CHECK();
  hipLaunchKernelGGL((mm_apply_kernel<2, true>), dim3(NA, B), dim3(256), 0, st, x, NA, NB, (const float*)rowmax,
                     (const float*)colmax, y);
  CWT_LAUNCH_CHECK();
  return 0;
}

// one channel, on the sum x + x2 of two [B][NA][NB] tensors (NeighConsensus' symmetric branches;
// the add the separate pass did, in the same order)
int launch_mutual_matching_sum(const float* x, const float* x2, int B, int NA, int NB, float* y, float* rowmax,
                               float* colpart, float* colmax, hipStream_t st) {
  const int nrbv = cdiv(NA, MM_RBV);
  hipLaunchKernelGGL((mm_rowcol_kernel<1>), dim3(nrbv, B), dim3(256), 0, st, x, NA, NB, rowmax, colpart, x2);
  CWT_LAUNCH_CHECK();
  hipLaunchKernelGGL(mm_colmax_kernel, dim3(cdiv(NB, 64), B), dim3(256), 0, st, (const float*)colpart, nrbv, NB,
                     colmax);
  CWT_LAUNCH_CHECK();
  hipLaunchKernelGGL((mm_apply_kernel<1>), dim3(NA, B), dim3(256), 0, st, x, NA, NB, (const float*)rowmax,
                     (const float*)colmax, y, x2);
  CWT_LAUNCH_CHECK();
  return 0;
}

int launch_mutual_matching(const float* x, int B, int NA, int NB, int C, float* y, float* rowmax, float* colpart,
                           float* colmax, hipStream_t st) {
  const int nrb = cdiv(NA, MM_RB);
  if (C != 1 && C != 2) {  // the scalar forms
    hipLaunchKernelGGL(mm_rowcol_any_kernel, dim3(nrb, B * C), dim3(256), 0, st, x, NA, NB, C, rowmax, colpart);
    CWT_LAUNCH_CHECK();
    hipLaunchKernelGGL(mm_colmax_kernel, dim3(cdiv(NB, 64), B * C), dim3(256), 0, st, (const float*)colpart, nrb,
                       NB, colmax);
    CWT_LAUNCH_CHECK();
    const long total = (long)B * NA * NB * C;
    hipLaunchKernelGGL(mm_apply_any_kernel, dim3((unsigned)std::min<long>(65536, cdiv(total, 256))), dim3(256), 0, st,
                       x, total, NA, NB, C, (const float*)rowmax, (const float*)colmax, y);
    CWT_LAUNCH_CHECK();
    return 0;
  }
  const int nrbv = cdiv(NA, MM_RBV);
  if (C == 1)
    hipLaunchKernelGGL((mm_rowcol_kernel<1>), dim3(nrbv, B), dim3(256), 0, st, x, NA, NB, rowmax, colpart);
  else
    hipLaunchKernelGGL((mm_rowcol_kernel<2>), dim3(nrbv, B), dim3(256), 0, st, x, NA, NB, rowmax, colpart);
  CWT_LAUNCH_CHECK();
  hipLaunchKernelGGL(mm_colmax_kernel, dim3(cdiv(NB, 64), B * C), dim3(256), 0, st, (const float*)colpart, nrbv, NB,
                     colmax);
  CWT_LAUNCH_CHECK();
  if (C == 1)
    hipLaunchKernelGGL(mm_apply_kernel<1>, dim3(NA, B), dim3(256), 0, st, x, NA, NB, (const float*)rowmax,
                       (const float*)colmax, y);
  else
    hipLaunchKernelGGL(mm_apply_kernel<2>, dim3(NA, B), dim3(256), 0, st, x, NA, NB, (const float*)rowmax,
                       (const float*)colmax, y);
  CWT_LAUNCH_CHECK();
  return 0;
}

// variant (cwt_debug_cp4d_layer): 0 the automatic choice, 1 never the rolling-window form, 2 only it
int launch_cp4d_layer_variant(const float* x, int B, int hA, int wA, int hB, int wB, int cin, int cout,
                              const float* Wa, const float* ba, const float* Wb, const float* bb, float* y, int variant,
                              hipStream_t st);
int launch_cp4d_layer(const float* x, int B, int hA, int wA, int hB, int wB, int cin, int cout, const float* Wa,
                      const float* ba, const float* Wb, const float* bb, float* y, hipStream_t st) {
  return launch_cp4d_layer_variant(x, B, hA, wA, hB, wB, cin, cout, Wa, ba, Wb, bb, y, 0, st);
}
int launch_cp4d_layer_variant(const float* x, int B, int hA, int wA, int hB, int wB, int cin, int cout,
                              const float* Wa, const float* ba, const float* Wb, const float* bb, float* y, int variant,
                              hipStream_t st) {
  // the matrix-core / register-blocked forms (round 4): for 10 -> 10 persistent workgroups with
  // the next tile's loads in flight (1,169 against 1,207 us at 60^2; the 2 -> 10 and 10 -> 1
  // layers measured slower that way: 331 / 605 against 297 / 471 us, profiles/r4/run_i), the
  // rest one tile per workgroup; CWT_CP4D_PERSIST=0 / 2: none / all persistent (A/B);
  // CWT_CP4D_MFMA=0 selects the scalar kernel
  static const bool mfma = !(getenv("CWT_CP4D_MFMA") && getenv("CWT_CP4D_MFMA")[0] == '0');
  if (((mfma && variant == 0 && (cp4d_roll_mode() == 2 || (cp4d_roll_mode() == 1 && cout == 10))) || variant == 2) &&
      (cout == 10 || cout == 1) &&
      launch_cp4d_roll(x, B, hA, wA, hB, wB, cin, cout == 10 ? 0 : 2, Wa, ba, Wb, bb, y, 0, st) == 0)
    return 0;
  if (variant == 2) return fail(CWT_EARG, "cp4d layer: no rolling-window form for this shape");
  static const int persist_mode = getenv("CWT_CP4D_PERSIST") ? atoi(getenv("CWT_CP4D_PERSIST")) : 1;
  const bool persist = persist_mode == 2 || (persist_mode == 1 && cin == 10 && cout == 10);
  if (mfma && persist) {
    const int ntiles = cdiv(hB, CM_T) * cdiv(wB, CM_T) * cdiv(hA, CM_T) * cdiv(wA, CM_T) * B;
    static const int dbg = getenv("CWT_CP4D_DBG") ? atoi(getenv("CWT_CP4D_DBG")) : 0;  // timing study only
    // cm_sched: order 1 cuts the 10 -> 10 layer's L2 misses 25 -> 15 M per launch at the same time
    static const int order = getenv("CWT_CP4D_ORDER") ? atoi(getenv("CWT_CP4D_ORDER")) : 1;
    int dev = 0, cu = 0;
    CWT_HIP(hipGetDevice(&dev));
    CWT_HIP(hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev));
#define CWT_CPP(CI, KERNEL)                                                                                  \
  if (cin == CI) {                                                                                           \
    static int occ = 0;                                                                                      \
    if (!occ) CWT_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (KERNEL<CI>), 256, 0));             \
    const int G = std::max(1, std::min(ntiles, std::max(1, occ) * cu));  /* a multiple of 8 when cu is */      \
    hipLaunchKernelGGL((KERNEL<CI>), dim3(G), dim3(256), 0, st, x, hA, wA, hB, wB, ntiles, Wa, ba, Wb, bb, y, dbg, order); \
    CWT_LAUNCH_CHECK();                                                                                      \
    return 0;                                                                                                \
  }
    if (cout == 10) {
      CWT_CPP(1, cp4d_mfma_persist_kernel)
      CWT_CPP(2, cp4d_mfma_persist_kernel)
      CWT_CPP(10, cp4d_mfma_persist_kernel)
    } else if (cout == 1) {
      CWT_CPP(10, cp4d_c1_persist_kernel)
    }
#undef CWT_CPP
  }
  if (mfma) {
    const dim3 g4(cdiv(hB, CM_T) * cdiv(wB, CM_T), cdiv(hA, CM_T) * cdiv(wA, CM_T), B);
#define CWT_CPM(CI, KERNEL)                                                                             \
  if (cin == CI) {                                                                                      \
    hipLaunchKernelGGL((KERNEL<CI>), g4, dim3(256), 0, st, x, hA, wA, hB, wB, Wa, ba, Wb, bb, y);       \
    CWT_LAUNCH_CHECK();                                                                                 \
    return 0;                                                                                           \
  }
    if (cout == 10) {
      CWT_CPM(1, cp4d_mfma_kernel)
      CWT_CPM(2, cp4d_mfma_kernel)
      CWT_CPM(10, cp4d_mfma_kernel)
    } else if (cout == 1) {
      CWT_CPM(10, cp4d_c1_kernel)
    }
#undef CWT_CPM
  }
  dim3 grid(cdiv(hB, CP_TBH) * cdiv(wB, CP_TBW), cdiv(hA, CP_TAH) * cdiv(wA, CP_TAW), B);
#define CWT_CP4D(CI, CO)                                                                                         \
  if (cin == CI && cout == CO) {                                                                                 \
    hipLaunchKernelGGL((cp4d_layer_kernel<CI, CO, 0>), grid, dim3(256), 0, st, x, hA, wA, hB, wB, Wa, ba, Wb, bb, y, 0); \
    CWT_LAUNCH_CHECK();                                                                                          \
    return 0;                                                                                                    \
  }
  CWT_CP4D(1, 10)
  CWT_CP4D(2, 10)
  CWT_CP4D(10, 10)
  CWT_CP4D(10, 1)
#undef CWT_CP4D
  return fail(CWT_EARG, "cp4d layer: channels (1|2 -> 10, 10 -> 10, 10 -> 1) only");
}

// the input gradient of one CenterPivotConv4d layer (cp4d_layer_kernel MODE 1): g [B][NA][NB][gin]
// is the layer's ReLU-masked output gradient, dx [B][NA][NB][gout] (gout = the layer's input
// channels), Wa / Wb the a-plane / b-plane filters the forward applied ([gin][gout][3][3])
int launch_cp4d_dgrad(const float* g, int B, int hA, int wA, int hB, int wB, int gin, int gout, const float* Wa,
                      const float* Wb, float* dx, int accum, hipStream_t st) {
  static const bool scalar = getenv("CWT_DGRAD_SCALAR") && getenv("CWT_DGRAD_SCALAR")[0] == '1';  // A/B only
  if (gout == 10 && (gin == 1 || gin == 10) && !scalar) {  // 10 output channels: the matrix-core form
    if (cp4d_roll_mode() != 0 &&
        launch_cp4d_roll(g, B, hA, wA, hB, wB, gin, 1, Wa, nullptr, Wb, nullptr, dx, accum, st) == 0)
      return 0;
    const dim3 g4(cdiv(hB, CM_T) * cdiv(wB, CM_T), cdiv(hA, CM_T) * cdiv(wA, CM_T), B);
    if (gin == 1)
      hipLaunchKernelGGL((cp4d_mfma_kernel<1, 1>), g4, dim3(256), 0, st, g, hA, wA, hB, wB, Wa, (const float*)nullptr,
                         Wb, (const float*)nullptr, dx, accum);
    else
      hipLaunchKernelGGL((cp4d_mfma_kernel<10, 1>), g4, dim3(256), 0, st, g, hA, wA, hB, wB, Wa, (const float*)nullptr,
                         Wb, (const float*)nullptr, dx, accum);
    CWT_LAUNCH_CHECK();
    return 0;
  }
  dim3 grid(cdiv(hB, CP_TBH) * cdiv(wB, CP_TBW), cdiv(hA, CP_TAH) * cdiv(wA, CP_TAW), B);
#define CWT_CPD(CI, CO)                                                                                     \
  if (gin == CI && gout == CO) {                                                                            \
    hipLaunchKernelGGL((cp4d_layer_kernel<CI, CO, 1>), grid, dim3(256), 0, st, g, hA, wA, hB, wB, Wa,       \
                       (const float*)nullptr, Wb, (const float*)nullptr, dx, accum);                        \
    CWT_LAUNCH_CHECK();                                                                                     \
    return 0;                                                                                               \
  }
  CWT_CPD(1, 10)
  CWT_CPD(10, 10)
  CWT_CPD(10, 1)
  CWT_CPD(10, 2)
#undef CWT_CPD
  return fail(CWT_EARG, "cp4d input gradient: channels (1 -> 10, 10 -> 10, 10 -> 1|2) only");
}

int launch_to_channels_last(const float* x, int B, int C, long P, float* y, hipStream_t st) {
  const long n = (long)B * C * P;
  hipLaunchKernelGGL(to_channels_last_kernel, dim3((unsigned)std::min<long>(65536, cdiv(n, 256))), dim3(256), 0, st, x,
                     B, C, P, y);
  CWT_LAUNCH_CHECK();
  return 0;
}

int launch_add_inplace(float* y, const float* x, long n, hipStream_t st) {
  hipLaunchKernelGGL(add_inplace_kernel, dim3((unsigned)std::min<long>(65536, cdiv(n, 256))), dim3(256), 0, st, y, x, n);
  CWT_LAUNCH_CHECK();
  return 0;
}

int launch_match_softmax(const float* corr, int B, int NA, int NB, float temp, int ldp, float* P, hipStream_t st) {
  hipLaunchKernelGGL(match_softmax_kernel, dim3(B * NA), dim3(256), 0, st, corr, NA, NB, temp, ldp, P);
  CWT_LAUNCH_CHECK();
  return 0;
}

int launch_match_vt(const float* v, int B, int NB, int C, int ldp, float* vt, hipStream_t st) {
  hipLaunchKernelGGL(match_vt_kernel, dim3(cdiv(ldp, 32), cdiv(C, 32), B), dim3(256), 0, st, v, NB, C, ldp, vt);
  CWT_LAUNCH_CHECK();
  return 0;
}

int launch_match_masks(float* corr, int B, int NA, int NB, const uint8_t* ig, const int64_t* s_mask, float* incons,
                       int* q2k, float* pv, int* pi, hipStream_t st, float drop_p, unsigned long long seed) {
  if (s_mask) {
    hipLaunchKernelGGL(match_row_argmax_kernel, dim3(B * NA), dim3(256), 0, st, (const float*)corr, ig, NA, NB, q2k);
    CWT_LAUNCH_CHECK();
    hipLaunchKernelGGL(match_col_argmax_kernel, dim3(cdiv(NB, 64), MATCH_COL_CHUNKS, B), dim3(256), 0, st,
                       (const float*)corr, ig, NA, NB, pv, pi);
    CWT_LAUNCH_CHECK();
    hipLaunchKernelGGL(match_cyc_kernel, dim3(cdiv((long)B * NB, 256)), dim3(256), 0, st, (const float*)pv,
                       (const int*)pi, (const int*)q2k, s_mask, B, NA, NB, incons);
    CWT_LAUNCH_CHECK();
    if (drop_p > 0.f) {
      hipLaunchKernelGGL(match_cyc_dropout_kernel, dim3(cdiv((long)B * NB, 256)), dim3(256), 0, st, incons, (long)B * NB,
                         drop_p, seed);
      CWT_LAUNCH_CHECK();
    }
  }
  if (ig || s_mask) {
    const long total = (long)B * NA * NB;
    hipLaunchKernelGGL(match_mask_apply_kernel, dim3((unsigned)std::min<long>(65536, cdiv(total, 256))), dim3(256), 0,
                       st, corr, ig, s_mask ? (const float*)incons : (const float*)nullptr, B, NA, NB);
    CWT_LAUNCH_CHECK();
  }
  return 0;
}

int launch_cv4d_layer(const float* x, int B, int hA, int wA, int hB, int wB, int cin, int cout, const float* W,
                      const float* bias, int swap, float* y, hipStream_t st) {
  const long total = (long)B * hA * wA * hB * wB;
  const dim3 grid((unsigned)std::min<long>(65536, cdiv(total, 256)));
#define CWT_CV4D(CI, CO)                                                                                      \
  if (cin == CI && cout == CO) {                                                                              \
    hipLaunchKernelGGL((cv4d_layer_kernel<CI, CO>), grid, dim3(256), 0, st, x, B, hA, wA, hB, wB, W, bias, swap, y); \
    CWT_LAUNCH_CHECK();                                                                                       \
    return 0;                                                                                                 \
  }
  CWT_CV4D(1, 10)
  CWT_CV4D(2, 10)
  CWT_CV4D(10, 10)
  CWT_CV4D(10, 1)
#undef CWT_CV4D
  return fail(CWT_EARG, "cv4d layer: channels (1|2 -> 10, 10 -> 10, 10 -> 1) only");
}

int launch_sce_descriptor(const float* x, int B, int h, int w, int C, int k, int ldg, float* g, hipStream_t st) {
  if (k < 1 || k % 2 == 0 || k * k > SCE_MAXK2 || ldg < k * k) return fail(CWT_EARG, "sce: odd kernel size, k*k <= 1024");
  const size_t lds = (size_t)(C + k * k) * 4;
  if (lds > 64 * 1024) return fail(CWT_EARG, "sce: C + k*k floats must fit 64 KB of LDS");
  hipLaunchKernelGGL(sce_descriptor_kernel, dim3((unsigned)((long)B * h * w)), dim3(256), lds, st, x, h, w, C, k, ldg, g);
  CWT_LAUNCH_CHECK();
  return 0;
}

int launch_channel_sum(const float* x, int B, int L, long P, float* y, hipStream_t st) {
  const long total = (long)B * P;
  hipLaunchKernelGGL(channel_sum_kernel, dim3((unsigned)std::min<long>(65536, cdiv(total, 256))), dim3(256), 0, st, x, B,
                     L, P, y);
  CWT_LAUNCH_CHECK();
  return 0;
}

}  // namespace cwt

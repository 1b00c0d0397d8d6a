// Backward of MatchNet's corr_forward chain and of the MMN head's WeightAverage / get_corr
// (VERDICT r3 item 6): reference src/model/match.py:21-163 (MutualMatching,
// NeighConsensus, corr_forward), src/model/conv4d.py:40-62 (CenterPivotConv4d),
// src/model/msm/msm_func.py:66-104 (WeightAverage), src/model/model_util.py:101-109 (get_corr),
// src/model/mmn.py:65-67 (the blend) -- the modules MMN (train_cca.py:101, train_aug.py:102) and
// DeTr's cross attention (train_trans.py:100) train through.
//
// Exact fp32; every reduction runs in a fixed order (no atomics), so a backward is deterministic.
// Layouts are the forward's (match.hip): 4-D tensors channels-last [B][a][b][C], a = (ha, wa),
// b = (hb, wb); WeightAverage's tpg [N·P][3co] = theta | phi | g before their biases.
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace cwt {

// ---- MutualMatching (match.py:34-53) backward, per channel of x[B][NA][NB][C] ----
// forward: u[a] = max_b x[a][b] + eps, v[b] = max_a x[a][b] + eps, y = x * ((x / u) * (x / v)).
// torch.max sends a maximum's gradient to ONE index (here the first maximal position), so
//   dx = dy * (x/u * x/v + x * (x/v / u + x/u / v))
//        - [b == argmax over b of row a] * sum_b' dy y / u[a]
//        - [a == argmax over a of column b] * sum_a' dy y / v[b].
constexpr int MB_RB = 16;  // rows of a per workgroup

__device__ __forceinline__ void argmax_merge(float& v, int& i, float v2, int i2) {
  if (v2 > v || (v2 == v && i2 < i)) {
    v = v2;
    i = i2;
  }
}

// row (max, first argmax) and per-row-block column partial (max, first argmax)
__global__ __launch_bounds__(256) void mmb_rowcol_kernel(const float* __restrict__ x, int NA, int NB, int C,
                                                         float* __restrict__ rowmax, int* __restrict__ rowarg,
                                                         float* __restrict__ colpv, int* __restrict__ colpi) {
  const int bc = blockIdx.y, b = bc / C, c = bc - b * C;
  const int a0 = blockIdx.x * MB_RB;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const float* xb = x + (long)b * NA * NB * C + c;
  __shared__ float sv[4][MB_RB];
  __shared__ int si[4][MB_RB];
  float rv[MB_RB];
  int ri[MB_RB];
#pragma unroll
  for (int r = 0; r < MB_RB; ++r) {
    rv[r] = -INFINITY;
    ri[r] = NB;
  }
  for (int j = t; j < NB; j += 256) {
    float cv = -INFINITY;
    int ci = NA;
#pragma unroll
    for (int r = 0; r < MB_RB; ++r) {
      const int a = a0 + r;
      if (a < NA) {
        const float v = xb[((long)a * NB + j) * C];
        if (v > cv) {
          cv = v;
          ci = a;
        }
        if (v > rv[r]) {
          rv[r] = v;
          ri[r] = j;
        }
      }
    }
    colpv[((long)bc * gridDim.x + blockIdx.x) * NB + j] = cv;
    colpi[((long)bc * gridDim.x + blockIdx.x) * NB + j] = ci;
  }
#pragma unroll
  for (int r = 0; r < MB_RB; ++r) {
    float v = rv[r];
    int i = ri[r];
    for (int o = 32; o > 0; o >>= 1) argmax_merge(v, i, __shfl_xor(v, o, 64), __shfl_xor(i, o, 64));
    if (lane == 0) {
      sv[wv][r] = v;
      si[wv][r] = i;
    }
  }
  __syncthreads();
  if (t < MB_RB && a0 + t < NA) {
    float v = sv[0][t];
    int i = si[0][t];
    for (int q = 1; q < 4; ++q) argmax_merge(v, i, sv[q][t], si[q][t]);
    rowmax[(long)bc * NA + a0 + t] = v;
    rowarg[(long)bc * NA + a0 + t] = i;
  }
}

__global__ __launch_bounds__(256) void mmb_colred_kernel(const float* __restrict__ colpv, const int* __restrict__ colpi,
                                                         int nrb, int NB, float* __restrict__ colmax,
                                                         int* __restrict__ colarg) {
  const int bc = blockIdx.y;
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= NB) return;
  float v = -INFINITY;
  int i = 0x7fffffff;
  for (int rb = 0; rb < nrb; ++rb)
    argmax_merge(v, i, colpv[((long)bc * nrb + rb) * NB + j], colpi[((long)bc * nrb + rb) * NB + j]);
  colmax[(long)bc * NB + j] = v;
  colarg[(long)bc * NB + j] = i;
}

// srow[a] = sum_b dy y over the row; scolp[row block][b] = the block's partial column sums
__global__ __launch_bounds__(256) void mmb_sums_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                       int NA, int NB, int C, const float* __restrict__ rowmax,
                                                       const float* __restrict__ colmax, float* __restrict__ srow,
                                                       float* __restrict__ scolp) {
  const float eps = 1e-5f;
  const int bc = blockIdx.y, b = bc / C, c = bc - b * C;
  const int a0 = blockIdx.x * MB_RB;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const long base = (long)b * NA * NB * C + c;
  __shared__ float red[4][MB_RB];
  float rs[MB_RB];
#pragma unroll
  for (int r = 0; r < MB_RB; ++r) rs[r] = 0.f;
  float u[MB_RB];
#pragma unroll
  for (int r = 0; r < MB_RB; ++r) u[r] = a0 + r < NA ? rowmax[(long)bc * NA + a0 + r] + eps : 1.f;
  for (int j = t; j < NB; j += 256) {
    const float vb_den = colmax[(long)bc * NB + j] + eps;
    float cs = 0.f;
#pragma unroll
    for (int r = 0; r < MB_RB; ++r) {
      const int a = a0 + r;
      if (a < NA) {
        const long i = base + ((long)a * NB + j) * C;
        const float v = x[i];
        const float y = v * ((v / u[r]) * (v / vb_den));
        const float p = dy[i] * y;
        rs[r] += p;
        cs += p;
      }
    }
    scolp[((long)bc * gridDim.x + blockIdx.x) * NB + j] = cs;
  }
#pragma unroll
  for (int r = 0; r < MB_RB; ++r) {
    const float v = wave_sum_dpp(rs[r]);
    if (lane == 0) red[wv][r] = v;
  }
  __syncthreads();
  if (t < MB_RB && a0 + t < NA) srow[(long)bc * NA + a0 + t] = (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
}

__global__ __launch_bounds__(256) void mmb_colsum_kernel(const float* __restrict__ scolp, int nrb, int NB,
                                                         float* __restrict__ scol) {
  const int bc = blockIdx.y;
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= NB) return;
  float s = 0.f;
  for (int rb = 0; rb < nrb; ++rb) s += scolp[((long)bc * nrb + rb) * NB + j];
  scol[(long)bc * NB + j] = s;
}

__global__ __launch_bounds__(256) void mmb_apply_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                        long total, int NA, int NB, int C,
                                                        const float* __restrict__ rowmax, const int* __restrict__ rowarg,
                                                        const float* __restrict__ colmax, const int* __restrict__ colarg,
                                                        const float* __restrict__ srow, const float* __restrict__ scol,
                                                        float* __restrict__ dx) {
  const float eps = 1e-5f;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int c = (int)(i % C);
    const long p = i / C;
    const int j = (int)(p % NB);
    const long ab = p / NB;
    const int a = (int)(ab % NA), b = (int)(ab / NA);
    const int bc = b * C + c;
    const float u = rowmax[(long)bc * NA + a] + eps, w = colmax[(long)bc * NB + j] + eps;
    const float v = x[i], g = dy[i];
    const float va = v / u, vb = v / w;
    float d = g * (va * vb + v * (vb / u + va / w));
    if (j == rowarg[(long)bc * NA + a]) d -= srow[(long)bc * NA + a] / u;
    if (a == colarg[(long)bc * NB + j]) d -= scol[(long)bc * NB + j] / w;
    dx[i] = d;
  }
}

int launch_mutual_matching_bwd(const float* x, const float* dy, int B, int NA, int NB, int C, float* dx,
                               const MmBwdWs& ws, hipStream_t st) {
  const int nrb = cdiv(NA, MB_RB);
  hipLaunchKernelGGL(mmb_rowcol_kernel, dim3(nrb, B * C), dim3(256), 0, st, x, NA, NB, C, ws.rowmax, ws.rowarg, ws.colpv,
                     ws.colpi);
  CWT_LAUNCH_CHECK();
  hipLaunchKernelGGL(mmb_colred_kernel, dim3(cdiv(NB, 256), B * C), dim3(256), 0, st, (const float*)ws.colpv,
                     (const int*)ws.colpi, nrb, NB, ws.colmax, ws.colarg);
  CWT_LAUNCH_CHECK();
  hipLaunchKernelGGL(mmb_sums_kernel, dim3(nrb, B * C), dim3(256), 0, st, x, dy, NA, NB, C, (const float*)ws.rowmax,
                     (const float*)ws.colmax, ws.srow, ws.colpv);
  CWT_LAUNCH_CHECK();
  hipLaunchKernelGGL(mmb_colsum_kernel, dim3(cdiv(NB, 256), B * C), dim3(256), 0, st, (const float*)ws.colpv, nrb, NB,
                     ws.scol);
  CWT_LAUNCH_CHECK();
  const long total = (long)B * NA * NB * C;
  hipLaunchKernelGGL(mmb_apply_kernel, dim3((unsigned)std::min<long>(65536, cdiv(total, 256))), dim3(256), 0, st, x, dy,
                     total, NA, NB, C, (const float*)ws.rowmax, (const int*)ws.rowarg, (const float*)ws.colmax,
                     (const int*)ws.colarg, (const float*)ws.srow, (const float*)ws.scol, dx);
  CWT_LAUNCH_CHECK();
  return 0;
}

// ---- ReLU backward: gm = g * (out > 0) (torch's threshold_backward on the ReLU's result) ----
__global__ void relu_mask_kernel(const float* __restrict__ g, const float* __restrict__ out, long n,
                                 float* __restrict__ gm) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    gm[i] = out[i] > 0.f ? g[i] : 0.f;
}

int launch_relu_mask(const float* g, const float* out, long n, float* gm, hipStream_t st) {
  hipLaunchKernelGGL(relu_mask_kernel, dim3((unsigned)std::min<long>(65536, cdiv(n, 256))), dim3(256), 0, st, g, out, n,
                     gm);
  CWT_LAUNCH_CHECK();
  return 0;
}

// ---- CenterPivotConv4d weight / bias gradients (conv4d.py:40-62) ----
// dWa[o][c][tap] = sum over (a, b) of gm[a][b][o] x[a + tap - 1][b][c] (zero padding), dWb the
// same over the b plane, db[o] = sum gm[a][b][o] (conv1's and conv2's biases both).  Workgroups
// stride over 2x8 (a) by 2x8 (b) tiles, stage the tile's cross-shaped input and its gradient in
// LDS, and keep their partial sums in registers: thread = one (side, tap, o) entry with CIN
// accumulators, 256 / (18 COUT) thread groups over the tile's 256 pairs.  Partials per
// workgroup [G][18 COUT CIN + COUT], summed in workgroup order by cp4d_wgrad_reduce_kernel.
constexpr int WG_TAH = 2, WG_TAW = 8, WG_TBH = 2, WG_TBW = 8;
constexpr int WG_NA = WG_TAH * WG_TAW, WG_NB = WG_TBH * WG_TBW;
constexpr int WG_HA = (WG_TAH + 2) * (WG_TAW + 2), WG_HB = (WG_TBH + 2) * (WG_TBW + 2);

template <int CIN, int COUT>
__global__ __launch_bounds__(256) void cp4d_wgrad_kernel(const float* __restrict__ x, const float* __restrict__ gm,
                                                         int B, int hA, int wA, int hB, int wB,
                                                         float* __restrict__ part) {
  constexpr int NE = 18 * COUT;
  constexpr int NG = 256 / NE;
  static_assert(NG >= 1, "COUT <= 14");
  __shared__ float xa[WG_HA][WG_NB][CIN];
  __shared__ float xb[WG_NA][WG_HB][CIN];
  __shared__ float gl[WG_NA * WG_NB][COUT];
  __shared__ float red[NG * NE][CIN + 1];
  const int NA = hA * wA, NB = hB * wB;
  const int t = threadIdx.x;
  const int e = t % NE, grp = t / NE;
  const bool active = grp < NG;
  const int side = e / (9 * COUT), tap = (e / COUT) % 9, o = e % COUT;
  const int ky = tap / 3, kx = tap - 3 * (tap / 3);
  float acc[CIN];
#pragma unroll
  for (int c = 0; c < CIN; ++c) acc[c] = 0.f;
  float bacc = 0.f;
  const int ntaw = (wA + WG_TAW - 1) / WG_TAW, ntah = (hA + WG_TAH - 1) / WG_TAH;
  const int ntbw = (wB + WG_TBW - 1) / WG_TBW, ntbh = (hB + WG_TBH - 1) / WG_TBH;
  const long ntb = (long)ntbh * ntbw, nta = (long)ntah * ntaw, ntiles = (long)B * nta * ntb;
  for (long tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const long tb = tile % ntb, rest = tile / ntb;
    const long ta = rest % nta, bz = rest / nta;
    const int ha0 = (int)(ta / ntaw) * WG_TAH, wa0 = (int)(ta % ntaw) * WG_TAW;
    const int hb0 = (int)(tb / ntbw) * WG_TBH, wb0 = (int)(tb % ntbw) * WG_TBW;
    const float* xz = x + bz * NA * NB * CIN;
    const float* gz = gm + bz * NA * NB * COUT;
    __syncthreads();  // the previous tile's LDS reads are done
    for (int i = t; i < WG_HA * WG_NB * CIN; i += 256) {  // a halo box at the tile's b positions
      const int c = i % CIN, p = i / CIN;
      const int bi = p % WG_NB, ai = p / WG_NB;
      const int ha = ha0 - 1 + ai / (WG_TAW + 2), wa = wa0 - 1 + ai % (WG_TAW + 2);
      const int hb = hb0 + bi / WG_TBW, wb = wb0 + bi % WG_TBW;
      const bool in = (unsigned)ha < (unsigned)hA && (unsigned)wa < (unsigned)wA && hb < hB && wb < wB;
      (&xa[0][0][0])[i] = in ? xz[((long)(ha * wA + wa) * NB + hb * wB + wb) * CIN + c] : 0.f;
    }
    for (int i = t; i < WG_NA * WG_HB * CIN; i += 256) {  // b halo box at the tile's a positions
      const int c = i % CIN, p = i / CIN;
      const int bi = p % WG_HB, ai = p / WG_HB;
      const int ha = ha0 + ai / WG_TAW, wa = wa0 + ai % WG_TAW;
      const int hb = hb0 - 1 + bi / (WG_TBW + 2), wb = wb0 - 1 + bi % (WG_TBW + 2);
      const bool in = ha < hA && wa < wA && (unsigned)hb < (unsigned)hB && (unsigned)wb < (unsigned)wB;
      (&xb[0][0][0])[i] = in ? xz[((long)(ha * wA + wa) * NB + hb * wB + wb) * CIN + c] : 0.f;
    }
    for (int i = t; i < WG_NA * WG_NB * COUT; i += 256) {  // the output gradient at the tile's pairs
      const int oo = i % COUT, p = i / COUT;
      const int ai = p / WG_NB, bi = p % WG_NB;
      const int ha = ha0 + ai / WG_TAW, wa = wa0 + ai % WG_TAW;
      const int hb = hb0 + bi / WG_TBW, wb = wb0 + bi % WG_TBW;
      const bool in = ha < hA && wa < wA && hb < hB && wb < wB;
      (&gl[0][0])[i] = in ? gz[((long)(ha * wA + wa) * NB + hb * wB + wb) * COUT + oo] : 0.f;
    }
    __syncthreads();
    if (active) {
      for (int p = grp; p < WG_NA * WG_NB; p += NG) {
        const int ai = p / WG_NB, bi = p - ai * WG_NB;
        const float gv = gl[p][o];
        const float* xv = side == 0
                              ? xa[(ai / WG_TAW + ky) * (WG_TAW + 2) + ai % WG_TAW + kx][bi]
                              : xb[ai][(bi / WG_TBW + ky) * (WG_TBW + 2) + bi % WG_TBW + kx];
#pragma unroll
        for (int c = 0; c < CIN; ++c) acc[c] = fmaf(gv, xv[c], acc[c]);
        bacc += gv;
      }
    }
  }
  __syncthreads();
  if (active) {
#pragma unroll
    for (int c = 0; c < CIN; ++c) red[t][c] = acc[c];
    red[t][CIN] = bacc;
  }
  __syncthreads();
  if (t < NE) {
    float s[CIN + 1];
#pragma unroll
    for (int c = 0; c <= CIN; ++c) s[c] = red[t][c];
    for (int g = 1; g < NG; ++g)
#pragma unroll
      for (int c = 0; c <= CIN; ++c) s[c] += red[g * NE + t][c];
    float* pw = part + (long)blockIdx.x * (NE * CIN + COUT);
#pragma unroll
    for (int c = 0; c < CIN; ++c) pw[t * CIN + c] = s[c];
    if (t < COUT) pw[NE * CIN + t] = s[CIN];  // side 0, tap 0, o = t
  }
}

// sum the partials in workgroup order; dWa / dWb [COUT][CIN][9] accumulate, and db1 / db2 [COUT]
// unless bias == 0 (cp4d_bias_grad_f64 sums those)
__global__ void cp4d_wgrad_reduce_kernel(const float* __restrict__ part, int G, int CIN, int COUT, float* dWa,
                                         float* dWb, float* db1, float* db2, int bias) {
  const int NE = 18 * COUT, n = NE * CIN + COUT;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= n || (!bias && idx >= NE * CIN)) return;
  float s = 0.f;
  for (int g = 0; g < G; ++g) s += part[(long)g * n + idx];
  if (idx < NE * CIN) {
    const int e = idx / CIN, c = idx - e * CIN;
    const int side = e / (9 * COUT), tap = (e / COUT) % 9, o = e % COUT;
    float* W = side ? dWb : dWa;
    W[(o * CIN + c) * 9 + tap] += s;
  } else {
    const int o = idx - NE * CIN;
    db1[o] += s;
    db2[o] += s;
  }
}

// The bias gradients db1 = db2 += sum over every (a, b) pair of gm[p][o]: a sum of up to B (hA wA)
// (hB wB) terms whose ReLU-masked values cancel heavily (the last consensus layer's single bias is
// a few 1e-3 of sum |gm|), so it is accumulated in double, in a fixed order: chunks of
// CB64_ROWS rows per workgroup (a thread's rows strided by 256, then a fixed LDS tree), then the
// chunks in order.  Deterministic and accurate to the fp32 rounding of the result.
constexpr int CB64_ROWS = 16384, CB64_MAXC = 16;
__global__ __launch_bounds__(256) void colsum_f64_part_kernel(const float* __restrict__ X, long R, int Cc,
                                                              double* __restrict__ part) {
  __shared__ double red[256][CB64_MAXC + 1];
  const int t = threadIdx.x;
  const long r0 = (long)blockIdx.x * CB64_ROWS;
  const long r1 = min(R, r0 + CB64_ROWS);
  double acc[CB64_MAXC];
#pragma unroll
  for (int o = 0; o < CB64_MAXC; ++o) acc[o] = 0.0;
  for (long r = r0 + t; r < r1; r += 256)
#pragma unroll
    for (int o = 0; o < CB64_MAXC; ++o)
      if (o < Cc) acc[o] += (double)X[r * Cc + o];
#pragma unroll
  for (int o = 0; o < CB64_MAXC; ++o) red[t][o] = acc[o];
  __syncthreads();
  for (int w = 128; w >= 1; w >>= 1) {
    if (t < w)
      for (int o = 0; o < Cc; ++o) red[t][o] += red[t + w][o];
    __syncthreads();
  }
  if (t < Cc) part[(long)blockIdx.x * Cc + t] = red[0][t];
}

__global__ void colsum_f64_final_kernel(const double* __restrict__ part, int nch, int Cc, float* db1, float* db2) {
  const int o = threadIdx.x;
  if (o >= Cc) return;
  double s = 0.0;
  for (int c = 0; c < nch; ++c) s += part[(long)c * Cc + o];
  db1[o] = (float)((double)db1[o] + s);
  if (db2) db2[o] = (float)((double)db2[o] + s);
}

// workgroups of the weight-gradient pass: 512 for the 10 -> 10 layer (two per CU by LDS), 2048 for
// the thinner layers (less LDS each; measured 0.52 against 1.26 ms for 2 -> 10 at 60^2)
static int wgrad_grid(int cin, int cout) { return cin * cout >= 100 ? 512 : 2048; }
int cp4d_wgrad_part_floats(int cin, int cout) {
  (void)cin;
  (void)cout;
  return std::max(512 * (18 * 10 * 10 + 10), 2048 * (18 * 10 * 2 + 10));  // the largest of the four layers
}

int launch_cp4d_wgrad(const float* x, const float* gm, int B, int hA, int wA, int hB, int wB, int cin, int cout,
                      float* part, size_t part_floats, float* dWa, float* dWb, float* db1, float* db2,
                      hipStream_t st) {
  const long ntiles = (long)B * cdiv(hA, WG_TAH) * cdiv(wA, WG_TAW) * cdiv(hB, WG_TBH) * cdiv(wB, WG_TBW);
  const int G = (int)std::min<long>(wgrad_grid(cin, cout), ntiles);
  const int n = 18 * cout * cin + cout;
  if ((size_t)G * n > part_floats) return fail(CWT_ESTATE, "cp4d wgrad: partial workspace too small");
  static const bool scalar = getenv("CWT_WGRAD_SCALAR") && getenv("CWT_WGRAD_SCALAR")[0] == '1';  // A/B only
  if (!scalar) {
    int rc = launch_cp4d_wgrad_mfma(x, gm, B, hA, wA, hB, wB, cin, cout, G, part, st);
    if (rc) return rc;
  } else {
#define CWT_WG(CI, CO)                                                                                        \
  if (cin == CI && cout == CO) {                                                                              \
    hipLaunchKernelGGL((cp4d_wgrad_kernel<CI, CO>), dim3(G), dim3(256), 0, st, x, gm, B, hA, wA, hB, wB, part); \
    CWT_LAUNCH_CHECK();                                                                                       \
  } else
    CWT_WG(1, 10)
    CWT_WG(2, 10)
    CWT_WG(10, 10)
    CWT_WG(10, 1)
    return fail(CWT_EARG, "cp4d wgrad: channels (1|2 -> 10, 10 -> 10, 10 -> 1) only");
#undef CWT_WG
  }
  hipLaunchKernelGGL(cp4d_wgrad_reduce_kernel, dim3(cdiv(n, 256)), dim3(256), 0, st, (const float*)part, G, cin, cout,
                     dWa, dWb, db1, db2, 0);
  CWT_LAUNCH_CHECK();
  // the biases in double (the partials above are consumed: their workspace takes the chunks)
  const long R = (long)B * hA * wA * hB * wB;
  const int nch = (int)cdiv(R, (long)CB64_ROWS);
  if (cout > CB64_MAXC || (size_t)nch * cout * 2 > part_floats) return fail(CWT_ESTATE, "cp4d bias sum: workspace");
  hipLaunchKernelGGL(colsum_f64_part_kernel, dim3(nch), dim3(256), 0, st, gm, R, cout, (double*)part);
  CWT_LAUNCH_CHECK();
  hipLaunchKernelGGL(colsum_f64_final_kernel, dim3(1), dim3(64), 0, st, (const double*)part, nch, cout, db1, db2);
  CWT_LAUNCH_CHECK();
  return 0;
}

// ---- softmax(temp * corr2d) readout backward (match.py:151-153) ----
// g[a][n] (+)= temp * P[a][n] * (dA[a][n] - sum_m P[a][m] dA[a][m]); one workgroup per row
__global__ __launch_bounds__(256) void match_softmax_bwd_kernel(const float* __restrict__ P, int ldp,
                                                                const float* __restrict__ dA, int NB, float temp,
                                                                int accum, float* __restrict__ g) {
  const long row = blockIdx.x;
  const float* pr = P + row * ldp;
  const float* dr = dA + row * NB;
  float* gr = g + row * NB;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  __shared__ float red[4];
  float s = 0.f;
  for (int j = t; j < NB; j += 256) s = fmaf(pr[j], dr[j], s);
  s = wave_sum_dpp(s);
  if (lane == 0) red[wv] = s;
  __syncthreads();
  const float dot = (red[0] + red[1]) + (red[2] + red[3]);
  for (int j = t; j < NB; j += 256) {
    const float v = temp * pr[j] * (dr[j] - dot);
    gr[j] = accum ? gr[j] + v : v;
  }
}

int launch_match_softmax_bwd(const float* P, int ldp, const float* dA, int rows, int NB, float temp, int accum,
                             float* g, hipStream_t st) {
  hipLaunchKernelGGL(match_softmax_bwd_kernel, dim3(rows), dim3(256), 0, st, P, ldp, dA, NB, temp, accum, g);
  CWT_LAUNCH_CHECK();
  return 0;
}

// ---- F.normalize (model_util.py:106-107) forward with the norms kept, and its backward ----
// xn = x / max(|x|, eps); dx = (dxn - xn (xn . dxn)) / |x| where |x| > eps, dxn / eps elsewhere
__global__ __launch_bounds__(256) void token_norm_kernel(const float* __restrict__ x, long T, int C, float eps,
                                                         float* __restrict__ xn, float* __restrict__ nrm) {
  const int lane = threadIdx.x & 63;
  for (long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6); r < T; r += (long)gridDim.x * 4) {
    const float* xr = x + r * C;
    float ss = 0.f;
    for (int c = lane; c < C; c += 64) ss = fmaf(xr[c], xr[c], ss);
    const float n = sqrtf(wave_sum_dpp(ss));
    const float inv = 1.f / fmaxf(n, eps);
    for (int c = lane; c < C; c += 64) xn[r * C + c] = xr[c] * inv;
    if (lane == 0) nrm[r] = n;
  }
}

__global__ __launch_bounds__(256) void token_norm_bwd_kernel(const float* __restrict__ xn, const float* __restrict__ nrm,
                                                             const float* __restrict__ dxn, long T, int C, int ld_d,
                                                             float eps, int accum, float* __restrict__ dx) {
  const int lane = threadIdx.x & 63;
  for (long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6); r < T; r += (long)gridDim.x * 4) {
    const float* xr = xn + r * C;
    const float* dr = dxn + r * ld_d;
    const float n = nrm[r];
    float s = 0.f;
    for (int c = lane; c < C; c += 64) s = fmaf(xr[c], dr[c], s);
    s = wave_sum_dpp(s);
    for (int c = lane; c < C; c += 64) {
      const float v = n > eps ? (dr[c] - xr[c] * s) / n : dr[c] / eps;
      dx[r * C + c] = accum ? dx[r * C + c] + v : v;
    }
  }
}

int launch_token_norm(const float* x, long T, int C, float eps, float* xn, float* nrm, hipStream_t st) {
  hipLaunchKernelGGL(token_norm_kernel, dim3((unsigned)std::min<long>(4096, (T + 3) / 4)), dim3(256), 0, st, x, T, C, eps,
                     xn, nrm);
  CWT_LAUNCH_CHECK();
  return 0;
}

int launch_token_norm_bwd(const float* xn, const float* nrm, const float* dxn, long T, int C, int ld_d, float eps,
                          int accum, float* dx, hipStream_t st) {
  hipLaunchKernelGGL(token_norm_bwd_kernel, dim3((unsigned)std::min<long>(4096, (T + 3) / 4)), dim3(256), 0, st, xn, nrm,
                     dxn, T, C, ld_d, eps, accum, dx);
  CWT_LAUNCH_CHECK();
  return 0;
}

// ---- WeightAverage (msm_func.py:66-104) backward, R = 3 ----
// Per pixel p with theta = tpg_t + b_t, phi_r / g_r the neighbour r's (replicate padding),
// cos_r = theta . phi_r / (n_t n_r) (n = max(|.|, 1e-8)), s = softmax(cos), wavg = sum_r s_r g_r:
//   ds_r = dwavg . g_r, dcos_r = s_r (ds_r - sum s ds),
//   dtheta = sum_r dcos_r phi_r / (n_t n_r) - theta (sum_r dcos_r cos_r) / |theta|^2,
//   dphi_r += dcos_r theta / (n_t n_r) - phi_r dcos_r cos_r / |phi_r|^2,  dg_r += s_r dwavg
// (the |.|^2 terms only where the norm exceeds the clamp).  wa_bwd_pix_kernel forms dtheta and
// the per-(p, r) coefficients; wa_bwd_nbr_kernel gathers each pixel's dphi / dg from the pixels
// whose neighbourhood holds it (at most the 3 x 3 around it), in a fixed order.
template <int CPT>
__global__ __launch_bounds__(256) void wa_bwd_pix_kernel(const float* __restrict__ tpg, int h, int w, int co,
                                                         const float* __restrict__ bt, const float* __restrict__ bp,
                                                         const float* __restrict__ bg,
                                                         const float* __restrict__ dwavg, float* __restrict__ coef,
                                                         float* __restrict__ dtpg) {
  const long P = (long)h * w;
  const long pix = blockIdx.x;
  const long n = pix / P;
  const int p = (int)(pix - n * P), y = p / w, x = p - y * w;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const long ld = 3L * co;
  __shared__ float red[4][28];
  __shared__ float cf[10];  // cA[9], cTh
  float th[CPT], dw[CPT];
  const float* tp = tpg + pix * ld;
#pragma unroll
  for (int k = 0; k < CPT; ++k) {
    th[k] = tp[t + 256 * k] + bt[t + 256 * k];
    dw[k] = dwavg[pix * co + t + 256 * k];
  }
  float part[28];
  part[18] = 0.f;
#pragma unroll
  for (int k = 0; k < CPT; ++k) part[18] = fmaf(th[k], th[k], part[18]);
#pragma unroll
  for (int r = 0; r < 9; ++r) {
    const int yy = min(max(y + r / 3 - 1, 0), h - 1), xx = min(max(x + r % 3 - 1, 0), w - 1);
    const float* q = tpg + (n * P + (long)yy * w + xx) * ld;
    float d = 0.f, nn = 0.f, dg = 0.f;
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const float ph = q[co + t + 256 * k] + bp[t + 256 * k];
      const float gv = q[2 * co + t + 256 * k] + bg[t + 256 * k];
      d = fmaf(ph, th[k], d);
      nn = fmaf(ph, ph, nn);
      dg = fmaf(dw[k], gv, dg);
    }
    part[r] = d;
    part[9 + r] = nn;
    part[19 + r] = dg;
  }
#pragma unroll
  for (int i = 0; i < 28; ++i) {
    const float v = wave_sum_dpp(part[i]);
    if (lane == 0) red[wv][i] = v;
  }
  __syncthreads();
  if (t == 0) {
    float tot[28];
#pragma unroll
    for (int i = 0; i < 28; ++i) tot[i] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
    const float tn_raw = sqrtf(tot[18]), tn = fmaxf(tn_raw, 1e-8f);
    float cs[9], sm[9], nr[9], m = -INFINITY;
#pragma unroll
    for (int r = 0; r < 9; ++r) {
      nr[r] = fmaxf(sqrtf(tot[9 + r]), 1e-8f);
      cs[r] = tot[r] / (nr[r] * tn);
      m = fmaxf(m, cs[r]);
    }
    float se = 0.f;
#pragma unroll
    for (int r = 0; r < 9; ++r) {
      sm[r] = expf(cs[r] - m);
      se += sm[r];
    }
    float sds = 0.f;
#pragma unroll
    for (int r = 0; r < 9; ++r) {
      sm[r] = sm[r] / se;
      sds = fmaf(sm[r], tot[19 + r], sds);
    }
    float cth = 0.f;
#pragma unroll
    for (int r = 0; r < 9; ++r) {
      const float dcos = sm[r] * (tot[19 + r] - sds);
      const float ca = dcos / (nr[r] * tn);
      const float cphi = sqrtf(tot[9 + r]) > 1e-8f ? dcos * cs[r] / tot[9 + r] : 0.f;
      cth = fmaf(dcos, cs[r], cth);
      cf[r] = ca;
      coef[pix * 27 + r] = ca;
      coef[pix * 27 + 9 + r] = cphi;
      coef[pix * 27 + 18 + r] = sm[r];
    }
    cf[9] = tn_raw > 1e-8f ? cth / tot[18] : 0.f;
  }
  __syncthreads();
  float dth[CPT];
#pragma unroll
  for (int k = 0; k < CPT; ++k) dth[k] = -cf[9] * th[k];
#pragma unroll
  for (int r = 0; r < 9; ++r) {
    const int yy = min(max(y + r / 3 - 1, 0), h - 1), xx = min(max(x + r % 3 - 1, 0), w - 1);
    const float* q = tpg + (n * P + (long)yy * w + xx) * ld + co;
    const float a = cf[r];
#pragma unroll
    for (int k = 0; k < CPT; ++k) dth[k] = fmaf(a, q[t + 256 * k] + bp[t + 256 * k], dth[k]);
  }
#pragma unroll
  for (int k = 0; k < CPT; ++k) dtpg[pix * ld + t + 256 * k] = dth[k];
}

template <int CPT>
__global__ __launch_bounds__(256) void wa_bwd_nbr_kernel(const float* __restrict__ tpg, int h, int w, int co,
                                                         const float* __restrict__ bt, const float* __restrict__ bp,
                                                         const float* __restrict__ dwavg,
                                                         const float* __restrict__ coef, float* __restrict__ dtpg) {
  const long P = (long)h * w;
  const long pix = blockIdx.x;
  const long n = pix / P;
  const int q = (int)(pix - n * P), yq = q / w, xq = q - yq * w;
  const int t = threadIdx.x;
  const long ld = 3L * co;
  float ph[CPT], dph[CPT], dg[CPT];
#pragma unroll
  for (int k = 0; k < CPT; ++k) {
    ph[k] = tpg[pix * ld + co + t + 256 * k] + bp[t + 256 * k];
    dph[k] = 0.f;
    dg[k] = 0.f;
  }
  for (int dy = -1; dy <= 1; ++dy) {
    const int yp = yq + dy;
    if (yp < 0 || yp >= h) continue;
    for (int dx = -1; dx <= 1; ++dx) {
      const int xp = xq + dx;
      if (xp < 0 || xp >= w) continue;
      const long pp = n * P + (long)yp * w + xp;
      for (int r = 0; r < 9; ++r) {
        const int yy = min(max(yp + r / 3 - 1, 0), h - 1), xx = min(max(xp + r % 3 - 1, 0), w - 1);
        if (yy != yq || xx != xq) continue;
        const float ca = coef[pp * 27 + r], cphi = coef[pp * 27 + 9 + r], s = coef[pp * 27 + 18 + r];
#pragma unroll
        for (int k = 0; k < CPT; ++k) {
          const float thp = tpg[pp * ld + t + 256 * k] + bt[t + 256 * k];
          dph[k] = fmaf(ca, thp, fmaf(-cphi, ph[k], dph[k]));
          dg[k] = fmaf(s, dwavg[pp * co + t + 256 * k], dg[k]);
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < CPT; ++k) {
    dtpg[pix * ld + co + t + 256 * k] = dph[k];
    dtpg[pix * ld + 2 * co + t + 256 * k] = dg[k];
  }
}

int launch_wa_bwd(const float* tpg, int N, int h, int w, int co, const float* bt, const float* bp, const float* bg,
                  const float* dwavg, float* coef, float* dtpg, hipStream_t st) {
  const dim3 grid((unsigned)((long)N * h * w));
#define CWT_WAB(CPT)                                                                                              \
  hipLaunchKernelGGL((wa_bwd_pix_kernel<CPT>), grid, dim3(256), 0, st, tpg, h, w, co, bt, bp, bg, dwavg, coef, dtpg); \
  CWT_LAUNCH_CHECK();                                                                                             \
  hipLaunchKernelGGL((wa_bwd_nbr_kernel<CPT>), grid, dim3(256), 0, st, tpg, h, w, co, bt, bp, dwavg,                \
                     (const float*)coef, dtpg);                                                                   \
  CWT_LAUNCH_CHECK();
  if (co == 256) {
    CWT_WAB(1)
  } else if (co == 512) {
    CWT_WAB(2)
  } else if (co == 1024) {
    CWT_WAB(4)
  } else {
    return fail(CWT_EARG, "WeightAverage backward: c_in / 2 must be 256, 512 or 1024");
  }
#undef CWT_WAB
  return 0;
}

// ---- small helpers ----
// out[c] (+)= sum_r X[r][c] (row stride ld): the bias gradients.  Two fixed-order stages: chunks
// of CS_ROWS rows summed per (64-column block, chunk) workgroup, 4 row lanes of 64 columns each
// combined in lane order; then the chunk partials summed in chunk order.
constexpr int CS_ROWS = 64;
__global__ __launch_bounds__(256) void colsum_part_kernel(const float* __restrict__ X, long R, int Cc, long ld,
                                                          float* __restrict__ part) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), rl = threadIdx.x >> 6;
  const long r0 = (long)blockIdx.y * CS_ROWS;
  __shared__ float red[4][64];
  float s = 0.f;
  if (c < Cc)
    for (int i = rl; i < CS_ROWS && r0 + i < R; i += 4) s += X[(r0 + i) * ld + c];
  red[rl][threadIdx.x & 63] = s;
  __syncthreads();
  if (rl == 0 && c < Cc) {
    const int l = threadIdx.x & 63;
    part[(long)blockIdx.y * Cc + c] = (red[0][l] + red[1][l]) + (red[2][l] + red[3][l]);
  }
}

__global__ void colsum_final_kernel(const float* __restrict__ part, int nch, int Cc, int accum, float* __restrict__ out) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= Cc) return;
  float s = 0.f;
  for (int k = 0; k < nch; ++k) s += part[(long)k * Cc + c];
  out[c] = accum ? out[c] + s : s;
}

size_t colsum_ws_floats(long R, int Cc) { return (size_t)cdiv(R, CS_ROWS) * Cc; }

int launch_colsum(const float* X, long R, int Cc, long ld, int accum, float* out, float* ws, size_t ws_floats,
                  hipStream_t st) {
  const int nch = cdiv(R, CS_ROWS);
  if (!ws || ws_floats < colsum_ws_floats(R, Cc)) return fail(CWT_ESTATE, "colsum: workspace too small");
  hipLaunchKernelGGL(colsum_part_kernel, dim3(cdiv(Cc, 64), nch), dim3(256), 0, st, X, R, Cc, ld, ws);
  CWT_LAUNCH_CHECK();
  hipLaunchKernelGGL(colsum_final_kernel, dim3(cdiv(Cc, 256)), dim3(256), 0, st, (const float*)ws, nch, Cc, accum, out);
  CWT_LAUNCH_CHECK();
  return 0;
}

// y[b][c][p] = x[b][p][c] (channels-last -> channel-first)
__global__ void to_channels_first_kernel(const float* __restrict__ x, int B, int C, long P, float* __restrict__ y) {
  const long total = (long)B * C * P;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long p = i % P;
    const int c = (int)((i / P) % C);
    const long b = i / ((long)C * P);
    y[i] = x[(b * P + p) * C + c];
  }
}

int launch_to_channels_first(const float* x, int B, int C, long P, float* y, hipStream_t st) {
  const long n = (long)B * C * P;
  hipLaunchKernelGGL(to_channels_first_kernel, dim3((unsigned)std::min<long>(65536, cdiv(n, 256))), dim3(256), 0, st, x,
                     B, C, P, y);
  CWT_LAUNCH_CHECK();
  return 0;
}

// out [R][ld] = X [R][Cc] with the pad columns zero
__global__ void copy_pad_kernel(const float* __restrict__ X, long R, int Cc, int ld, float* __restrict__ out) {
  const long total = R * ld;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long r = i / ld;
    const int c = (int)(i - r * ld);
    out[i] = c < Cc ? X[r * Cc + c] : 0.f;
  }
}

int launch_copy_pad(const float* X, long R, int Cc, int ld, float* out, hipStream_t st) {
  const long n = R * ld;
  hipLaunchKernelGGL(copy_pad_kernel, dim3((unsigned)std::min<long>(65536, cdiv(n, 256))), dim3(256), 0, st, X, R, Cc,
                     ld, out);
  CWT_LAUNCH_CHECK();
  return 0;
}

// MMN blend (mmn.py:65-67) backward: d_att[b][i] = (d_mean[i] + att_wt d_fq[i]) / B,
// d_fq_in[i] = (1 - att_wt) d_fq[i]
__global__ void mmn_blend_bwd_kernel(const float* __restrict__ d_fq, const float* __restrict__ d_mean, int B, long n,
                                     float att_wt, float* __restrict__ d_att, float* __restrict__ d_fq_in) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float g = d_fq ? d_fq[i] : 0.f;
    const float dm = ((d_mean ? d_mean[i] : 0.f) + att_wt * g) / (float)B;
    for (int b = 0; b < B; ++b) d_att[(long)b * n + i] = dm;
    if (d_fq_in) d_fq_in[i] = (1.f - att_wt) * g;
  }
}

int launch_mmn_blend_bwd(const float* d_fq, const float* d_mean, int B, long n, float att_wt, float* d_att,
                         float* d_fq_in, hipStream_t st) {
  hipLaunchKernelGGL(mmn_blend_bwd_kernel, dim3((unsigned)std::min<long>(65536, cdiv(n, 256))), dim3(256), 0, st, d_fq,
                     d_mean, B, n, att_wt, d_att, d_fq_in);
  CWT_LAUNCH_CHECK();
  return 0;
}

}  // namespace cwt

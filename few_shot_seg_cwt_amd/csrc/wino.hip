// Winograd F(2x2, 3x3) and F(4x4, 3x3) for the stride-1 3x3 convs of the fp32-width conv stack
// (x6 path): the layer2-4 conv2s and the bottleneck conv (resnet.py:57-96 Bottleneck.conv2 after
// pspnet.py:103-112's dilation surgery, pspnet.py:124-129 bottleneck).
//
// A 3x3 conv with dilation d (= its padding) splits into d*d independent dense 3x3 convs, one per
// output sub-grid (oy mod d, ox mod d): output (py + d i, px + d j) reads only inputs of the same
// sub-grid.  On each sub-grid, m x m output tiles (Lavin & Gray; correlation form, as conv2d):
//   Y = A^T [ (G g G^T) (.) (B^T D B) ] A,   D the (m+2)x(m+2) input tile at sub-grid rows
//   m ti - 1 .. m ti + m.
// F(2x2,3x3) (m = 2, points 0, +-1):
//   B^T = [1 0 -1 0; 0 1 1 0; 0 -1 1 0; 0 1 0 -1],  G = [1 0 0; .5 .5 .5; .5 -.5 .5; 0 0 1],
//   A^T = [1 1 1 0; 0 1 -1 -1].
// F(4x4,3x3) (m = 4, points 0, +-1, +-2):
//   B^T = [4 0 -5 0 1 0; 0 -4 -4 1 1 0; 0 4 -4 -1 1 0; 0 -2 -1 2 1 0; 0 2 -1 -2 1 0; 0 4 0 -5 0 1],
//   G = [1/4 0 0; -1/6 -1/6 -1/6; -1/6 1/6 -1/6; 1/24 1/12 1/6; 1/24 -1/12 1/6; 0 0 1],
//   A^T = [1 1 1 1 1 0; 0 1 -1 2 -2 0; 0 1 1 4 4 0; 0 1 -1 8 -8 1].
// The products become P = (m+2)^2 GEMMs (one per transformed position xi) over every tile t and
// input channel: M[xi][t][co] = sum_ci V[xi][t][ci] U[xi][co][ci] -- P x (T x Ci x Co)
// multiply-adds where the direct conv has 9 x (m^2 T x Ci x Co): 2.25x (m = 2) or 4x (m = 4) fewer
// matrix-core products, and V / M hold 4x (m = 2) or 2.25x (m = 4) the pixels of the input /
// output.  They run as ONE batched launch of the x6 GEMM body (conv_x6.hip, PREC 6: V split three
// ways in registers, U pre-split at load), at the same fp32-width product arithmetic as the direct
// conv.  The transforms are fp32 arithmetic with small integer coefficients (B, A) and one
// rounding of G g G^T (weights, computed in double at load).  Their rounding error is of the size
// of an fp32 GEMM's own accumulation error (F(4x4): about 10x F(2x2)'s); the per-conv tests bound
// both forms against a float64 conv (tests/test_gpu_conv_s.py, bar 1e-5 of max |y|).
//
// Layouts: x / y fp32 NHWC (pixel stride Ci / y_ld); V [P][T][Ci] and Mb [P][T][Co] fp32, tile
// t = (((n d + py) d + px) TY + ti) TX + tj, TY = ceil(ceil(H/d)/m) (tiles reaching past a
// sub-grid's edge read zeros and store nothing there).
#include "common.h"
#include "kernels.h"

namespace cwt {

WinoGeom wino_geom(int N, int H, int W, int d, int m) {
  WinoGeom g;
  g.N = N;
  g.H = H;
  g.W = W;
  g.d = d;
  g.m = m;
  g.P = (m + 2) * (m + 2);
  g.TY = ((H + d - 1) / d + m - 1) / m;
  g.TX = ((W + d - 1) / d + m - 1) / m;
  g.T = (long)N * d * d * g.TY * g.TX;
  return g;
}

// U[xi][co][ci] = (G g G^T)[xi] from the packed fp32 weights [Co][K] (K = packed_k(ci, tap, 9)),
// in double, rounded once to fp32
__global__ void wino_weights_kernel(const float* __restrict__ w, int Co, int Ci, float* __restrict__ U) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)Co * Ci) return;
  const int co = (int)(idx / Ci), ci = (int)(idx - (long)co * Ci);
  const long K = 9L * Ci;
  double g[3][3];
#pragma unroll
  for (int t = 0; t < 9; ++t) g[t / 3][t % 3] = (double)w[(long)co * K + packed_k(ci, t, 9)];
  double gg[4][3];  // G g
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    gg[0][c] = g[0][c];
    gg[1][c] = 0.5 * (g[0][c] + g[1][c] + g[2][c]);
    gg[2][c] = 0.5 * (g[0][c] - g[1][c] + g[2][c]);
    gg[3][c] = g[2][c];
  }
  const long plane = (long)Co * Ci;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const double u[4] = {gg[r][0], 0.5 * (gg[r][0] + gg[r][1] + gg[r][2]), 0.5 * (gg[r][0] - gg[r][1] + gg[r][2]),
                         gg[r][2]};
#pragma unroll
    for (int c = 0; c < 4; ++c) U[(r * 4 + c) * plane + idx] = (float)u[c];
  }
}

// F(4x4,3x3): U[xi][co][ci], xi in 0..35, from G = [1/4 0 0; -1/6 -1/6 -1/6; -1/6 1/6 -1/6;
// 1/24 1/12 1/6; 1/24 -1/12 1/6; 0 0 1], in double, rounded once to fp32
__device__ __forceinline__ void wino4_g(const double g0, const double g1, const double g2, double u[6]) {
  u[0] = g0 / 4.0;
  u[1] = -(g0 + g1 + g2) / 6.0;
  u[2] = -(g0 - g1 + g2) / 6.0;
  u[3] = g0 / 24.0 + g1 / 12.0 + g2 / 6.0;
  u[4] = g0 / 24.0 - g1 / 12.0 + g2 / 6.0;
  u[5] = g2;
}

__global__ void wino4_weights_kernel(const float* __restrict__ w, int Co, int Ci, float* __restrict__ U) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)Co * Ci) return;
  const int co = (int)(idx / Ci), ci = (int)(idx - (long)co * Ci);
  const long K = 9L * Ci;
  double g[3][3];
#pragma unroll
  for (int t = 0; t < 9; ++t) g[t / 3][t % 3] = (double)w[(long)co * K + packed_k(ci, t, 9)];
  double gg[6][3];  // G g (columns)
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    double u[6];
    wino4_g(g[0][c], g[1][c], g[2][c], u);
#pragma unroll
    for (int r = 0; r < 6; ++r) gg[r][c] = u[r];
  }
  const long plane = (long)Co * Ci;
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    double u[6];
    wino4_g(gg[r][0], gg[r][1], gg[r][2], u);
#pragma unroll
    for (int c = 0; c < 6; ++c) U[(r * 6 + c) * plane + idx] = (float)u[c];
  }
}

int launch_wino_weights(const float* w_packed, int Co, int Ci, float* U, hipStream_t st, int m) {
  const long n = (long)Co * Ci;
  if (m == 4)
    hipLaunchKernelGGL(wino4_weights_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, st, w_packed, Co, Ci, U);
  else if (m == 2)
    hipLaunchKernelGGL(wino_weights_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, st, w_packed, Co, Ci, U);
  else
    return fail(CWT_EARG, "winograd: output tile must be 2 or 4");
  CWT_LAUNCH_CHECK();
  return 0;
}

// The input transforms' thread index with the blocks remapped XCD-contiguous: the dispatcher
// deals blocks round-robin over the 8 XCDs (block b on XCD b % 8, MI355X_MICROARCH.md), so
// logically consecutive blocks -- neighbouring tiles, whose input patches overlap by half -- would
// each fetch the shared rows into a different XCD's L2; remapped, one XCD takes one contiguous run
// of tiles and the overlap hits its L2
__device__ __forceinline__ long wino_xcd_index() {
  const unsigned nb = gridDim.x, b = blockIdx.x;
  const unsigned q = nb >> 3, r = nb & 7, xcd = b & 7, slot = b >> 3;
  const unsigned L = xcd < r ? xcd * (q + 1) + slot : r * (q + 1) + (xcd - r) * q + slot;
  return (long)L * blockDim.x + threadIdx.x;
}

__device__ __forceinline__ void wino_tile(long t, const WinoGeom& g, int& n, int& py, int& px, int& ti, int& tj) {
  tj = (int)(t % g.TX);
  long r = t / g.TX;
  ti = (int)(r % g.TY);
  r /= g.TY;
  px = (int)(r % g.d);
  r /= g.d;
  py = (int)(r % g.d);
  n = (int)(r / g.d);
}

// V = B^T D B per tile and 4 channels; one thread per (tile, channel quad), consecutive threads
// take consecutive channel quads (coalesced 16-B loads and stores)
__global__ __launch_bounds__(256) void wino_in_kernel(const float* __restrict__ x, WinoGeom g, int Ci,
                                                      float* __restrict__ V) {
  const int q4 = Ci >> 2;
  const long idx = wino_xcd_index();
  if (idx >= g.T * q4) return;
  const long t = idx / q4;
  const int c = (int)(idx - t * q4) * 4;
  int n, py, px, ti, tj;
  wino_tile(t, g, n, py, px, ti, tj);
  f32x4 D[4][4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int iy = py + g.d * (2 * ti - 1 + u);
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int ix = px + g.d * (2 * tj - 1 + v);
      const bool in = (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
      D[u][v] = in ? *(const f32x4*)(x + (((long)n * g.H + iy) * g.W + ix) * Ci + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  f32x4 R[4][4];  // B^T D (rows)
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    R[0][v] = D[0][v] - D[2][v];
    R[1][v] = D[1][v] + D[2][v];
    R[2][v] = D[2][v] - D[1][v];
    R[3][v] = D[1][v] - D[3][v];
  }
  const long plane = g.T * Ci;
  float* vp = V + t * Ci + c;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const f32x4 o[4] = {R[u][0] - R[u][2], R[u][1] + R[u][2], R[u][2] - R[u][1], R[u][1] - R[u][3]};
#pragma unroll
    for (int v = 0; v < 4; ++v) *(f32x4*)(vp + (u * 4 + v) * plane) = o[v];
  }
}

// F(4x4,3x3) input transform of one 6-vector: B^T d, B^T = [4 0 -5 0 1 0; 0 -4 -4 1 1 0;
// 0 4 -4 -1 1 0; 0 -2 -1 2 1 0; 0 2 -1 -2 1 0; 0 4 0 -5 0 1]
__device__ __forceinline__ void wino4_bt(const f32x4 d[6], f32x4 r[6]) {
  r[0] = 4.f * d[0] - 5.f * d[2] + d[4];
  r[1] = (d[3] + d[4]) - 4.f * (d[1] + d[2]);
  r[2] = (d[4] - d[3]) + 4.f * (d[1] - d[2]);
  r[3] = (d[4] - d[2]) + 2.f * (d[3] - d[1]);
  r[4] = (d[4] - d[2]) + 2.f * (d[1] - d[3]);
  r[5] = 4.f * d[1] - 5.f * d[3] + d[5];
}

// V = B^T D B for F(4x4,3x3): one thread per (tile, channel quad) as wino_in_kernel; the 6x6
// input tile column by column (B^T D), then each row of it (. B)
__global__ __launch_bounds__(256) void wino4_in_kernel(const float* __restrict__ x, WinoGeom g, int Ci,
                                                       float* __restrict__ V) {
  const int q4 = Ci >> 2;
  const long idx = wino_xcd_index();
  if (idx >= g.T * q4) return;
  const long t = idx / q4;
  const int c = (int)(idx - t * q4) * 4;
  int n, py, px, ti, tj;
  wino_tile(t, g, n, py, px, ti, tj);
  f32x4 R[6][6];  // B^T D: R[u][v]
#pragma unroll
  for (int v = 0; v < 6; ++v) {
    const int ix = px + g.d * (4 * tj - 1 + v);
    f32x4 D[6];
#pragma unroll
    for (int u = 0; u < 6; ++u) {
      const int iy = py + g.d * (4 * ti - 1 + u);
      const bool in = (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
      D[u] = in ? *(const f32x4*)(x + (((long)n * g.H + iy) * g.W + ix) * Ci + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    f32x4 r[6];
    wino4_bt(D, r);
#pragma unroll
    for (int u = 0; u < 6; ++u) R[u][v] = r[u];
  }
  const long plane = g.T * Ci;
  float* vp = V + t * Ci + c;
#pragma unroll
  for (int u = 0; u < 6; ++u) {
    f32x4 o[6];
    wino4_bt(R[u], o);
#pragma unroll
    for (int v = 0; v < 6; ++v) *(f32x4*)(vp + (u * 6 + v) * plane) = o[v];
  }
}

int launch_wino_in(const float* x, const WinoGeom& g, int Ci, float* V, hipStream_t st) {
  if (Ci % 4) return fail(CWT_EARG, "wino_in: Ci % 4");
  const long n = g.T * (Ci / 4);
  if (g.m == 4)
    hipLaunchKernelGGL(wino4_in_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, st, x, g, Ci, V);
  else if (g.m == 2)
    hipLaunchKernelGGL(wino_in_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, st, x, g, Ci, V);
  else
    return fail(CWT_EARG, "winograd: output tile must be 2 or 4");
  CWT_LAUNCH_CHECK();
  return 0;
}

// Y = A^T M A per tile and 4 output channels, then the conv's epilogue in the direct kernels'
// order: fmaf(y, scale, shift), + residual, ReLU; pixels past a sub-grid's edge are not stored
__global__ __launch_bounds__(256) void wino_out_kernel(const float* __restrict__ Mb, WinoGeom g, int Co,
                                                       const float* __restrict__ scale, const float* __restrict__ shift,
                                                       const float* __restrict__ res, int res_ld, int relu,
                                                       float* __restrict__ y, int y_ld, int y_off) {
  const int q4 = Co >> 2;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= g.T * q4) return;
  const long t = idx / q4;
  const int c = (int)(idx - t * q4) * 4;
  int n, py, px, ti, tj;
  wino_tile(t, g, n, py, px, ti, tj);
  const long plane = g.T * Co;
  const float* mp = Mb + t * Co + c;
  f32x4 m[4][4];
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int v = 0; v < 4; ++v) m[u][v] = *(const f32x4*)(mp + (u * 4 + v) * plane);
  f32x4 s[2][4];  // A^T M (rows)
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    s[0][v] = m[0][v] + m[1][v] + m[2][v];
    s[1][v] = m[1][v] - m[2][v] - m[3][v];
  }
  const f32x4 sc = *(const f32x4*)(scale + c), sh = *(const f32x4*)(shift + c);
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const f32x4 o[2] = {s[a][0] + s[a][1] + s[a][2], s[a][1] - s[a][2] - s[a][3]};
    const int oy = py + g.d * (2 * ti + a);
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int ox = px + g.d * (2 * tj + b);
      if (oy >= g.H || ox >= g.W) continue;
      const long pix = ((long)n * g.H + oy) * g.W + ox;
      f32x4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = fmaf(o[b][i], sc[i], sh[i]);
      if (res) v += *(const f32x4*)(res + pix * res_ld + c);
      if (relu) {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = fmaxf(v[i], 0.f);
      }
      *(f32x4*)(y + pix * y_ld + y_off + c) = v;
    }
  }
}

// F(4x4,3x3) output transform of one 6-vector: A^T m, A^T = [1 1 1 1 1 0; 0 1 -1 2 -2 0;
// 0 1 1 4 4 0; 0 1 -1 8 -8 1]
__device__ __forceinline__ void wino4_at(const f32x4 m[6], f32x4 o[4]) {
  const f32x4 p12 = m[1] + m[2], m12 = m[1] - m[2], p34 = m[3] + m[4], m34 = m[3] - m[4];
  o[0] = m[0] + p12 + p34;
  o[1] = m12 + 2.f * m34;
  o[2] = p12 + 4.f * p34;
  o[3] = m12 + 8.f * m34 + m[5];
}

// Y = A^T M A for F(4x4,3x3), then the conv's epilogue as wino_out_kernel: the 6x6 block of M
// column by column (A^T M), then each of its 4 rows (. A)
__global__ __launch_bounds__(256) void wino4_out_kernel(const float* __restrict__ Mb, WinoGeom g, int Co,
                                                        const float* __restrict__ scale, const float* __restrict__ shift,
                                                        const float* __restrict__ res, int res_ld, int relu,
                                                        float* __restrict__ y, int y_ld, int y_off) {
  const int q4 = Co >> 2;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= g.T * q4) return;
  const long t = idx / q4;
  const int c = (int)(idx - t * q4) * 4;
  int n, py, px, ti, tj;
  wino_tile(t, g, n, py, px, ti, tj);
  const long plane = g.T * Co;
  const float* mp = Mb + t * Co + c;
  f32x4 s[4][6];  // A^T M: s[a][v]
#pragma unroll
  for (int v = 0; v < 6; ++v) {
    f32x4 m[6], o[4];
#pragma unroll
    for (int u = 0; u < 6; ++u) m[u] = *(const f32x4*)(mp + (u * 6 + v) * plane);
    wino4_at(m, o);
#pragma unroll
    for (int a = 0; a < 4; ++a) s[a][v] = o[a];
  }
  const f32x4 sc = *(const f32x4*)(scale + c), sh = *(const f32x4*)(shift + c);
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    f32x4 o[4];
    wino4_at(s[a], o);
    const int oy = py + g.d * (4 * ti + a);
    if (oy >= g.H) break;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int ox = px + g.d * (4 * tj + b);
      if (ox >= g.W) break;
      const long pix = ((long)n * g.H + oy) * g.W + ox;
      f32x4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = fmaf(o[b][i], sc[i], sh[i]);
      if (res) v += *(const f32x4*)(res + pix * res_ld + c);
      if (relu) {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = fmaxf(v[i], 0.f);
      }
      *(f32x4*)(y + pix * y_ld + y_off + c) = v;
    }
  }
}

int launch_wino_out(const float* Mb, const WinoGeom& g, int Co, const float* scale, const float* shift, const float* res,
                    int res_ld, int relu, float* y, int y_ld, int y_off, hipStream_t st) {
  if (Co % 4 || y_ld % 4 || y_off % 4 || (res && res_ld % 4)) return fail(CWT_EARG, "wino_out: 16-B channel groups");
  const long n = g.T * (Co / 4);
  if (g.m == 4)
    hipLaunchKernelGGL(wino4_out_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, st, Mb, g, Co, scale, shift, res,
                       res_ld, relu, y, y_ld, y_off);
  else if (g.m == 2)
    hipLaunchKernelGGL(wino_out_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, st, Mb, g, Co, scale, shift, res,
                       res_ld, relu, y, y_ld, y_off);
  else
    return fail(CWT_EARG, "winograd: output tile must be 2 or 4");
  CWT_LAUNCH_CHECK();
  return 0;
}

}  // namespace cwt

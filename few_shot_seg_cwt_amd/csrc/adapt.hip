// Support-set inner loop (reference test.py:164-187, train.py:206-231).
//
// Per SGD step the reference launches ~10 kernels (1x1 conv, bilinear upsample to S x S,
// log-softmax, weighted NLL, and the three backwards) and materialises four S x S x 2
// fp32 tensors.  Here one kernel does the whole step:
//   z      = W . f_s                       at low resolution, per tile (+1-pixel halo)
//   z_hi   = bilinear(align_corners) (z)   per high-res pixel, never stored
//   g_hi   = w_y (softmax(z_hi) - onehot)  weighted CE gradient (the 1/sum(w) is folded
//                                          into the learning rate)
//   g_lo   = U^T g_hi                      adjoint of the upsample, accumulated in LDS
//   dW    += g_lo . f_s^T                  f_s tile already in registers from the z pass
// Workgroup = (lo-res row pair r, 16-column block, shot).  With two classes the gradient
// of class 0 is exactly minus that of class 1 (softmax sums to one, so does the one-hot),
// so only dW[1] is reduced: one 2 KB fp32 atomic add per workgroup into acc[s % 3].
// The next step's kernel applies W <- W - lr/sum(w) * dW on the fly, so a step is one
// launch; three accumulator slots let step s zero slot s+1 without a race.
// f_s (7.4 MB per shot at 60x60x512) is re-read every step from L2 / Infinity Cache.
//
// Several independent episodes (E, each with its own W, labels, class weight and replica
// accumulators) run in the same launches: grid.z = E * shots.  A step is latency-bound (one
// dependent launch per SGD step), so E episodes share the ~200 launch boundaries of one.
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace cwt {

struct AdaptScalars {
  unsigned long long nbg, nfg;  // label counts (class 0 / class 1)
  float wfg;                    // CE class weight of class 1
  float lr_eff;                 // lr / sum_p w_{y_p}
};

// int64 labels -> u8 (0, 1, 255 for anything else) plus per-block label counts (no atomics,
// so nothing has to be zeroed first; adapt_setup_kernel sums the blocks in fixed order).
constexpr int PREP_MAXBLK = 256;
// Episode e = blockIdx.y owns lbl[e*total, (e+1)*total) and part[e][PREP_MAXBLK][2].
__global__ void adapt_prep_kernel(const int64_t* __restrict__ lbl, long total, uint8_t* __restrict__ out,
                                  unsigned long long* __restrict__ part) {
  lbl += (long)blockIdx.y * total;
  out += (long)blockIdx.y * total;
  part += (long)blockIdx.y * 2 * PREP_MAXBLK;
  unsigned long long nb = 0, nf = 0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    int64_t v = lbl[i];
    out[i] = (uint8_t)(v == 0 ? 0 : (v == 1 ? 1 : 255));
    nb += (v == 0);
    nf += (v == 1);
  }
  __shared__ unsigned long long red[2][16];
  for (int o = 32; o > 0; o >>= 1) {
    nb += __shfl_xor(nb, o, 64);
    nf += __shfl_xor(nf, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = nb;
    red[1][threadIdx.x >> 6] = nf;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long b = 0, f = 0;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) {
      b += red[0][i];
      f += red[1][i];
    }
    part[2 * blockIdx.x] = b;
    part[2 * blockIdx.x + 1] = f;
  }
}

// One block: label counts -> class weight and effective learning rate, the per-call pointers
// of the captured step graph, and the zeroing of the first accumulator slot (or of the CE
// loss numerator) -- one launch where there were two memsets and three kernels.
// mode 0: weight = [1, nbg/nfg]        (test.py:169-175, train.py:211-217)
// mode 1: weight = [1, nbg/(nfg+1e-12)] (train.py:237-243, query loss)
struct AdaptDevArgs;

constexpr int ADAPT_CB = 16;           // lo-res columns per workgroup
// dW[1] accumulator replicas: ~240 workgroups adding 2 KB each into ONE 2 KB row run at the
// contended atomic rate (~0.09 TB/s, ~5 us per step; MI355X_MICROARCH.md Global float
// atomics); spreading them over R rows (workgroup id % R) removes the contention and the
// next step sums the R rows when it loads W.
constexpr int ADAPT_RMAX = 32;                 // replica rows allocated per slot
constexpr int ADAPT_R_DEFAULT = 8;             // replica rows used (CWT_ADAPT_R overrides: 4, 8, 16 or 32)
constexpr int ADAPT_SLOT = ADAPT_RMAX * 512;   // floats per accumulator slot
constexpr int ADAPT_NP = 2 * (ADAPT_CB + 1);
constexpr int ADAPT_NSTAMP = 10;  // timing-study stamps per (step, workgroup)
constexpr long ADAPT_ESTRIDE = 3L * ADAPT_SLOT;  // accumulator floats per episode (3 slots)
constexpr int ADAPT_WSTRIDE = 2 * 1024;          // W ping-pong floats per episode
constexpr int ADAPT_PPW = (ADAPT_NP + 3) / 4;  // lo pixels per wave

// Per-call pointers, read by the kernels from device memory so that one captured graph of
// the 200 step launches serves every call with the same geometry.
struct AdaptDevArgs {
  const float* f;     // NHWC [n][h][w][512]
  const float* w_in;  // initial W [2][512]
  float* w_out;       // adapted W [2][512]
};

// One block per episode e = blockIdx.x: its scalars sc[e], its pointers dargs[e] (f + e *
// f_stride, w_in / w_out + e * w_stride) and the zeroing of zero[e * zero_stride + [0, nzero)).
__global__ void adapt_setup_kernel(const unsigned long long* __restrict__ part, int nblk, AdaptScalars* sc, float lr,
                                   int mode, AdaptDevArgs* dargs, const float* f, long f_stride, const float* w_in,
                                   float* w_out, int w_stride, float* zero, long zero_stride, int nzero,
                                   double* zero_d) {
  __shared__ unsigned long long red[2][PREP_MAXBLK];
  const int t = threadIdx.x;
  const int e = blockIdx.x;
  part += (long)e * 2 * PREP_MAXBLK;
  sc += e;
  if (zero) zero += (long)e * zero_stride;
  red[0][t] = t < nblk ? part[2 * t] : 0ull;
  red[1][t] = t < nblk ? part[2 * t + 1] : 0ull;
  __syncthreads();
  for (int o = PREP_MAXBLK / 2; o > 0; o >>= 1) {  // integer sums: order-independent
    if (t < o) {
      red[0][t] += red[0][t + o];
      red[1][t] += red[1][t + o];
    }
    __syncthreads();
  }
  if (t == 0) {
    const unsigned long long nbg = red[0][0], nfg = red[1][0];
    sc->nbg = nbg;
    sc->nfg = nfg;
    const double nb = (double)nbg, nf = (double)nfg;
    const double r = (mode == 0) ? nb / nf : nb / (nf + 1e-12);
    const float wfg = (float)r;  // torch.tensor([1.0, r]) -> float32
    sc->wfg = wfg;
    const double sumw = nb + nf * (double)wfg;
    sc->lr_eff = (float)((double)lr / sumw);
    if (dargs) {
      dargs[e].f = f + e * f_stride;
      dargs[e].w_in = w_in + (long)e * w_stride;
      dargs[e].w_out = w_out + (long)e * w_stride;
    }
    if (zero_d) *zero_d = 0.0;
  }
  if (zero)
    for (int i = t; i < nzero; i += blockDim.x) zero[i] = 0.f;
}

// Per-episode state e = blockIdx.z / nshot: dargs[e], sc[e], and the W / accumulator buffers
// below offset by e * ADAPT_WSTRIDE / e * ADAPT_ESTRIDE floats.
struct AdaptStepArgs {
  const AdaptDevArgs* dargs;
  const float* f;        // the library's copy of f_s, NHWC [E][n][h][w][512] (a direct global pointer:
                         // no per-step pointer chase, and global_load rather than flat_load)
  const uint8_t* lbl;    // [E][n][S][S]
  const AdaptScalars* sc;
  const float* w_src;    // W before the previous update ([2][512]); null at step 0 (dargs->w_in)
  const float* acc_prev; // dW[1] replicas [R][512] of the previous step, or null at step 0
  float* w_dst;          // block (0,0,0) stores the current W here (may be null)
  float* acc_cur;        // dW[1] replicas [R][512] of this step (zeroed)
  float* acc_zero;       // slot [R][512] to zero for the next step (may be null)
  int h, w, S, nshot, nep;  // shots per episode, episodes
  float sy, sx;          // align_corners scales (h-1)/(S-1), (w-1)/(S-1)
  int nrep;              // replica rows in use
  unsigned long long* stamps;  // CWT_ADAPT_DBG & 32: per (step, workgroup) ADAPT_NSTAMP clock stamps
  int step;
  int dbg;               // ablation flags for timing studies only (CWT_ADAPT_DBG): 1 skip replica
                         // reads, 2 skip the high-res pass, 4 skip the global atomics, 8 skip f loads,
                         // 16 return at entry
};

// Accumulate the weighted-CE gradient of high-res pixels of this tile into gs[ri][xi]
// (class-1 component; class 0 is its negative).  z[ri][xi][2] low-res logits in LDS.
// Returns this thread's sum of w_y * nll (used by the query loss).
template <bool WITH_LOSS>
__device__ __forceinline__ float hires_tile_grad(const float (*z)[ADAPT_CB + 1][2], float (*gs)[ADAPT_CB + 1],
                                                 const uint8_t* __restrict__ lbl, int S, int h, int w, int r,
                                                 int cb, int ncb, float sy, float sx, float wfg) {
  const int t = threadIdx.x;
  const int rg = t >> 7;
  const int x_begin = cb * 8 * ADAPT_CB;
  const int x_end = (cb == ncb - 1) ? S : min(S - 1, x_begin + 8 * ADAPT_CB);
  const int ylo = 8 * r + 4 * rg;
  const int yhi = (r == h - 2 && rg == 1) ? S : ylo + 4;  // last pair also owns row S-1
  float loss = 0.f;
  for (int X = x_begin + (t & 127); X < x_end; X += 128) {
    Lerp lx = lerp_coord(X, w, sx);
    const int xi0 = lx.i0 - cb * ADAPT_CB, xi1 = lx.i1 - cb * ADAPT_CB;
    float a00 = 0.f, a01 = 0.f, a10 = 0.f, a11 = 0.f;  // [row of i0/i1][x0/x1]
    float b0 = 0.f, b1 = 0.f;                          // contributions when i0 == i1 == r+1
    for (int Y = ylo; Y < yhi; ++Y) {
      const int y = lbl[(long)Y * S + X];
      if (y == 255) continue;
      Lerp ly = lerp_coord(Y, h, sy);
      const int ri0 = ly.i0 - r, ri1 = ly.i1 - r;
      float l0 = ly.l0 * (lx.l0 * z[ri0][xi0][0] + lx.l1 * z[ri0][xi1][0]) +
                 ly.l1 * (lx.l0 * z[ri1][xi0][0] + lx.l1 * z[ri1][xi1][0]);
      float l1 = ly.l0 * (lx.l0 * z[ri0][xi0][1] + lx.l1 * z[ri0][xi1][1]) +
                 ly.l1 * (lx.l0 * z[ri1][xi0][1] + lx.l1 * z[ri1][xi1][1]);
      const float d = l1 - l0;
      const float p1 = 1.f / (1.f + __expf(-d));
      const float wy = (y == 1) ? wfg : 1.f;
      const float g = wy * (p1 - (float)y);
      if (WITH_LOSS) {
        // nll = logsumexp(l) - l_y, computed stably
        const float m = fmaxf(l0, l1);
        const float lse = m + __logf(__expf(l0 - m) + __expf(l1 - m));
        loss += wy * (lse - (y == 1 ? l1 : l0));
      }
      if (ri0 == 0) {
        a00 += ly.l0 * lx.l0 * g;
        a01 += ly.l0 * lx.l1 * g;
        a10 += ly.l1 * lx.l0 * g;
        a11 += ly.l1 * lx.l1 * g;
      } else {  // Y = S-1: only row r+1 with weight 1
        b0 += lx.l0 * g;
        b1 += lx.l1 * g;
      }
    }
    atomicAdd(&gs[0][xi0], a00);
    atomicAdd(&gs[0][xi1], a01);
    atomicAdd(&gs[1][xi0], a10 + b0);
    atomicAdd(&gs[1][xi1], a11 + b1);
  }
  return loss;
}

constexpr int ADAPT_T = 1024;                          // threads per step workgroup
constexpr int ADAPT_NW = ADAPT_T / 64;                 // waves
constexpr int ADAPT_PPW16 = (ADAPT_NP + ADAPT_NW - 1) / ADAPT_NW;  // lo pixels per wave (3)

// One SGD step over one spatial tile (lo-res rows r, r+1; columns cb*16 .. cb*16+16) of
// every shot of G episodes (episode group blockIdx.z): the workgroup walks its T = G * shots
// tiles in turn, prefetching tile k+1's f and labels while it computes tile k, and adds one
// 2-KB dW row per episode.  (One workgroup per tile and shot would take ceil(T) rounds of
// the whole grid; the walk shares the launch, the W publish and the reduction.)
// Per tile, 16 waves: wave v owns hi-res row 8r + v/2 and 64 of the tile's 128 hi-res columns
// (one pixel per lane; with S-1 == 8(h-1) the interpolation weights are exact multiples of
// 1/8, so an aligned lane octet shares its two lo-res columns and is pre-reduced by DPP
// before one lane adds it into LDS).  Wave g < G reads episode g's W and R gradient replicas
// and publishes its current W through LDS.  f of the tile stays in registers between the z
// pass and the dW pass.
// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, not for its
// outstanding global loads (__syncthreads() would also drain vmcnt, i.e. wait for the next
// tile's prefetch).  Every cross-wave exchange in the step kernel goes through LDS.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// The loads of a tile are branch-free (clamped addresses, validity applied at use) so that
// they stay in flight across the previous tile's passes: a load under a divergent branch makes
// the compiler drain vmcnt at the join.
struct AdaptTile {
  float fv[ADAPT_PPW16][8];  // pixels past the tile / image hold a clamped (finite) pixel: their
                             // zd is never read and their gs stays 0
  int y_main[2], y_extra[2];  // raw label bytes; y_in / y_ex_in below say which are real
};

template <int G, bool STAMPS>  // STAMPS: the timing-study build (CWT_ADAPT_DBG & 32), never the timed one
__global__ __launch_bounds__(ADAPT_T) void adapt_step_kernel(AdaptStepArgs a) {
  constexpr int C = 512;
  __shared__ float wl[G][2][C];
  __shared__ float zd[2][ADAPT_CB + 1];  // z1 - z0: the softmax over two classes needs only the difference
  __shared__ float gs[2][2][ADAPT_CB + 1];  // double-buffered over tiles
  __shared__ float red[ADAPT_NW][C];
  if (a.dbg & 16) return;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int cb = blockIdx.x, r = blockIdx.y;
  unsigned long long* stp = nullptr;  // timing study (CWT_ADAPT_DBG & 32): wave 0's clock at each phase
  if (STAMPS && t == 0) {
    stp = a.stamps + ((long)a.step * gridDim.x * gridDim.y * gridDim.z + blockIdx.x +
                      gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)) * ADAPT_NSTAMP;
    stp[0] = __builtin_amdgcn_s_memrealtime();
    stp[1] = __builtin_amdgcn_s_memtime();
  }
  auto stamp = [&](int i) {
    if (STAMPS && stp) stp[i] = __builtin_amdgcn_s_memtime();
  };
  const int ep0 = blockIdx.z * G;
  const int ng = min(G, a.nep - ep0);  // episodes of this group
  const int T = ng * a.nshot;           // tiles walked
  const int ncb = gridDim.x;
  const int S = a.S;
  const int x0 = cb * ADAPT_CB;
  const int ncol = min(ADAPT_CB + 1, a.w - x0);
  const int x_begin = cb * 8 * ADAPT_CB;
  const int x_end = (cb == ncb - 1) ? S : x_begin + 8 * ADAPT_CB;
  const int Y = 8 * r + (wv >> 1);
  // rows 8r .. 8r+7 belong to this pair; the last pair also owns row S-1 (waves 0, 1)
  const bool extra = (r == a.h - 2) && (wv >> 1) == 0;
  const int xw = x_begin + 64 * (wv & 1);        // wave-uniform column base (+128 per round)
  const int nrounds = (x_end - xw + 127) / 128;  // 1, or 2 when the last block has 129 columns
  const bool first_blk = (cb | r) == 0;          // the tile (0, 0) workgroup also keeps the episode's W history

  // ---- loads that do not depend on W: the tile's f pixels and this lane's labels ----
  bool y_in[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) y_in[kk] = kk < nrounds && xw + 128 * kk + lane < x_end;
  auto load_tile = [&](AdaptTile& tl, int k) {
    const float* fimg = a.f + (long)(ep0 * a.nshot + k) * a.h * a.w * C;
#pragma unroll
    for (int j = 0; j < ADAPT_PPW16; ++j) {
      const int p = min(wv + ADAPT_NW * j, ADAPT_NP - 1);
      const int ri = p / (ADAPT_CB + 1), xi = min(p % (ADAPT_CB + 1), ncol - 1);
      const float* src = fimg + ((long)(r + ri) * a.w + x0 + xi) * C + lane * 8;
      const f32x4 u = *(const f32x4*)src, v = *(const f32x4*)(src + 4);
      tl.fv[j][0] = u[0]; tl.fv[j][1] = u[1]; tl.fv[j][2] = u[2]; tl.fv[j][3] = u[3];
      tl.fv[j][4] = v[0]; tl.fv[j][5] = v[1]; tl.fv[j][6] = v[2]; tl.fv[j][7] = v[3];
    }
    const uint8_t* lbl = a.lbl + (long)(ep0 * a.nshot + k) * S * S;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int X = min(xw + 128 * kk + lane, S - 1);
      tl.y_main[kk] = lbl[(long)Y * S + X];
      tl.y_extra[kk] = lbl[(long)(S - 1) * S + X];
    }
  };
  AdaptTile cur;
  load_tile(cur, 0);
  float wfg_g[G];  // class-1 CE weight per episode, read once (a load inside the tile loop would
                   // drain the prefetch)
#pragma unroll
  for (int g = 0; g < G; ++g) wfg_g[g] = a.sc[ep0 + min(g, ng - 1)].wfg;

  // ---- current W (wave g < ng, episode ep0 + g): W_src - lr_eff * sum of the previous step's replicas ----
  if (wv < ng) {
    const int ep = ep0 + wv;
    const long eacc = ep * ADAPT_ESTRIDE, ew = (long)ep * ADAPT_WSTRIDE;
    const float lr = a.sc[ep].lr_eff;
    const float* wsrc = a.w_src ? a.w_src + ew : a.dargs[ep].w_in;
    f32x4 w0a = *(const f32x4*)(wsrc + lane * 8), w0b = *(const f32x4*)(wsrc + lane * 8 + 4);
    f32x4 w1a = *(const f32x4*)(wsrc + C + lane * 8), w1b = *(const f32x4*)(wsrc + C + lane * 8 + 4);
    if (a.acc_prev && !(a.dbg & 1)) {
      f32x4 d0 = {0.f, 0.f, 0.f, 0.f}, d1 = {0.f, 0.f, 0.f, 0.f};
      const float* ap = a.acc_prev + eacc + lane * 8;
      if (a.nrep == ADAPT_R_DEFAULT) {  // all replica loads in flight together
        f32x4 v0[ADAPT_R_DEFAULT], v1[ADAPT_R_DEFAULT];
#pragma unroll
        for (int rr = 0; rr < ADAPT_R_DEFAULT; ++rr) {
          v0[rr] = *(const f32x4*)(ap + rr * 512);
          v1[rr] = *(const f32x4*)(ap + rr * 512 + 4);
        }
#pragma unroll
        for (int rr = 0; rr < ADAPT_R_DEFAULT; ++rr) {
          d0 += v0[rr];
          d1 += v1[rr];
        }
      } else {
#pragma unroll 4
        for (int rr = 0; rr < a.nrep; ++rr) {
          d0 += *(const f32x4*)(ap + rr * 512);
          d1 += *(const f32x4*)(ap + rr * 512 + 4);
        }
      }
      w1a -= lr * d0;
      w0a += lr * d0;
      w1b -= lr * d1;
      w0b += lr * d1;
    }
    *(f32x4*)&wl[wv][0][lane * 8] = w0a;
    *(f32x4*)&wl[wv][0][lane * 8 + 4] = w0b;
    *(f32x4*)&wl[wv][1][lane * 8] = w1a;
    *(f32x4*)&wl[wv][1][lane * 8 + 4] = w1b;
    if (first_blk && a.w_dst) {
      float* wd = a.w_dst + ew;
      *(f32x4*)(wd + lane * 8) = w0a;
      *(f32x4*)(wd + lane * 8 + 4) = w0b;
      *(f32x4*)(wd + C + lane * 8) = w1a;
      *(f32x4*)(wd + C + lane * 8 + 4) = w1b;
    }
  }
  if (first_blk && a.acc_zero)
    for (int g = 0; g < ng; ++g)
      for (int i = t; i < a.nrep * 128; i += ADAPT_T)
        ((f32x4*)(a.acc_zero + (ep0 + g) * ADAPT_ESTRIDE))[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (t < ADAPT_NP) (&gs[0][0][0])[t] = 0.f;
  stamp(2);
  lds_barrier();
  stamp(3);

  const float inv8 = 0.125f;
  float d[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) d[q] = 0.f;
  if (STAMPS && stp) {  // timing study: when tile 0's f and labels have landed
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stp[9] = __builtin_amdgcn_s_memtime();
  }
  for (int k = 0; k < T; ++k) {
    const int g = k / a.nshot, n = k - g * a.nshot;
    const int buf = k & 1;
    AdaptTile nxt;
    if (k + 1 < T) load_tile(nxt, k + 1);  // in flight during this tile's passes

    // ---- zd = (W1 - W0) . f for the tile's low-res pixels ----
    {
      float dw[8];
      const f32x4 a0 = *(const f32x4*)&wl[g][0][lane * 8], b0 = *(const f32x4*)&wl[g][0][lane * 8 + 4];
      const f32x4 a1 = *(const f32x4*)&wl[g][1][lane * 8], b1 = *(const f32x4*)&wl[g][1][lane * 8 + 4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        dw[q] = a1[q] - a0[q];
        dw[4 + q] = b1[q] - b0[q];
      }
      float sd[ADAPT_PPW16];
#pragma unroll
      for (int j = 0; j < ADAPT_PPW16; ++j) {
        float s = 0.f;
#pragma unroll
        for (int q = 0; q < 8; ++q) s = fmaf(dw[q], cur.fv[j][q], s);
        sd[j] = s;
      }
#pragma unroll
      for (int j = 0; j < ADAPT_PPW16; ++j) sd[j] = wave_sum_dpp(sd[j]);  // independent chains interleave
#pragma unroll
      for (int j = 0; j < ADAPT_PPW16; ++j) {
        const int p = wv + ADAPT_NW * j;
        if (p < ADAPT_NP && lane == 0) (&zd[0][0])[p] = sd[j];
      }
    }
    lds_barrier();
    if (k == 0) stamp(4);
    // the other gs buffer was last read by the previous tile's dW pass, which every thread
    // finished before the barrier above
    if (t < ADAPT_NP) (&gs[buf ^ 1][0][0])[t] = 0.f;

    // ---- hi-res pass: weighted-CE gradient, bilinear adjoint into gs (class-1 component) ----
    if (!(a.dbg & 2)) {
      const float wfg = G == 1 ? wfg_g[0] : (g == 0 ? wfg_g[0] : wfg_g[G - 1]);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        if (kk >= nrounds) break;  // wave-uniform
        const int X = xw + 128 * kk + lane;
        const bool xin = X < x_end;
        // x interpolation, exact: S-1 == 8(w-1) so src = X/8
        const int ix = min(X >> 3, a.w - 1);
        const int xi0 = ix - x0, xi1 = (ix < a.w - 1) ? xi0 + 1 : xi0;
        const float lx1 = (float)(X & 7) * inv8, lx0 = 1.f - lx1;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          if (e == 1 && !extra) break;  // wave-uniform
          const int y = !y_in[kk] ? 255 : e ? cur.y_extra[kk] : cur.y_main[kk];
          // row S-1 reads lo row r+1 with weight 1; rows 8r+i read rows r, r+1 with (1-i/8, i/8)
          const int ri0 = e, ri1 = 1;
          const float ly1 = e ? 0.f : (float)(Y & 7) * inv8, ly0 = 1.f - ly1;
          float gv = 0.f;
          if (xin && y != 255) {
            const float dd = ly0 * (lx0 * zd[ri0][xi0] + lx1 * zd[ri0][xi1]) + ly1 * (lx0 * zd[ri1][xi0] + lx1 * zd[ri1][xi1]);
            const float p1 = __builtin_amdgcn_rcpf(1.f + __expf(-dd));
            gv = ((y == 1) ? wfg : 1.f) * (p1 - (float)y);
          }
          // ly0 / ly1 are wave-uniform: reduce lx * g over the octet once, scale per row after
          const float sa = octet_sum(lx0 * gv), sb = octet_sum(lx1 * gv);
          const float v00 = ly0 * sa, v01 = ly0 * sb, v10 = ly1 * sa, v11 = ly1 * sb;
          if ((lane & 7) == 0 && xin) {
            if (e == 0) {
              atomicAdd(&gs[buf][0][xi0], v00);
              atomicAdd(&gs[buf][0][xi1], v01);
            }
            atomicAdd(&gs[buf][1][xi0], v10 + (e ? v00 : 0.f));
            atomicAdd(&gs[buf][1][xi1], v11 + (e ? v01 : 0.f));
          }
        }
      }
    }
    lds_barrier();
    if (k == 0) stamp(5);

    // ---- dW[1] partial += sum_p g[p] f[p] over the tile ----
#pragma unroll
    for (int j = 0; j < ADAPT_PPW16; ++j) {
      const int p = wv + ADAPT_NW * j;
      if (p < ADAPT_NP) {
        const float gp = (&gs[buf][0][0])[p];
#pragma unroll
        for (int q = 0; q < 8; ++q) d[q] = fmaf(gp, cur.fv[j][q], d[q]);
      }
    }
    if (n == a.nshot - 1) {  // last shot of episode ep0 + g: reduce over waves, one 2-KB atomic row
      *(f32x4*)&red[wv][lane * 8] = f32x4{d[0], d[1], d[2], d[3]};
      *(f32x4*)&red[wv][lane * 8 + 4] = f32x4{d[4], d[5], d[6], d[7]};
#pragma unroll
      for (int q = 0; q < 8; ++q) d[q] = 0.f;
      lds_barrier();
      if (k == 0) stamp(6);
      if (t < C && !(a.dbg & 4)) {
        float s = 0.f;
#pragma unroll
        for (int v = 0; v < ADAPT_NW; ++v) s += red[v][t];
        atomicAdd(&a.acc_cur[(ep0 + g) * ADAPT_ESTRIDE + ((blockIdx.x + gridDim.x * blockIdx.y) % a.nrep) * 512 + t],
                  s);
      }
      // red is rewritten only after the next episode's tiles, i.e. after >= 2 more barriers
    }
    if (k + 1 < T) cur = nxt;
  }
  if (STAMPS && stp) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // thread 0's atomic has been performed
    stp[7] = __builtin_amdgcn_s_memtime();
    stp[8] = __builtin_amdgcn_s_memrealtime();
  }
}

__global__ void adapt_final_kernel(const float* w_src, const float* acc, const AdaptScalars* sc,
                                   const AdaptDevArgs* dargs, int nrep) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= 512) return;
  const int ep = blockIdx.y;
  w_src += (long)ep * ADAPT_WSTRIDE;
  if (acc) acc += ep * ADAPT_ESTRIDE;
  sc += ep;
  dargs += ep;
  float* w_out = dargs->w_out;
  const float lr = sc->lr_eff;
  float d = 0.f;
  if (acc)
    for (int rr = 0; rr < nrep; ++rr) d += acc[rr * 512 + k];
  w_out[k] = w_src[k] + lr * d;
  w_out[512 + k] = w_src[512 + k] - lr * d;
}

// The 200 step launches + the final update, enqueued on `st` (directly or while capturing).
// timing study buffer (CWT_ADAPT_DBG & 32), read back by cwt_debug_adapt_stamps
unsigned long long* g_adapt_stamps = nullptr;
long g_adapt_stamps_n = 0;

static int enqueue_adapt_steps(const AdaptDevArgs* dargs, const float* f_ws, const uint8_t* lbl_ws,
                               const AdaptScalars* sc, float* acc3, float* wbuf, int E, int n, int h, int w, int S,
                               int iters, hipStream_t st) {
  AdaptStepArgs a;
  a.dargs = dargs;
  a.f = f_ws;
  a.lbl = lbl_ws;
  a.sc = sc;
  a.h = h;
  a.w = w;
  a.S = S;
  a.nshot = n;
  a.nep = E;
  a.sy = align_corners_scale(h, S);
  a.sx = align_corners_scale(w, S);
  const char* dbg = getenv("CWT_ADAPT_DBG");
  a.dbg = dbg ? atoi(dbg) : 0;
  a.stamps = nullptr;
  const char* nr = getenv("CWT_ADAPT_R");
  a.nrep = nr ? atoi(nr) : ADAPT_R_DEFAULT;
  if (a.nrep != 4 && a.nrep != 8 && a.nrep != 16 && a.nrep != 32) a.nrep = ADAPT_R_DEFAULT;
  const int ncb = cdiv(S - 1, 8 * ADAPT_CB);
  // episodes per workgroup: 2 when there are several (shares the launch between them)
  const char* gs_env = getenv("CWT_ADAPT_G");
  const int G = (gs_env ? atoi(gs_env) : 2) >= 2 && E > 1 ? 2 : 1;
  dim3 grid(ncb, h - 1, cdiv(E, G));
  if (a.dbg & 32) {
    if ((long)iters * grid.x * grid.y * grid.z * ADAPT_NSTAMP > g_adapt_stamps_n)
      return fail(CWT_ESTATE, "timing-study stamp buffer too small");
    a.stamps = g_adapt_stamps;
  }
  for (int s = 0; s < iters; ++s) {
    a.step = s;
    a.w_src = (s == 0) ? nullptr : wbuf + ((s - 1) & 1) * 1024;
    a.acc_prev = (s == 0) ? nullptr : acc3 + ((s - 1) % 3) * ADAPT_SLOT;
    a.w_dst = wbuf + (s & 1) * 1024;
    a.acc_cur = acc3 + (s % 3) * ADAPT_SLOT;
    a.acc_zero = acc3 + ((s + 1) % 3) * ADAPT_SLOT;
    if (a.stamps) {
      if (G == 2)
        hipLaunchKernelGGL((adapt_step_kernel<2, true>), grid, dim3(ADAPT_T), 0, st, a);
      else
        hipLaunchKernelGGL((adapt_step_kernel<1, true>), grid, dim3(ADAPT_T), 0, st, a);
    } else if (G == 2) {
      hipLaunchKernelGGL((adapt_step_kernel<2, false>), grid, dim3(ADAPT_T), 0, st, a);
    } else {
      hipLaunchKernelGGL((adapt_step_kernel<1, false>), grid, dim3(ADAPT_T), 0, st, a);
    }
    CWT_LAUNCH_CHECK();
  }
  const int last = iters - 1;
  hipLaunchKernelGGL(adapt_final_kernel, dim3(2, E), dim3(256), 0, st, (const float*)(wbuf + (last & 1) * 1024),
                     (const float*)(acc3 + (last % 3) * ADAPT_SLOT), sc, dargs, a.nrep);
  CWT_LAUNCH_CHECK();
  return 0;
}

AdaptGraphCache::~AdaptGraphCache() {
  for (auto& e : entries) (void)hipGraphExecDestroy(e.exec);
  if (cap_stream) (void)hipStreamDestroy(cap_stream);
}

size_t adapt_ws_sizes(int E, int n, int h, int w, int S, size_t* fws, size_t* lbl, size_t* sc, size_t* acc,
                      size_t* wbuf, size_t* dargs) {
  *fws = (size_t)E * n * h * w * 512 * sizeof(float);
  *lbl = (size_t)E * n * S * S;
  *sc = (size_t)E * (sizeof(AdaptScalars) + 2 * PREP_MAXBLK * sizeof(unsigned long long)) + 64;
  *acc = (size_t)E * ADAPT_ESTRIDE * sizeof(float);
  *wbuf = (size_t)E * ADAPT_WSTRIDE * sizeof(float);
  *dargs = (size_t)E * sizeof(AdaptDevArgs);
  return 0;
}

// E episodes of n shots each: f [E][n][h][w][512], lbl64 [E][n][S][S], W [E][2][512].
int launch_adapt(const float* f, const int64_t* lbl64, int E, int n, int h, int w, int S, float lr, int iters,
                 float* W, float* f_ws /*[E][n][h][w][512]*/, uint8_t* lbl_ws, AdaptScalars* sc /*[E] + partial counts*/,
                 float* acc3 /*[E][3][R][512]*/, float* wbuf /*[E][2][2][512]*/, AdaptDevArgs* dargs /*[E]*/,
                 AdaptGraphCache* cache, hipStream_t st) {
  const long total = (long)n * S * S;  // labels per episode
  // the step graph reads f from the library's buffer (fixed address, baked into the graph)
  if (iters > 0 && f != f_ws)
    CWT_HIP(hipMemcpyAsync(f_ws, f, (size_t)E * n * h * w * 512 * sizeof(float), hipMemcpyDeviceToDevice, st));
  unsigned long long* part = (unsigned long long*)(sc + E);  // [E][PREP_MAXBLK][2] after the scalars
  const int pblocks = (int)std::min<long>(PREP_MAXBLK, cdiv(total, 1024));
  hipLaunchKernelGGL(adapt_prep_kernel, dim3(pblocks, E), dim3(1024), 0, st, lbl64, total, lbl_ws, part);
  CWT_LAUNCH_CHECK();
  hipLaunchKernelGGL(adapt_setup_kernel, dim3(E), dim3(PREP_MAXBLK), 0, st, (const unsigned long long*)part, pblocks,
                     sc, lr, 0, dargs, f, (long)n * h * w * 512, (const float*)W, W, 1024,
                     iters > 0 ? acc3 : (float*)nullptr, ADAPT_ESTRIDE, ADAPT_SLOT, (double*)nullptr);
  CWT_LAUNCH_CHECK();
  if (iters <= 0) return 0;
  const char* dbg = getenv("CWT_ADAPT_DBG");
  if (dbg && (atoi(dbg) & 32)) {  // timing study: stamp buffer sized for G = 1 (allocated outside any capture)
    const long n_st = (long)iters * cdiv(S - 1, 8 * ADAPT_CB) * (h - 1) * E * ADAPT_NSTAMP;
    if (n_st > g_adapt_stamps_n) {
      CWT_HIP(hipDeviceSynchronize());
      if (g_adapt_stamps) CWT_HIP(hipFree(g_adapt_stamps));
      CWT_HIP(hipMalloc(&g_adapt_stamps, n_st * sizeof(unsigned long long)));
      g_adapt_stamps_n = n_st;
    }
  }
  if (!cache) return enqueue_adapt_steps(dargs, f_ws, lbl_ws, sc, acc3, wbuf, E, n, h, w, S, iters, st);
  // graph path: one instantiated graph per (geometry, workspace pointers)
  AdaptGraphCache::Entry key{E, n, h, w, S, iters, (const void*)f_ws, (const void*)lbl_ws, (const void*)sc,
                             (const void*)acc3, (const void*)wbuf, (const void*)dargs, nullptr};
  hipGraphExec_t exec = nullptr;
  for (auto& e : cache->entries)
    if (e.same(key)) exec = e.exec;
  if (!exec) {
    if (!cache->cap_stream) CWT_HIP(hipStreamCreateWithFlags(&cache->cap_stream, hipStreamNonBlocking));
    hipGraph_t g;
    CWT_HIP(hipStreamBeginCapture(cache->cap_stream, hipStreamCaptureModeThreadLocal));
    int rc = enqueue_adapt_steps(dargs, f_ws, lbl_ws, sc, acc3, wbuf, E, n, h, w, S, iters, cache->cap_stream);
    hipError_t e2 = hipStreamEndCapture(cache->cap_stream, &g);
    if (rc) return rc;
    if (e2 != hipSuccess) return fail((int)e2, std::string("adapt graph capture: ") + hipGetErrorString(e2));
    hipError_t e3 = hipGraphInstantiate(&exec, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (e3 != hipSuccess) return fail((int)e3, std::string("adapt graph instantiate: ") + hipGetErrorString(e3));
    key.exec = exec;
    cache->entries.push_back(key);
  }
  CWT_HIP(hipGraphLaunch(exec, st));
  return 0;
}

// ---------------------------------------------------------------------------------------
// Outer-loop query CE (train.py:237-243,261-265) on precomputed low-res logits:
// loss = sum w_y nll / sum w_y, dlogits = U^T (w_y (p - onehot)) / sum w_y.
// Same tiling as the inner-loop step; logits read from memory instead of W . f.
// ---------------------------------------------------------------------------------------
struct SegCEArgs {
  const float* logits;  // [B][2][h][w]
  const uint8_t* lbl;   // [B][S][S]
  const AdaptScalars* sc;
  float* dlogits;       // [B][2][h][w], zeroed; accumulates U^T g (unscaled)
  double* loss_num;     // [1] sum w nll
  int h, w, S;
  float sy, sx;
};

__global__ __launch_bounds__(256) void seg_ce_kernel(SegCEArgs a) {
  __shared__ float z[2][ADAPT_CB + 1][2];
  __shared__ float gs[2][ADAPT_CB + 1];
  __shared__ float lsum[4];
  const int t = threadIdx.x;
  const int cb = blockIdx.x, r = blockIdx.y, b = blockIdx.z;
  const int ncb = gridDim.x;
  const int x0 = cb * ADAPT_CB;
  const int ncol = min(ADAPT_CB + 1, a.w - x0);
  const long plane = (long)a.h * a.w;
  if (t < 2 * (ADAPT_CB + 1)) {
    const int ri = t / (ADAPT_CB + 1), xi = t % (ADAPT_CB + 1);
    gs[ri][xi] = 0.f;
    if (xi < ncol) {
      z[ri][xi][0] = a.logits[(long)b * 2 * plane + (long)(r + ri) * a.w + x0 + xi];
      z[ri][xi][1] = a.logits[(long)b * 2 * plane + plane + (long)(r + ri) * a.w + x0 + xi];
    }
  }
  __syncthreads();
  float l = hires_tile_grad<true>(z, gs, a.lbl + (long)b * a.S * a.S, a.S, a.h, a.w, r, cb, ncb, a.sy, a.sx,
                                  a.sc->wfg);
  l = wave_sum(l);
  if ((t & 63) == 0) lsum[t >> 6] = l;
  __syncthreads();
  if (t == 0) atomicAdd(a.loss_num, (double)((lsum[0] + lsum[1]) + (lsum[2] + lsum[3])));
  if (t < 2 * (ADAPT_CB + 1)) {
    const int ri = t / (ADAPT_CB + 1), xi = t % (ADAPT_CB + 1);
    if (xi < ncol) {
      const float g = gs[ri][xi];
      const long off = (long)b * 2 * plane + (long)(r + ri) * a.w + x0 + xi;
      atomicAdd(&a.dlogits[off + plane], g);
      atomicAdd(&a.dlogits[off], -g);
    }
  }
}

__global__ void seg_ce_final_kernel(const AdaptScalars* sc, const double* loss_num, float* loss_out, float* dlogits,
                                    long n) {
  const double sumw = (double)sc->nbg + (double)sc->nfg * (double)sc->wfg;
  const float inv = (float)(1.0 / sumw);
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) loss_out[0] = (float)(loss_num[0] / sumw);
  for (; i < n; i += (long)gridDim.x * blockDim.x) dlogits[i] *= inv;
}

int launch_seg_ce(const float* logits, const int64_t* target, int B, int h, int w, int S, float* loss_out,
                  float* dlogits, uint8_t* lbl_ws, AdaptScalars* sc, double* loss_num, hipStream_t st) {
  const long total = (long)B * S * S;
  unsigned long long* part = (unsigned long long*)(sc + 1);
  const int pblocks = (int)std::min<long>(PREP_MAXBLK, cdiv(total, 1024));
  hipLaunchKernelGGL(adapt_prep_kernel, dim3(pblocks, 1), dim3(1024), 0, st, target, total, lbl_ws, part);
  CWT_LAUNCH_CHECK();
  hipLaunchKernelGGL(adapt_setup_kernel, dim3(1), dim3(PREP_MAXBLK), 0, st, (const unsigned long long*)part, pblocks,
                     sc, 1.0f, 1, (AdaptDevArgs*)nullptr, (const float*)nullptr, 0L, (const float*)nullptr,
                     (float*)nullptr, 0, dlogits, 0L, B * 2 * h * w, loss_num);
  CWT_LAUNCH_CHECK();
  SegCEArgs a;
  a.logits = logits;
  a.lbl = lbl_ws;
  a.sc = sc;
  a.dlogits = dlogits;
  a.loss_num = loss_num;
  a.h = h;
  a.w = w;
  a.S = S;
  a.sy = align_corners_scale(h, S);
  a.sx = align_corners_scale(w, S);
  dim3 grid(cdiv(S - 1, 8 * ADAPT_CB), h - 1, B);
  hipLaunchKernelGGL(seg_ce_kernel, grid, dim3(256), 0, st, a);
  CWT_LAUNCH_CHECK();
  long n = (long)B * 2 * h * w;
  hipLaunchKernelGGL(seg_ce_final_kernel, dim3(cdiv(n, 256)), dim3(256), 0, st, (const AdaptScalars*)sc,
                     (const double*)loss_num, loss_out, dlogits, n);
  CWT_LAUNCH_CHECK();
  return 0;
}

}  // namespace cwt

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
#include <type_traits>

#include "common.h"
#include "kernels.h"
#include "tail_body.h"

namespace cwt {

struct AdaptScalars {
  unsigned long long nbg, nfg;  // label counts (class 0 / class 1)
  float wfg;                    // CE class weight of class 1
  float lr_eff;                 // lr / sum_p w_{y_p}
  // the persistent loop's dW[1] exchange in 64-bit fixed point (exact, order-free integer sums:
  // deterministic): value = integer * fx_inv, integer = rint(partial * fx_scale), fx_scale = 2^k
  // with every sum below 2^58: |dW[1]_c| <= max|f| * sum_p |g_p| <= max|f| * sum_p w_{y_p} (the
  // loop's per-pixel CE gradients are w_y (p - onehot), unnormalised, and the bilinear adjoint
  // keeps the L1 norm); the quantum 2^-k is ~2^-57 of that bound.  A non-finite f gives
  // fx_scale 0 and fx_inv NaN: W becomes NaN, as the reference's would
  double fx_scale, fx_inv;
};

// int64 labels -> u8 (0, 1, 255 for anything else) plus per-block label counts (no atomics,
// so nothing has to be zeroed first; adapt_setup_kernel sums the blocks in fixed order).
constexpr int PREP_MAXBLK = 256;
// Episode e = blockIdx.y owns lbl[e*total, (e+1)*total) and part[e][PREP_MAXBLK][2].
// f (optional, [E][fcount]): per-block max of |f| as float bits (an unsigned max: NaN and Inf
// above every finite value) into fpart[e][block], for the fixed-point scale of AdaptScalars.
__global__ void adapt_prep_kernel(const int64_t* __restrict__ lbl, long total, uint8_t* __restrict__ out,
                                  unsigned long long* __restrict__ part, const float* __restrict__ f = nullptr,
                                  long fcount = 0, unsigned* __restrict__ fpart = nullptr) {
  lbl += (long)blockIdx.y * total;
  out += (long)blockIdx.y * total;
  part += (long)blockIdx.y * 2 * PREP_MAXBLK;
  if (f) {
    const float* fe = f + (long)blockIdx.y * fcount;
    unsigned mb = 0u;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < fcount / 4; i += (long)gridDim.x * blockDim.x) {
      const f32x4 v = ((const f32x4*)fe)[i];
      mb = max(max(mb, __float_as_uint(fabsf(v[0]))), __float_as_uint(fabsf(v[1])));
      mb = max(max(mb, __float_as_uint(fabsf(v[2]))), __float_as_uint(fabsf(v[3])));
    }
    for (int o = 32; o > 0; o >>= 1) mb = max(mb, (unsigned)__shfl_xor((int)mb, o, 64));
    __shared__ unsigned fred[16];
    if ((threadIdx.x & 63) == 0) fred[threadIdx.x >> 6] = mb;
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int i = 0; i < (int)(blockDim.x >> 6); ++i) mb = max(mb, fred[i]);
      fpart[(long)blockIdx.y * PREP_MAXBLK + blockIdx.x] = mb;
    }
  }
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
constexpr long ADAPT_ESTRIDE = 4L * ADAPT_SLOT;  // accumulator floats per episode (3 float slots; the
                                                 // persistent loop's 4 int64 slots of 16 rows)
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
                                   double* zero_d, unsigned* zero_u = nullptr, int nzero_u = 0,
                                   const unsigned* fpart = nullptr) {
  __shared__ unsigned long long red[2][PREP_MAXBLK];
  __shared__ unsigned fred[PREP_MAXBLK];
  const int t = threadIdx.x;
  const int e = blockIdx.x;
  part += (long)e * 2 * PREP_MAXBLK;
  sc += e;
  if (zero) zero += (long)e * zero_stride;
  red[0][t] = t < nblk ? part[2 * t] : 0ull;
  red[1][t] = t < nblk ? part[2 * t + 1] : 0ull;
  fred[t] = (fpart && t < nblk) ? fpart[(long)e * PREP_MAXBLK + t] : 0u;
  __syncthreads();
  for (int o = PREP_MAXBLK / 2; o > 0; o >>= 1) {  // integer sums / maxima: order-independent
    if (t < o) {
      red[0][t] += red[0][t + o];
      red[1][t] += red[1][t + o];
      fred[t] = max(fred[t], fred[t + o]);
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
    // fixed-point scale of the dW exchange: every sum below 2^58 (see AdaptScalars).  The loop's
    // per-pixel gradients are unnormalised (the 1 / sum_p w_{y_p} rides in lr_eff), so
    // |dW[1]_c| <= max|f| * sumw
    const unsigned mb = fred[0];
    if (mb >= 0x7f800000u) {  // NaN / Inf in f
      sc->fx_scale = 0.0;
      sc->fx_inv = __builtin_nan("");
    } else {
      const double bound = (double)__uint_as_float(mb) * (sumw > 1.0 ? sumw : 1.0);
      const int k = bound > 0.0 ? 57 - ilogb(bound) : 0;  // bound < 2^(ilogb + 1)
      sc->fx_scale = ldexp(1.0, k);
      sc->fx_inv = ldexp(1.0, -k);
    }
    if (dargs) {
      dargs[e].f = f + e * f_stride;
      dargs[e].w_in = w_in + (long)e * w_stride;
      dargs[e].w_out = w_out + (long)e * w_stride;
    }
    if (zero_d) *zero_d = 0.0;
  }
  if (zero)
    for (int i = t; i < nzero; i += blockDim.x) zero[i] = 0.f;
  if (zero_u && e == 0)
    for (int i = t; i < nzero_u; i += blockDim.x) zero_u[i] = 0u;
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
  const int t = threadIdx.x, lane = t & 63, wv = __builtin_amdgcn_readfirstlane(t >> 6);  // wv: SGPR
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

// ---------------------------------------------------------------------------------------
// Persistent inner loop: all `iters` SGD steps of every episode in ONE launch.
//
// The step kernel above pays, per step, a dependent-launch boundary (~1.8 us), the dispatch
// skew of ~240 workgroups and a W publish that re-reads the previous step's replicas, and it
// re-streams f_s from L2 every step.  Here G <= #CU workgroups (one per CU) stay resident for
// the whole loop:
//   * a unit = one step-kernel tile (lo-res rows r, r+1 x PA_NC columns incl. the right halo,
//     i.e. 64 lo-res pixels) of one shot of one episode; workgroup g owns units
//     [g*U/G, (g+1)*U/G).  A 1-shot 473^2 episode has 2 x 59 = 118 units, 641^2 3 x 80 = 240.
//   * wave v owns channels [32v, 32v+32) and lane p lo-res pixel p of the unit, so f_s of a
//     unit is 32 VGPRs per lane: with one unit per workgroup it is loaded ONCE and stays in
//     registers for all 200 steps (no per-step f traffic at all); with more it is streamed.
//   * z = (W1-W0).f per pixel: 32 FMAs per lane against the wave's slice of d = W1-W0 (LDS
//     broadcast), then the 16 per-wave partials are summed in fixed order.
//   * hi-res pass: the step kernel's (one pixel per lane, octet pre-reduction by DPP), but
//     each octet writes its two adjoint terms to slots of its own (no LDS atomics; the 16
//     slots of a lo-res pixel are summed in fixed order).
//   * dW[1] = sum_p g_p f_p: 32 FMAs per lane per unit, then a 64-lane butterfly
//     (pa_butterfly) leaves lane 2c+{0,1} holding channel 32v+c; 32 no-return 64-bit
//     fixed-point integer atomics per wave into replica row (g % nrep) of the step's slot (round 6:
//     exact and order-free, so the loop is deterministic; they execute at the memory side).
//   * grid barrier: every wave waits for its atomics (vmcnt(0)), workgroup barrier, one lane
//     adds 1 to arrival counter (g % nrep) (agent scope); wave 0 polls the counters with sc1
//     loads until they sum to G*(s+1) (MI355X_MICROARCH.md hand-off table, counter row); every
//     workgroup then reads the slot's replica rows with sc1 loads and applies W1 -= lr_eff*D,
//     W0 += lr_eff*D in the same order, so W stays identical everywhere.
//     (A barrier-free variant -- 64-bit fixed-point adds carrying a contribution count, polled
//     element by element -- was exact and deterministic but 1.7x slower per step: 118 x 1024
//     threads polling the same 32 KB contend with the adds at the memory side.)
//   * slots: step s adds into slot s%4; at the start of step s every workgroup zeroes its 1/G
//     share of slot (s+2)%4 (its last readers passed barrier s-1; its next adders start after
//     barrier s+1; the write-through zero stores are complete when the workgroup arrives at
//     barrier s).  (One workgroup zeroing the whole slot made it the last arriver of most steps.)
// Every spin is bounded: a barrier that does not complete within ~4 s sets the error word and
// the grid exits (wrong W, no hang).  Requires all G workgroups co-resident: G <= #CU and one
// 1024-thread workgroup per CU.
// ---------------------------------------------------------------------------------------
constexpr int PA_T = 1024;
constexpr int PA_NW = 16;
constexpr int PA_UC = 31;            // max lo-res columns owned per unit (a.uc: 31, or 15 when that fits the CUs)
constexpr int PA_NC = PA_UC + 1;     // storage stride of a unit's lo-res row (held columns: a.uc + 1)
constexpr int PA_NPX = 2 * PA_NC;    // lo-res pixels per unit: one per lane
constexpr int PA_CPW = 512 / PA_NW;  // channels per wave
constexpr int PA_R = 16;             // max replica rows of dW[1] (and arrival counters) per slot
constexpr int PA_R_DEFAULT = 8;      // rows used (CWT_ADAPT_PR: 2, 4, 8 or 16)
constexpr int PA_NSLOT = 4;          // accumulator slots (step s adds into s % 4)
constexpr int PA_EW = 4;             // episodes one workgroup's units may span
constexpr bool PA_HIRES2 = true;     // the lockstep pair's hi-res passes interleaved (hires_pass2)
#ifndef PA_CNT_STRIDE_WORDS
#define PA_CNT_STRIDE_WORDS 32
#endif
constexpr int PA_CNT_STRIDE = PA_CNT_STRIDE_WORDS;  // words between control words (32: one per 128-B line)
constexpr int PA_CNT_WORDS = (PA_R + 1) * PA_CNT_STRIDE;  // arrival counters + error word
constexpr long PA_SPIN_LIMIT = 4000000;
#ifndef PA_POLL_SLEEP
#define PA_POLL_SLEEP 1  // s_sleep units (64 clocks) between arrival polls
#endif
static_assert(PA_NSLOT * ADAPT_SLOT <= ADAPT_ESTRIDE && PA_R <= ADAPT_RMAX, "slots must fit an episode's accumulators");

struct PersistArgs {
  const float* f;          // [E][n][h][w][512] (read in place: no per-call copy)
  const uint8_t* lbl;      // [E][n][S][S]
  const AdaptScalars* sc;  // [E]
  const AdaptDevArgs* dargs;  // [E]: w_in / w_out
  float* acc;              // [E][PA_NSLOT][ADAPT_RMAX][512]; slots 0 and 1 zeroed by the setup kernel
  unsigned* cnt;           // [PA_CNT_WORDS], zeroed by the setup kernel
  int h, w, S, nshot, nep, iters;
  int ncb, ntile, units, G;
  int nrep;    // replica rows in use
  int uc;      // lo-res columns owned per unit (15 or 31)
  long spin_limit;   // polls per barrier before the grid gives up (PA_SPIN_LIMIT by default)
  unsigned* status;  // the context's mapped host status word (cwt_ctx_status), or null
  float* wq = nullptr;  // the fused tail: [G][2][512] per-workgroup copies of the adapted W
};

// Episode e's accumulator slot k of the persistent loop as 64-bit fixed-point replica rows
// [PA_R][512] (the same bytes as ADAPT_SLOT floats)
__device__ __forceinline__ unsigned long long* pa_fx_slot(const PersistArgs& a, int e, int k) {
  return (unsigned long long*)(a.acc + (long)e * ADAPT_ESTRIDE + (long)k * ADAPT_SLOT);
}
// rint(v * scale) as a two's-complement 64-bit integer (scale = 2^k: the product is exact in double)
__device__ __forceinline__ unsigned long long pa_fx(float v, double scale) {
  return (unsigned long long)(long long)__builtin_rint((double)v * scale);
}
static_assert(PA_R * 512 * 8 <= ADAPT_SLOT * 4, "a fixed-point slot must fit an accumulator slot");

struct PaUnit {
  int e, img, r, x0, ncol, x_end;
  bool extra_row;  // this unit's row pair is the last: it also owns hi-res row S-1
};

__device__ __forceinline__ PaUnit pa_unit(const PersistArgs& a, int u) {
  PaUnit q;
  const int per_ep = a.nshot * a.ntile;
  q.e = u / per_ep;
  const int rem = u - q.e * per_ep;
  const int shot = rem / a.ntile, tile = rem - shot * a.ntile;
  q.img = q.e * a.nshot + shot;
  q.r = tile / a.ncb;
  const int cb = tile - q.r * a.ncb;
  q.x0 = cb * a.uc;
  q.ncol = min(a.uc + 1, a.w - q.x0);
  q.x_end = (cb == a.ncb - 1) ? a.S : 8 * (q.x0 + a.uc);
  q.extra_row = q.r == a.h - 2;
  return q;
}

// Per-lane state of one unit: f of lane p's pixel over the wave's 32 channels, and the labels
// of the lane's hi-res pixels (2 column rounds x {row 8r + wv/2, row S-1}); 255 = no pixel.
struct PaTile {
  float fr[PA_CPW];
  int y[2][2];
};

__device__ __forceinline__ void pa_load(PaTile& t, const PersistArgs& a, const PaUnit& q, int wv, int lane) {
  const int ri = lane >> 5, xs = min(lane & 31, q.ncol - 1);
  const float* src = a.f + (((long)q.img * a.h + q.r + ri) * a.w + q.x0 + xs) * 512 + wv * PA_CPW;
#pragma unroll
  for (int j = 0; j < PA_CPW / 4; ++j) {
    const f32x4 v = *(const f32x4*)(src + 4 * j);
    t.fr[4 * j] = v[0]; t.fr[4 * j + 1] = v[1]; t.fr[4 * j + 2] = v[2]; t.fr[4 * j + 3] = v[3];
  }
  const uint8_t* lb = a.lbl + (long)q.img * a.S * a.S;
  const int Y = 8 * q.r + (wv >> 1);
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int X = 8 * q.x0 + 64 * (wv & 1) + 128 * k + lane;
    const int Xc = min(X, a.S - 1);
    const int ym = lb[(long)Y * a.S + Xc], ye = lb[(long)(a.S - 1) * a.S + Xc];
    const bool xin = X < q.x_end;
    t.y[k][0] = xin ? ym : 255;
    t.y[k][1] = (xin && q.extra_row && (wv >> 1) == 0) ? ye : 255;
  }
}

// NRES 3 (units streamed): wave wv moves its 32-channel slice of a unit's f (64 pixels x 128 B)
// into its private 8-KB LDS region by LDS-DMA, 8 pieces of 8 pixels; 16-B chunk c of pixel p is
// stored at slot c ^ ((p >> 1) & 7), so the per-pixel ds_read_b128 of pa_read_f are
// conflict-free.  Only the wave itself reads its region: the hand-off needs no barrier.
__device__ __forceinline__ void pa_issue_f(const PersistArgs& a, const PaUnit& q, int wv, int lane, float* fw) {
  const int pr = lane >> 3, sl = lane & 7;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int p = j * 8 + pr;
    const int c = sl ^ ((p >> 1) & 7);
    const int ri = p >> 5, xs = min(p & 31, q.ncol - 1);
    const float* src = a.f + (((long)q.img * a.h + q.r + ri) * a.w + q.x0 + xs) * 512 + wv * PA_CPW + c * 4;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)((char*)fw + j * 1024), 16, 0, 0);
  }
}
__device__ __forceinline__ void pa_read_f(float (&fr)[PA_CPW], const float* fw, int lane) {
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const f32x4 v = *(const f32x4*)(fw + lane * PA_CPW + ((c ^ ((lane >> 1) & 7)) << 2));
    fr[4 * c] = v[0]; fr[4 * c + 1] = v[1]; fr[4 * c + 2] = v[2]; fr[4 * c + 3] = v[3];
  }
}
__device__ __forceinline__ void pa_labels(int (&y)[2][2], const PersistArgs& a, const PaUnit& q, int wv, int lane) {
  const uint8_t* lb = a.lbl + (long)q.img * a.S * a.S;
  const int Y = 8 * q.r + (wv >> 1);
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int X = 8 * q.x0 + 64 * (wv & 1) + 128 * k + lane;
    const int Xc = min(X, a.S - 1);
    const int ym = lb[(long)Y * a.S + Xc], ye = lb[(long)(a.S - 1) * a.S + Xc];
    const bool xin = X < q.x_end;
    y[k][0] = xin ? ym : 255;
    y[k][1] = (xin && q.extra_row && (wv >> 1) == 0) ? ye : 255;
  }
}

__device__ __forceinline__ unsigned pack_y(const int (&y)[2][2]) {
  return (unsigned)y[0][0] | ((unsigned)y[0][1] << 8) | ((unsigned)y[1][0] << 16) | ((unsigned)y[1][1] << 24);
}

// 64-lane reduction of 32 per-lane values (channel j in v[j]) leaving lane L with channel L >> 1:
// five halving steps, each pairing lanes that differ in one lane bit (the lane with the bit set
// keeps the upper half of the channels, its partner the lower), then one plain pair sum.
//   bit 5, 4: v_permlane32_swap / v_permlane16_swap exchange whole halves / rows of two VGPRs,
//             so after the swap both partners just add (no select);
//   bit 3, 2: DPP row_mirror / row_half_mirror (partners 15-i / 7-i share the higher bits);
//   bit 1, 0: DPP quad_perm xor 2 / xor 1.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
// bits 4 .. 0 of the butterfly on the 16 values left after the permlane32 step
__device__ __forceinline__ void pa_butterfly16(float (&v)[PA_CPW], int lane) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[j]), __float_as_uint(v[j + 8]), false, false);
    v[j] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  {
    const bool up = (lane & 8) != 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float send = up ? v[j] : v[j + 4], keep = up ? v[j + 4] : v[j];
      v[j] = keep + dpp_mov<0x140>(send);
    }
  }
  {
    const bool up = (lane & 4) != 0;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const float send = up ? v[j] : v[j + 2], keep = up ? v[j + 2] : v[j];
      v[j] = keep + dpp_mov<0x141>(send);
    }
  }
  {
    const bool up = (lane & 2) != 0;
    const float send = up ? v[0] : v[1], keep = up ? v[1] : v[0];
    v[0] = keep + dpp_mov<0x4E>(send);
  }
  v[0] += dpp_mov<0xB1>(v[0]);
}
__device__ __forceinline__ void pa_butterfly(float (&v)[PA_CPW], int lane) {
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[j]), __float_as_uint(v[j + 16]), false, false);
    v[j] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  pa_butterfly16(v, lane);
}
// The same reduction of 32 values produced on the fly (fv(j): channel j's value): channels j and
// j + 16 are formed together and enter the permlane32 step at once, so at most 16 of them are
// live (the three-unit form keeps two units' f in registers beside them)
template <class FV>
__device__ __forceinline__ float pa_butterfly_fn(FV fv, int lane) {
  float v[PA_CPW];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(fv(j)), __float_as_uint(fv(j + 16)), false, false);
    v[j] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    if (j & 1) asm volatile("" ::: "memory");  // bounds the LDS reads fv may issue ahead (registers)
  }
  pa_butterfly16(v, lane);
  return v[0];
}

// Per-unit LDS scratch of the lockstep forms: the z partials, and the hi-res pass's per-octet
// adjoint slots.  Three units (NRES 4) alias them: the z partials are dead (summed into zd)
// two barriers before the slots are written, and the slots are read before the next step's z.
template <int NU>
struct PaScrSep {
  float zpart[NU][PA_NW][PA_NPX];
  float P0[NU][8][2][PA_NC + 1];
  float P1[NU][8][2][PA_NC + 1];
};
template <int NU>
struct PaScrAlias {
  union {
    float zpart[NU][PA_NW][PA_NPX];
    struct {
      float P0[NU][8][2][PA_NC + 1];
      float P1[NU][8][2][PA_NC + 1];
    };
  };
};

// STAMPS (CWT_ADAPT_DBG & 32, a separate instantiation; never the timed one): thread 0 records
// s_memtime at 8 points of every step, realtime at its arrival ([8]) and when its poll matched
// ([9]) into stamps[step][g][10], and realtime/memtime at entry and exit into
// stamps[iters][g][0..3] (tools/persist_stamps.py).
// NRES 1: one unit per workgroup, its f in registers; 2: up to two units per workgroup, the
// first in registers, the second in LDS (128 KB, lane-major: conflict-free); 4: up to three
// units in lockstep, the first and third in registers, the second in LDS; 3: units streamed
// every step, each wave's slice by LDS-DMA into its private 8 KB while the previous unit is
// computed; 0: units streamed from L2 into registers (opt-in, slower).  Fewer workgroups make each step's barrier cheaper and leave CUs to the
// next episode's extractor pass (EpisodePipeline).
// MODE only separates instantiations so that rocprofv3's per-kernel statistics attribute each
// launch to the leg that made it: 0 the product kernel (every timed launch); 1 STAMPS (above);
// 2 FLOOR, the latency-floor study (CWT_ADAPT_DBG & 64: every unit's arithmetic and atomics
// skipped, what is left is the per-step exchange); 3 SIDE, code identical to 0, launched for
// bench.py's side legs (CWT_ADAPT_DBG & 128: the loop timed alone, the exact-fp32 leg) so that
// they do not mix into the timed kernel's rocprof average.
// The kernel's body: false when the grid gave up (barrier spin bound or another workgroup's abort).
template <int NRES, int MODE>
__device__ __forceinline__ bool adapt_persist_body(const PersistArgs& a, unsigned long long* stamps) {
  constexpr bool STAMPS = MODE == 1;
  constexpr bool FLOOR = MODE == 2;
  constexpr int C = 512;
  constexpr int EWK = (NRES >= 2) ? 2 : NRES == 1 ? 1 : PA_EW;  // episodes a workgroup's units may span
  constexpr bool LOCK = NRES == 2 || NRES == 4;  // units in lockstep, the second one's f in fl2
  // NRES 5: two units in lockstep, both in registers (the second one in cur2, as NRES 4's third):
  // no LDS reads of f in the z and dW passes
  constexpr bool BREG = NRES == 5;
  // NRES 6: NRES 3 with the workgroup's first unit resident in registers (res): its f is never
  // streamed, the DMA ring carries only the units after it (5-shot 641^2: 4-5 units per workgroup,
  // about a fifth of the per-step stream)
  constexpr bool STREAM = NRES == 3 || NRES == 6;
  constexpr bool RES1 = NRES == 6;
  __shared__ float fl2[LOCK ? PA_NW : 1][PA_CPW][LOCK ? 64 : 1];
  __shared__ __attribute__((aligned(16))) float fs3[(NRES == 3 || NRES == 6) ? PA_NW * 64 * PA_CPW : 4];  // NRES 3, 6: per-wave f slices
  __shared__ float dlw[PA_NW][EWK][PA_CPW];     // d = W1 - W0 of each wave's channels (wave-private)
  __shared__ float wlw[PA_NW][EWK][2][PA_CPW];  // W0, W1 of each wave's channels (wave-private)
  // NRES 2 runs its two units in lockstep (one set of LDS barriers, one butterfly and one set
  // of atomics per step when both units belong to one episode): the second unit's copies [1]
  constexpr int NU = (NRES == 2 || NRES == 5) ? 2 : NRES == 4 ? 3 : 1;
  __shared__ std::conditional_t<NRES == 4, PaScrAlias<NU>, PaScrSep<NU>> scr;
  auto& zpart_u = scr.zpart;
  auto& P0_u = scr.P0;
  auto& P1_u = scr.P1;
  __shared__ float zd_u[NU][PA_NPX];
  __shared__ float gs_u[NU][PA_NPX];
  auto& zpart = zpart_u[0];
  auto& zd = zd_u[0];
  auto& gs = gs_u[0];
  auto& P0 = P0_u[0];
  auto& P1 = P1_u[0];
  __shared__ float wfg_l[EWK], lr_l[EWK];
  __shared__ double fxs_l[EWK], fxi_l[EWK];  // the episodes' fixed-point scales (AdaptScalars)
  __shared__ int abort_flag;
  const int t = threadIdx.x, lane = t & 63, wv = __builtin_amdgcn_readfirstlane(t >> 6);  // wv: SGPR
  const int g = blockIdx.x, G = a.G;
  const int u0 = (int)(((long)g * a.units) / G), u1 = (int)(((long)(g + 1) * a.units) / G);
  const int per_ep = a.nshot * a.ntile;
  const int e_lo = u0 / per_ep, e_hi = (u1 - 1) / per_ep;
  const int new_ = e_hi - e_lo + 1;  // episodes spanned (<= PA_EW, checked on the host)
  const int nrep = a.nrep;
  const int rep = g % nrep;
  unsigned* err = a.cnt + PA_R * PA_CNT_STRIDE;
  unsigned long long* stp_end = (STAMPS && t == 0) ? stamps + ((long)a.iters * G + g) * 10 : nullptr;
  if (STAMPS && t == 0) {
    stp_end[0] = __builtin_amdgcn_s_memrealtime();
    stp_end[1] = __builtin_amdgcn_s_memtime();
  }

  // W of the spanned episodes is split over the waves: wave wv keeps channels [32wv, 32wv+32)
  // in a private LDS slice (lane L < 32: channel 32wv + L) and only ever touches its own slice,
  // so W needs no workgroup barrier; every workgroup applies the same updates in the same
  // order, so the copies stay identical
  const int cw = wv * PA_CPW + (lane & 31);
#pragma unroll
  for (int ew = 0; ew < EWK; ++ew) {
    const float* wi = a.dargs[min(e_lo + ew, a.nep - 1)].w_in;
    const float w0 = wi[cw], w1 = wi[C + cw];
    if (lane < 32) {
      wlw[wv][ew][0][lane] = w0;
      wlw[wv][ew][1][lane] = w1;
      dlw[wv][ew][lane] = w1 - w0;
    }
  }
  if (t == 0) abort_flag = 0;
  if (t < new_) {
    wfg_l[t] = a.sc[e_lo + t].wfg;
    lr_l[t] = a.sc[e_lo + t].lr_eff;
    fxs_l[t] = a.sc[e_lo + t].fx_scale;
    fxi_l[t] = a.sc[e_lo + t].fx_inv;
  }
  PaTile cur;
  PaUnit q = pa_unit(a, u0);
  float* fw = fs3 + (STREAM ? wv * 64 * PA_CPW : 0);
  int ynx[2][2] = {{255, 255}, {255, 255}};  // NRES 3, 6: labels of the unit whose f is in flight
  PaTile res;  // NRES 6: the resident first unit
  if (RES1) {
    pa_load(res, a, q, wv, lane);
    if (u1 - u0 > 1) {
      const PaUnit qn = pa_unit(a, u0 + 1);
      pa_issue_f(a, qn, wv, lane, fw);
      pa_labels(ynx, a, qn, wv, lane);
    }
  } else if (STREAM) {
    pa_issue_f(a, q, wv, lane, fw);
    pa_labels(ynx, a, q, wv, lane);
  } else {
    pa_load(cur, a, q, wv, lane);
  }
  int y2[2][2] = {{255, 255}, {255, 255}};  // NRES 2 / 4: labels of the second unit (its f is in fl2)
  if (LOCK && u1 - u0 == 1) {  // no second unit: its f reads as zero in the lockstep dW pass
#pragma unroll
    for (int j = 0; j < PA_CPW; ++j) fl2[wv][j][lane] = 0.f;
  }
  PaTile cur2;  // NRES 4: the third unit (registers); NRES 5: the second; zero when the workgroup has fewer
  if (BREG) {
    if (u1 - u0 > 1) {
      pa_load(cur2, a, pa_unit(a, u0 + 1), wv, lane);
    } else {
#pragma unroll
      for (int j = 0; j < PA_CPW; ++j) cur2.fr[j] = 0.f;
#pragma unroll
      for (int k = 0; k < 2; ++k) cur2.y[k][0] = cur2.y[k][1] = 255;
    }
  }
  if (NRES == 4) {
    if (u1 - u0 > 2) {
      pa_load(cur2, a, pa_unit(a, u0 + 2), wv, lane);
    } else {
#pragma unroll
      for (int j = 0; j < PA_CPW; ++j) cur2.fr[j] = 0.f;
#pragma unroll
      for (int k = 0; k < 2; ++k) cur2.y[k][0] = cur2.y[k][1] = 255;
    }
  }
  if (LOCK && u1 - u0 > 1) {
    PaTile tmp;
    pa_load(tmp, a, pa_unit(a, u0 + 1), wv, lane);
#pragma unroll
    for (int j = 0; j < PA_CPW; ++j) fl2[wv][j][lane] = tmp.fr[j];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      y2[k][0] = tmp.y[k][0];
      y2[k][1] = tmp.y[k][1];
    }
  }
  // NRES 4: the three units' labels one byte each (unit A's f stays in cur.fr)
  const unsigned yap = pack_y(cur.y), ycp = pack_y(cur2.y);
  const unsigned y2p = BREG ? ycp : pack_y(y2);
  __syncthreads();

  const int i_row = wv >> 1;
  const float ly1 = (float)i_row * 0.125f, ly0 = 1.f - ly1;
  for (int s = 0; s < a.iters; ++s) {
    // an opaque copy of the thread id per step: lane-dependent addresses and label decodes are
    // recomputed (a few VALU ops) instead of being hoisted out of the 200-step loop, where they
    // would hold registers the lockstep forms need for f (or be spilled to scratch)
    int t_op = (int)threadIdx.x;
    if constexpr (NRES >= 2) asm volatile("" : "+v"(t_op));  // (NRES 1 has the registers: hoisting wins)
    const int t = t_op, lane = t_op & 63;
    const int cw = wv * PA_CPW + (lane & 31);
    const int slot = s % PA_NSLOT;
    unsigned long long* stp = (STAMPS && t == 0) ? stamps + ((long)s * G + g) * 10 : nullptr;
    auto stamp = [&](int i) {
      if (STAMPS && stp) stp[i] = __builtin_amdgcn_s_memtime();
    };
    stamp(0);
    // zero this workgroup's share of slot (s+2)%4 (write-through stores, done by our arrival);
    // NRES 3 does it after its units, so that its per-unit DMA waits do not wait for the stores
    auto zero_share = [&]() {
      if (s + 2 < a.iters) {
        const int zs = (s + 2) % PA_NSLOT;
        const int tot = a.nep * nrep * C, per = (tot + G - 1) / G;
        for (int i = g * per + t; i < min(tot, (g + 1) * per); i += PA_T) {
          const int e = i / (nrep * C), k = i - e * (nrep * C);
          __hip_atomic_store(pa_fx_slot(a, e, zs) + k, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    };
    if (!STREAM) zero_share();
    // NRES 3: each unit's dW is reduced over the wave by the butterfly as usual, and the one
    // value a lane then holds (channel lane >> 1) is summed over the step's units of one episode
    // in a register; one atomic per episode and step (none in flight at the next unit's DMA wait)
    // dW[1] partial v of channel 32 wv + (lane >> 1) of episode e into replica row rep of the step's
    // slot: one no-return 64-bit fixed-point atomic (integer adds: exact and order-free, so every
    // workgroup reads the same sums whatever the arrival order -- a deterministic loop)
    auto add_dw = [&](int e, float v) {
      __hip_atomic_fetch_add(pa_fx_slot(a, e, slot) + rep * C + wv * PA_CPW + (lane >> 1), pa_fx(v, fxs_l[e - e_lo]),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    float dsum3 = 0.f;
    int dsum3_e = e_lo;
    auto flush3 = [&]() {
      if ((lane & 1) == 0) add_dw(dsum3_e, dsum3);
      dsum3 = 0.f;
    };
    // one unit's z / hi-res / dW passes; fget(j): f of lane p's pixel, channel 32*wv + j
    auto unit_body = [&](const PaUnit& q, int u, auto fget, const int (&ylab)[2][2]) {
      const int ew = q.e - e_lo;
      // ---- z = d . f: this wave's 32-channel partial for lane p's pixel; d = W1 - W0 of the
      // wave's channels from its private LDS slice (LDS broadcast; written by this wave only,
      // so no workgroup barrier) ----
      {
        float sdot = 0.f;
#pragma unroll
        for (int j = 0; j < PA_CPW / 4; ++j) {
          const f32x4 d4 = *(const f32x4*)&dlw[wv][ew][4 * j];
          sdot = fmaf(d4[0], fget(4 * j), sdot);
          sdot = fmaf(d4[1], fget(4 * j + 1), sdot);
          sdot = fmaf(d4[2], fget(4 * j + 2), sdot);
          sdot = fmaf(d4[3], fget(4 * j + 3), sdot);
        }
        zpart[wv][lane] = sdot;
      }
      lds_barrier();
      if (t < PA_NPX) {
        float z = 0.f;
#pragma unroll
        for (int v = 0; v < PA_NW; ++v) z += zpart[v][t];
        zd[t] = z;
      }
      lds_barrier();
      if (u == u0) stamp(1);
      // ---- hi-res pass: weighted-CE gradient, bilinear adjoint pre-reduced per octet ----
      {
        const bool has_extra = q.extra_row && i_row == 0;
        const float wf = wfg_l[ew];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          if (k == 1 && a.uc < 16) break;  // 8 * 15 columns (+ the last block's tail) fit one round
          const int X = 8 * q.x0 + 64 * (wv & 1) + 128 * k + lane;
          const int slot_x = 8 * (wv & 1) + 16 * k + (lane >> 3);  // = (X >> 3) - x0 before clamping
          const int ix = min(X >> 3, a.w - 1);
          const int xi0 = min(ix - q.x0, PA_NC - 1);
          const int xi1 = (ix < a.w - 1) ? min(xi0 + 1, PA_NC - 1) : xi0;
          const float lx1 = (float)(X & 7) * 0.125f, lx0 = 1.f - lx1;
          float sa[2] = {0.f, 0.f}, sb[2] = {0.f, 0.f};
#pragma unroll
          for (int e2 = 0; e2 < 2; ++e2) {
            if (e2 == 1 && !has_extra) break;  // wave-uniform: only the last row pair's row-0 waves
            const int y = ylab[k][e2];
            float gv = 0.f;
            if (y != 255) {
              const float dd = e2 ? (lx0 * zd[PA_NC + xi0] + lx1 * zd[PA_NC + xi1])
                                  : ly0 * (lx0 * zd[xi0] + lx1 * zd[xi1]) +
                                        ly1 * (lx0 * zd[PA_NC + xi0] + lx1 * zd[PA_NC + xi1]);
              const float p1 = __builtin_amdgcn_rcpf(1.f + __expf(-dd));
              gv = ((y == 1) ? wf : 1.f) * (p1 - (float)y);
            }
            sa[e2] = octet_sum(lx0 * gv);
            sb[e2] = octet_sum(lx1 * gv);
          }
          if ((lane & 7) == 0) {
            P0[i_row][0][slot_x] = ly0 * sa[0];
            P1[i_row][0][slot_x + 1] = ly0 * sb[0];
            P0[i_row][1][slot_x] = ly1 * sa[0] + sa[1];
            P1[i_row][1][slot_x + 1] = ly1 * sb[0] + sb[1];
          }
        }
      }
      lds_barrier();
      if (t < PA_NPX) {
        const int ri = t >> 5, xi = t & 31;
        float gsum = 0.f;
        if (xi <= a.uc) {  // held columns only (the rest were not written this unit)
#pragma unroll
          for (int i = 0; i < 8; ++i) gsum += P0[i][ri][xi];
          if (xi > 0) {
#pragma unroll
            for (int i = 0; i < 8; ++i) gsum += P1[i][ri][xi];
          }
        }
        gs[t] = gsum;
      }
      lds_barrier();
      if (u == u0) stamp(2);
      // ---- dW[1] of the unit: lane p's pixel times its gradient, over the wave's channels ----
      {
        float accd[PA_CPW];
        const float gp = gs[lane];
        if constexpr (RES1) {  // the products formed on the fly (at most 16 live beside res and cur)
          accd[0] = pa_butterfly_fn([&](int j) { return gp * fget(j); }, lane);
        } else {
#pragma unroll
          for (int j = 0; j < PA_CPW; ++j) accd[j] = gp * fget(j);
          pa_butterfly(accd, lane);  // lane L: channel (L >> 1) of the wave's slice, summed over 64 lanes
        }
        if (STREAM) {  // summed over the step's units of the episode, flushed on a change of episode
          if (q.e != dsum3_e) {
            flush3();
            dsum3_e = q.e;
          }
          dsum3 += accd[0];
        } else if ((lane & 1) == 0) {
          add_dw(q.e, accd[0]);
        }
      }
    };
    // NRES 2 with two units: both units' phases share the barriers; lane p holds pixel p of
    // each unit (unit A's f in registers, unit B's in fl2), LDS copies [0] / [1]
    // ylab: the lane's four labels packed one per byte (k * 2 + e2).  The lane-dependent geometry
    // is derived from an opaque copy of the lane id, so it is recomputed every step instead of
    // being hoisted out of the 200-step loop into registers the lockstep forms do not have
    auto hires_pass = [&](const PaUnit& q, int ew, unsigned ylab, const float* zdp, float (*P0p)[2][PA_NC + 1],
                          float (*P1p)[2][PA_NC + 1]) {
      const bool has_extra = q.extra_row && i_row == 0;
      const float wf = wfg_l[ew];
      int ln = lane;
      asm volatile("" : "+v"(ln), "+v"(ylab));
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        if (k == 1 && a.uc < 16) break;
        const int X = 8 * q.x0 + 64 * (wv & 1) + 128 * k + ln;
        const int slot_x = 8 * (wv & 1) + 16 * k + (ln >> 3);
        const int ix = min(X >> 3, a.w - 1);
        const int xi0 = min(ix - q.x0, PA_NC - 1);
        const int xi1 = (ix < a.w - 1) ? min(xi0 + 1, PA_NC - 1) : xi0;
        const float lx1 = (float)(X & 7) * 0.125f, lx0 = 1.f - lx1;
        float sa[2] = {0.f, 0.f}, sb[2] = {0.f, 0.f};
#pragma unroll
        for (int e2 = 0; e2 < 2; ++e2) {
          if (e2 == 1 && !has_extra) break;
          const int y = (int)((ylab >> (8 * (2 * k + e2))) & 255u);
          float gv = 0.f;
          if (y != 255) {
            const float dd = e2 ? (lx0 * zdp[PA_NC + xi0] + lx1 * zdp[PA_NC + xi1])
                                : ly0 * (lx0 * zdp[xi0] + lx1 * zdp[xi1]) + ly1 * (lx0 * zdp[PA_NC + xi0] + lx1 * zdp[PA_NC + xi1]);
            const float p1 = __builtin_amdgcn_rcpf(1.f + __expf(-dd));
            gv = ((y == 1) ? wf : 1.f) * (p1 - (float)y);
          }
          sa[e2] = octet_sum(lx0 * gv);
          sb[e2] = octet_sum(lx1 * gv);
        }
        if ((lane & 7) == 0) {
          P0p[i_row][0][slot_x] = ly0 * sa[0];
          P1p[i_row][0][slot_x + 1] = ly0 * sb[0];
          P0p[i_row][1][slot_x] = ly1 * sa[0] + sa[1];
          P1p[i_row][1][slot_x + 1] = ly1 * sb[0] + sb[1];
        }
      }
    };
    // The lockstep pair's two hi-res passes in ONE loop body (round 5): the per-pixel chain (bilinear
    // z from LDS -> exp / rcp -> two DPP octet sums -> LDS) is latency-bound, and two independent
    // units' chains interleave where two consecutive passes ran back to back (stamps, profiles/r5:
    // 1.94 us for the pair against 0.95 for one unit).  The rare extra-row terms (the last row
    // pair's row S - 1, e2 = 1) run for both units when either has them; a unit without them has
    // labels 255 there, i.e. a zero gradient, as in the single pass.
    auto hires_pass2 = [&](const PaUnit& qa, int ewa, unsigned ya, const float* zda, float (*P0a)[2][PA_NC + 1],
                           float (*P1a)[2][PA_NC + 1], const PaUnit& qb, int ewb, unsigned yb, const float* zdb,
                           float (*P0b)[2][PA_NC + 1], float (*P1b)[2][PA_NC + 1]) {
      const bool extra = (qa.extra_row || qb.extra_row) && i_row == 0;
      const float wf[2] = {wfg_l[ewa], wfg_l[ewb]};
      int ln = lane;
      asm volatile("" : "+v"(ln), "+v"(ya), "+v"(yb));
      const unsigned yl[2] = {ya, yb};
      const float* zdp[2] = {zda, zdb};
      float (*P0p[2])[2][PA_NC + 1] = {P0a, P0b};
      float (*P1p[2])[2][PA_NC + 1] = {P1a, P1b};
      const int x0[2] = {qa.x0, qb.x0};
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        if (k == 1 && a.uc < 16) break;
        int slot_x[2], xi0[2], xi1[2];
        float lx0[2], lx1[2], sa[2][2], sb[2][2];
#pragma unroll
        for (int uu = 0; uu < 2; ++uu) {
          const int X = 8 * x0[uu] + 64 * (wv & 1) + 128 * k + ln;
          slot_x[uu] = 8 * (wv & 1) + 16 * k + (ln >> 3);
          const int ix = min(X >> 3, a.w - 1);
          xi0[uu] = min(ix - x0[uu], PA_NC - 1);
          xi1[uu] = (ix < a.w - 1) ? min(xi0[uu] + 1, PA_NC - 1) : xi0[uu];
          lx1[uu] = (float)(X & 7) * 0.125f;
          lx0[uu] = 1.f - lx1[uu];
          sa[uu][1] = sb[uu][1] = 0.f;
        }
#pragma unroll
        for (int e2 = 0; e2 < 2; ++e2) {
          if (e2 == 1 && !extra) break;
#pragma unroll
          for (int uu = 0; uu < 2; ++uu) {
            const float* zd_ = zdp[uu];
            const int y = (int)((yl[uu] >> (8 * (2 * k + e2))) & 255u);
            float gv = 0.f;
            if (y != 255) {
              const float dd = e2 ? (lx0[uu] * zd_[PA_NC + xi0[uu]] + lx1[uu] * zd_[PA_NC + xi1[uu]])
                                  : ly0 * (lx0[uu] * zd_[xi0[uu]] + lx1[uu] * zd_[xi1[uu]]) +
                                        ly1 * (lx0[uu] * zd_[PA_NC + xi0[uu]] + lx1[uu] * zd_[PA_NC + xi1[uu]]);
              const float p1 = __builtin_amdgcn_rcpf(1.f + __expf(-dd));
              gv = ((y == 1) ? wf[uu] : 1.f) * (p1 - (float)y);
            }
            sa[uu][e2] = octet_sum(lx0[uu] * gv);
            sb[uu][e2] = octet_sum(lx1[uu] * gv);
          }
        }
        if ((lane & 7) == 0) {
#pragma unroll
          for (int uu = 0; uu < 2; ++uu) {
            P0p[uu][i_row][0][slot_x[uu]] = ly0 * sa[uu][0];
            P1p[uu][i_row][0][slot_x[uu] + 1] = ly0 * sb[uu][0];
            P0p[uu][i_row][1][slot_x[uu]] = ly1 * sa[uu][0] + sa[uu][1];
            P1p[uu][i_row][1][slot_x[uu] + 1] = ly1 * sb[uu][0] + sb[uu][1];
          }
        }
      }
    };
    auto gs_of = [&](int tt, float (*P0p)[2][PA_NC + 1], float (*P1p)[2][PA_NC + 1]) {
      const int ri = tt >> 5, xi = tt & 31;
      float gsum = 0.f;
      if (xi <= a.uc) {
#pragma unroll
        for (int i = 0; i < 8; ++i) gsum += P0p[i][ri][xi];
        if (xi > 0) {
#pragma unroll
          for (int i = 0; i < 8; ++i) gsum += P1p[i][ri][xi];
        }
      }
      return gsum;
    };
    auto pair_body = [&](const PaUnit& qa, const PaUnit& qb, bool has_b) {  // !has_b: unit B absent (fl2 zero)
      const int ewa = qa.e - e_lo, ewb = qb.e - e_lo;
      {
        float sda = 0.f, sdb = 0.f;
#pragma unroll
        for (int j = 0; j < PA_CPW / 4; ++j) {
          const f32x4 da = *(const f32x4*)&dlw[wv][ewa][4 * j];
          const f32x4 db = *(const f32x4*)&dlw[wv][ewb][4 * j];
          float fb[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) fb[r] = BREG ? cur2.fr[4 * j + r] : fl2[wv][4 * j + r][lane];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            sda = fmaf(da[r], cur.fr[4 * j + r], sda);
            sdb = fmaf(db[r], fb[r], sdb);
          }
          if (!BREG && (j & 1)) asm volatile("" ::: "memory");  // at most 8 of unit B's LDS reads in flight (registers)
        }
        zpart_u[0][wv][lane] = sda;
        zpart_u[NU - 1][wv][lane] = sdb;
      }
      lds_barrier();
      if (t < 2 * PA_NPX) {
        const int uu = t >> 6, tt = t & 63;
        float z = 0.f;
#pragma unroll
        for (int v = 0; v < PA_NW; ++v) z += zpart_u[uu][v][tt];
        zd_u[uu][tt] = z;
      }
      lds_barrier();
      stamp(1);
      if (PA_HIRES2) {  // both units' passes interleaved (unit B absent: labels 255, zero gradient)
        hires_pass2(qa, ewa, pack_y(cur.y), zd_u[0], P0_u[0], P1_u[0], qb, ewb, has_b ? y2p : 0xFFFFFFFFu,
                    zd_u[NU - 1], P0_u[NU - 1], P1_u[NU - 1]);
      } else {
        hires_pass(qa, ewa, pack_y(cur.y), zd_u[0], P0_u[0], P1_u[0]);
        if (has_b) hires_pass(qb, ewb, y2p, zd_u[NU - 1], P0_u[NU - 1], P1_u[NU - 1]);
      }
      lds_barrier();
      if (t < 2 * PA_NPX) {
        const int uu = t >> 6, tt = t & 63;
        gs_u[uu][tt] = gs_of(tt, P0_u[uu], P1_u[uu]);
      }
      lds_barrier();
      stamp(2);
      if constexpr (BREG) {
        // both units in registers: each episode's dW formed on the fly inside the butterfly
        // (channels j and j + 16 together, at most 16 values live beside the two units' f)
        const float ga = gs_u[0][lane], gb = has_b ? gs_u[NU - 1][lane] : 0.f;
#pragma unroll
        for (int pass = 0; pass < 2; ++pass) {
          const int e = pass ? qb.e : qa.e;
          if (pass && qb.e == qa.e) break;
          const float ma = qa.e == e ? ga : 0.f, mb = qb.e == e ? gb : 0.f;
          const float dsum = pa_butterfly_fn([&](int j) { return fmaf(mb, cur2.fr[j], ma * cur.fr[j]); }, lane);
          if ((lane & 1) == 0) add_dw(e, dsum);
        }
      } else {
        float accd[PA_CPW];
        const float ga = gs_u[0][lane], gb = has_b ? gs_u[NU - 1][lane] : 0.f;
        if (qa.e == qb.e) {  // one butterfly and one set of atomics for both units
#pragma unroll
          for (int j = 0; j < PA_CPW; ++j) accd[j] = ga * cur.fr[j];
#pragma unroll
          for (int j0 = 0; j0 < PA_CPW; j0 += 8) {
            float fb[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) fb[k] = BREG ? cur2.fr[j0 + k] : fl2[wv][j0 + k][lane];
#pragma unroll
            for (int k = 0; k < 8; ++k) accd[j0 + k] = fmaf(gb, fb[k], accd[j0 + k]);
            if (!BREG) asm volatile("" ::: "memory");
          }
          pa_butterfly(accd, lane);
          if ((lane & 1) == 0) add_dw(qa.e, accd[0]);
        } else {
#pragma unroll
          for (int uu = 0; uu < 2; ++uu) {
            const PaUnit& q = uu ? qb : qa;
#pragma unroll
            for (int j = 0; j < PA_CPW; ++j) accd[j] = uu ? gb * (BREG ? cur2.fr[j] : fl2[wv][j][lane]) : ga * cur.fr[j];
            pa_butterfly(accd, lane);
            if ((lane & 1) == 0) add_dw(q.e, accd[0]);
          }
        }
      }
    };
    // NRES 4: three units in lockstep (A = u0 and C = u0 + 2 in registers, B = u0 + 1 in fl2),
    // one set of LDS barriers; units of one episode share one butterfly and one set of atomics
    auto triple_body = [&](int nb) {
      const PaUnit qa = pa_unit(a, u0);
      const PaUnit qb = pa_unit(a, nb > 1 ? u0 + 1 : u0);
      const PaUnit qc = pa_unit(a, nb > 2 ? u0 + 2 : u0);
      const int ewa = qa.e - e_lo, ewb = qb.e - e_lo, ewc = qc.e - e_lo;
      {
        float sda = 0.f, sdb = 0.f, sdc = 0.f;
#pragma unroll
        for (int j = 0; j < PA_CPW / 4; ++j) {
          const f32x4 da = *(const f32x4*)&dlw[wv][ewa][4 * j];
          const f32x4 db = *(const f32x4*)&dlw[wv][ewb][4 * j];
          const f32x4 dc = *(const f32x4*)&dlw[wv][ewc][4 * j];
          float fb[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) fb[r] = fl2[wv][4 * j + r][lane];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            sda = fmaf(da[r], cur.fr[4 * j + r], sda);
            sdb = fmaf(db[r], fb[r], sdb);
            sdc = fmaf(dc[r], cur2.fr[4 * j + r], sdc);
          }
          if (j & 1) asm volatile("" ::: "memory");
        }
        zpart_u[0][wv][lane] = sda;
        zpart_u[1][wv][lane] = sdb;
        zpart_u[NU - 1][wv][lane] = sdc;
      }
      lds_barrier();
      if (t < NU * PA_NPX) {
        const int uu = t >> 6, tt = t & 63;
        float z = 0.f;
#pragma unroll
        for (int v = 0; v < PA_NW; ++v) z += zpart_u[uu][v][tt];
        zd_u[uu][tt] = z;
      }
      lds_barrier();
      stamp(1);
      hires_pass(qa, ewa, yap, zd_u[0], P0_u[0], P1_u[0]);
      if (nb > 1) hires_pass(qb, ewb, y2p, zd_u[1], P0_u[1], P1_u[1]);
      if (nb > 2) hires_pass(qc, ewc, ycp, zd_u[NU - 1], P0_u[NU - 1], P1_u[NU - 1]);
      lds_barrier();
      if (t < NU * PA_NPX) {
        const int uu = t >> 6, tt = t & 63;
        gs_u[uu][tt] = gs_of(tt, P0_u[uu], P1_u[uu]);
      }
      lds_barrier();
      stamp(2);
      const float ga = gs_u[0][lane], gb = nb > 1 ? gs_u[1][lane] : 0.f, gc = nb > 2 ? gs_u[NU - 1][lane] : 0.f;
      // consecutive units: qa.e <= qb.e <= qc.e, at most two episodes (span <= 2, host-checked)
#pragma unroll
      for (int pass = 0; pass < 2; ++pass) {
        const int e = pass ? qc.e : qa.e;
        if (pass && qc.e == qa.e) break;
        const float ma = qa.e == e ? ga : 0.f, mb = qb.e == e ? gb : 0.f, mc = qc.e == e ? gc : 0.f;
        const float dsum = pa_butterfly_fn(
            [&](int j) { return fmaf(mc, cur2.fr[j], fmaf(mb, fl2[wv][j][lane], ma * cur.fr[j])); }, lane);
        if ((lane & 1) == 0) add_dw(e, dsum);
      }
    };
    if constexpr (FLOOR) {
      // timing study: no unit work (NRES 3 still drains its in-flight DMA)
      if (STREAM) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if constexpr (NRES == 4) {
      triple_body(u1 - u0);
    } else if constexpr (NRES == 2 || NRES == 5) {
      const bool has_b = u1 - u0 == 2;
      pair_body(q, has_b ? pa_unit(a, u0 + 1) : q, has_b);
    } else
    for (int u = u0; u < u1; ++u) {
      if (RES1 && u == u0) {  // the resident unit, computed while the next unit's DMA is in flight
        unit_body(pa_unit(a, u0), u0, [&](int jj) { return res.fr[jj]; }, res.y);
        continue;
      }
      if (STREAM) {  // this wave's slice of unit u landed (nothing younger is in flight), then
                     // the next unit's DMA goes out while unit u is computed
        const PaUnit qu = pa_unit(a, u);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        pa_read_f(cur.fr, fw, lane);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          cur.y[k][0] = ynx[k][0];
          cur.y[k][1] = ynx[k][1];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slice is read: it may be refilled
        if (u + 1 < u1) {  // (the next step's first unit goes out after this step's arrival)
          const PaUnit qn = pa_unit(a, u + 1);
          pa_issue_f(a, qn, wv, lane, fw);
          pa_labels(ynx, a, qn, wv, lane);
        }
        unit_body(qu, u, [&](int jj) { return cur.fr[jj]; }, cur.y);
        continue;
      }
      if (NRES == 2 && u != u0) {
        unit_body(pa_unit(a, u), u, [&](int jj) { return fl2[wv][jj][lane]; }, y2);
        continue;
      }
      if (NRES == 0 && u != u0) {  // streamed: this unit's f and labels (the first one was prefetched)
        q = pa_unit(a, u);
        pa_load(cur, a, q, wv, lane);
      } else if (NRES == 0) {
        q = pa_unit(a, u);
      }
      unit_body(q, u, [&](int jj) { return cur.fr[jj]; }, cur.y);
    }
    if (STREAM) {
      flush3();
      zero_share();
    }
    stamp(3);
    // ---- grid barrier s ----
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's atomics (and zero stores) performed
    __syncthreads();
    stamp(4);
    if (STAMPS && stp) stp[8] = __builtin_amdgcn_s_memrealtime();
    if (t == 0) __hip_atomic_fetch_add(a.cnt + rep * PA_CNT_STRIDE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (STREAM && s + 1 < a.iters && u0 + (RES1 ? 1 : 0) < u1) {  // next step's first streamed unit:
      const PaUnit qn = pa_unit(a, u0 + (RES1 ? 1 : 0));               // W-independent, lands during the wait
      pa_issue_f(a, qn, wv, lane, fw);
      pa_labels(ynx, a, qn, wv, lane);
    }
    if (NRES == 0 && s + 1 < a.iters) {  // next step's first unit: W-independent, lands during the wait
      q = pa_unit(a, u0);
      pa_load(cur, a, q, wv, lane);
    }
    if (wv == 0) {
      // one sc1 poll of the arrival counters at a time (two in flight measured slower: the extra
      // polls delay the arrivals' atomics at the memory side), summed by DPP
      const unsigned target = (unsigned)G * (unsigned)(s + 1);
      const unsigned* cp = a.cnt + (lane < nrep ? lane : 0) * PA_CNT_STRIDE;
      long spins = 0;
      while (true) {
        unsigned c = __hip_atomic_load(cp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        c = lane < nrep ? c : 0u;  // sum over lanes 0..15 (nrep <= 16) by DPP row shifts, read from lane 15
        c += __builtin_amdgcn_update_dpp(0u, c, 0x111, 0xF, 0xF, true);  // row_shr:1
        c += __builtin_amdgcn_update_dpp(0u, c, 0x112, 0xF, 0xF, true);  // row_shr:2
        c += __builtin_amdgcn_update_dpp(0u, c, 0x114, 0xF, 0xF, true);  // row_shr:4
        c += __builtin_amdgcn_update_dpp(0u, c, 0x118, 0xF, 0xF, true);  // row_shr:8
        if ((unsigned)__builtin_amdgcn_readlane((int)c, 15) >= target) break;
        if (++spins > a.spin_limit || __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
          if (lane == 0) {
            __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // surface it: the host reads this word after its next synchronising readback
            // (a plain system-scope store, not an atomic: PCIe atomics to host memory are not assumed)
            if (a.status) __hip_atomic_store(a.status, 1u /*CWT_STATUS_ADAPT_BARRIER*/, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_SYSTEM);
            abort_flag = 1;
          }
          break;
        }
        __builtin_amdgcn_s_sleep(PA_POLL_SLEEP);
      }
    }
    stamp(5);
    if (STAMPS && stp) stp[9] = __builtin_amdgcn_s_memrealtime();
    lds_barrier();
    stamp(6);
    if (abort_flag) return false;
    // ---- W of every spanned episode: W1 -= lr_eff * D, W0 += lr_eff * D (same order everywhere).
    // Each wave reads D of its own 32 channels only (its W slice): lanes L < 32 sum replica rows [0, nrep/2),
    // lanes L + 32 rows [nrep/2, nrep), and one v_permlane32_swap adds the halves (the same two
    // partial sums in every workgroup: a + b == b + a) -- no workgroup barrier, no LDS ----
    {
      const int nh = nrep >> 1, hh = lane >> 5;
#pragma unroll
      for (int ew = 0; ew < EWK; ++ew) {
        if (ew >= new_) break;
        const unsigned long long* ap = pa_fx_slot(a, e_lo + ew, slot) + (long)hh * nh * C + cw;
        unsigned long long v[PA_R / 2];
#pragma unroll
        for (int r = 0; r < PA_R / 2; ++r)
          v[r] = r < nh ? __hip_atomic_load(ap + r * C, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
        unsigned long long Di = 0ull;
#pragma unroll
        for (int r = 0; r < PA_R / 2; ++r) Di += v[r];
        // rows [0,nh) + rows [nh,nrep) in every lane (integers: the sum is exact), then one rounding
        const auto slo = __builtin_amdgcn_permlane32_swap((unsigned)Di, (unsigned)Di, false, false);
        const auto shi = __builtin_amdgcn_permlane32_swap((unsigned)(Di >> 32), (unsigned)(Di >> 32), false, false);
        const unsigned long long Do = ((unsigned long long)(lane < 32 ? shi[1] : shi[0]) << 32) |
                                      (unsigned long long)(lane < 32 ? slo[1] : slo[0]);
        const float D = (float)((double)(long long)(Di + Do) * fxi_l[ew]);
        if (lane < 32) {
          const float lr = lr_l[ew];
          const float w1 = wlw[wv][ew][1][lane] - lr * D, w0 = wlw[wv][ew][0][lane] + lr * D;
          wlw[wv][ew][1][lane] = w1;
          wlw[wv][ew][0][lane] = w0;
          dlw[wv][ew][lane] = w1 - w0;
        }
      }
    }
    stamp(7);
  }
  if (STAMPS && t == 0) {
    stp_end[2] = __builtin_amdgcn_s_memrealtime();
    stp_end[3] = __builtin_amdgcn_s_memtime();
  }
  // ---- adapted W: written by the workgroup that owns the episode's first unit ----
#pragma unroll
  for (int ew = 0; ew < EWK; ++ew) {
    const int e = e_lo + ew;
    if (ew < new_ && (long)e * per_ep >= u0 && lane < 32) {
      float* wo = a.dargs[e].w_out;
      wo[cw] = wlw[wv][ew][0][lane];
      wo[C + cw] = wlw[wv][ew][1][lane];
    }
  }
  // the fused tail (one episode: every workgroup holds its W): this workgroup's own copy, read
  // back by this workgroup only
  if (a.wq && lane < 32) {
    float* wq = a.wq + (long)g * 2 * C;
    wq[cw] = wlw[wv][0][0][lane];
    wq[C + cw] = wlw[wv][0][1][lane];
  }
  return true;
}

template <int NRES, int MODE = 0>
__global__ __launch_bounds__(PA_T) void adapt_persist_kernel(PersistArgs a, unsigned long long* stamps = nullptr) {
  (void)adapt_persist_body<NRES, MODE>(a, stamps);
}

// The inner loop with the post-loop episode tail fused behind its last step (one episode, one
// query; EpisodePipeline's adapt context): the loop's workgroups, already resident, run the
// tail's phases (episode_tail_body, tail_body.h) on their first TL_T threads -- the other waves
// exit, and a workgroup barrier then waits for the remaining ones only -- instead of a separate
// grid that must wait for CUs the extractor passes hold.  fst (optional): this launch's slot of
// three realtime stamps, {min over workgroups of the start, max of the loop's end, max of the
// tail's end} (the host pre-sets {~0, 0, 0}); the profile splits the launch into loop and tail
// with them.
template <int NRES>
__global__ __launch_bounds__(PA_T) void adapt_persist_tail_kernel(PersistArgs a, TailArgs ta, unsigned long long* fst) {
  __shared__ __attribute__((aligned(16))) char tail_smem[sizeof(TailTok)];
  __shared__ int tail_abort, tail_last;
  if (fst && threadIdx.x == 0)
    __hip_atomic_fetch_min(fst, (unsigned long long)__builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
  if (!adapt_persist_body<NRES, 0>(a, nullptr)) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this workgroup's W copy is written
  __syncthreads();
  if (fst && threadIdx.x == 0)
    __hip_atomic_fetch_max(fst + 1, (unsigned long long)__builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
  if (threadIdx.x >= TL_T) return;
  ta.q = a.wq + (long)blockIdx.x * 2 * 512;
  episode_tail_body<false>(ta, blockIdx.x, tail_smem, tail_abort, tail_last);
  if (fst && threadIdx.x == 0)
    __hip_atomic_fetch_max(fst + 2, (unsigned long long)__builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// Host side of the persistent loop: G = min(units, CUs).  Returns 1 (not an error) when the
// geometry does not fit it (the caller then uses the per-step launches).
static int g_cu_count = 0;
static int persist_geometry(int E, int n, int h, int w, int upw_pref, int* G_out, int* units_out, int* ncb_out,
                            int* nres_out, int* uc_out) {
  if (!g_cu_count) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&g_cu_count, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      g_cu_count = 0;
    if (g_cu_count <= 0) return 1;
  }
  // 31 owned columns: 15 halves each workgroup's hi-res pixels but doubles the workgroups, and
  // the barrier's atomics and arrivals cost more than that saves (1-shot 473: 7.0 vs 5.9 us per
  // step, tools/persist_stamps.py); CWT_ADAPT_UC=15 selects it
  int uc = PA_UC;
  const char* ucs = getenv("CWT_ADAPT_UC");
  if (ucs && (atoi(ucs) == 15 || atoi(ucs) == 31)) uc = atoi(ucs);
  const int ncb = cdiv(w - 1, uc);
  const int ntile = (h - 1) * ncb;
  const long units = (long)E * n * ntile;
  // units per workgroup: 1 (f in registers) or 2 (the second unit's f in LDS): half the
  // workgroups and CUs left for a concurrent extractor pass.  The context's choice
  // (cwt_ctx_set_adapt_units: EpisodePipeline asks for 2), else CWT_ADAPT_UPW, else 1 while
  // that takes at most half the CUs (1-shot 473^2: 118 workgroups) and 2 beyond
  const char* upws = getenv("CWT_ADAPT_UPW");
  const int upw = upw_pref ? upw_pref : upws ? (atoi(upws) == 1 ? 1 : 2) : (units <= g_cu_count / 2 ? 1 : 2);
  int G = (int)std::min<long>((units + upw - 1) / upw, g_cu_count);
  const long k = (units + G - 1) / G;  // units per workgroup (max)
  const long per_ep = (long)n * ntile;
  const long span = (k - 1 + per_ep - 1) / per_ep + 1;  // episodes a workgroup's range can touch
  // k >= 4 (5-shot 641^2: 1200 units, 4-5 per workgroup): units streamed per wave through LDS
  // (nres 3), 6.04 against 6.35 ms for the step launches; at k = 3 (5-shot 473^2) the stream is
  // slower than the step launches (4.09 against 3.53 ms: the 37 MB per step of f come from the
  // Infinity Cache and the 3-unit workgroups set the pace), so those keep the step launches.
  // CWT_ADAPT_STREAM=0 disables it, =1 allows it from k = 3.
  const char* sts = getenv("CWT_ADAPT_STREAM");
  const int stream_from = sts ? (sts[0] == '0' ? 1 << 30 : 3) : 4;
  // k = 3 (5-shot 473^2: 590 units on 197 workgroups): three units in lockstep, two in
  // registers and one in LDS (nres 4); CWT_ADAPT_LOCK3=0 returns it to the step launches
  const char* l3s = getenv("CWT_ADAPT_LOCK3");
  const bool lock3 = !(l3s && l3s[0] == '0');
  // k = 2: both units in registers (nres 5) unless CWT_ADAPT_BREG=0 (the second unit's f in LDS, nres 2)
  const char* brs = getenv("CWT_ADAPT_BREG");
  const bool breg = !(brs && brs[0] == '0');
  int nres = k == 1 ? 1 : (k == 2 && span <= 2) ? (breg ? 5 : 2) : (k == 3 && span <= 2 && lock3) ? 4 : 0;
  if (nres == 0 && k >= stream_from && span <= 2) nres = 3;
  // the streamed form with the first unit resident in registers (nres 6): opt in with
  // CWT_ADAPT_RES1=1 -- measured slower (5-shot 641^2 alone: 6.77 against 5.87 ms; the resident f
  // does not fit beside the streamed unit at 1,024 threads and 25 VGPRs spill to scratch, whose
  // per-step reloads cost more than the fifth of the stream they save; profiles/r4/run_n)
  const char* r1s = getenv("CWT_ADAPT_RES1");
  if (nres == 3 && r1s && r1s[0] == '1') nres = 6;
  if (span > (nres >= 2 ? 2 : PA_EW)) return 1;
  // three units per workgroup: as few workgroups as that takes (5-shot 473^2: 197, not 256 with
  // two or three units each -- the step waits for the three-unit ones either way, and fewer
  // workgroups make the barrier cheaper and leave CUs free)
  if (nres == 4) G = (int)((units + 2) / 3);
  *G_out = G;
  *units_out = (int)units;
  *ncb_out = ncb;
  *uc_out = uc;
  *nres_out = nres;
  // the register-streamed form (nres 0) is not faster than the step launches: opt in only
  const char* pe = getenv("CWT_ADAPT_PERSIST");
  if (!*nres_out && !(pe && pe[0] == '2')) return 1;
  return 0;
}

static int enqueue_adapt_persist(const float* f, const uint8_t* lbl_ws, const AdaptScalars* sc, float* acc3,
                                 unsigned* cnt, const AdaptDevArgs* dargs, int E, int n, int h, int w, int S,
                                 int iters, int G, int units, int ncb, int nres, int uc, unsigned* status,
                                 long spin_limit, hipStream_t st, const FusedTail* tail) {
  PersistArgs a;
  a.status = status;
  a.spin_limit = spin_limit > 0 ? spin_limit : PA_SPIN_LIMIT;
  a.f = f;
  a.lbl = lbl_ws;
  a.sc = sc;
  a.dargs = dargs;
  a.acc = acc3;
  a.cnt = cnt;
  a.h = h;
  a.w = w;
  a.S = S;
  a.nshot = n;
  a.nep = E;

  a.iters = iters;
  a.ncb = ncb;
  a.ntile = (h - 1) * ncb;
  a.units = units;
  a.G = G;
  a.uc = uc;
  const char* pr = getenv("CWT_ADAPT_PR");
  a.nrep = pr ? atoi(pr) : PA_R_DEFAULT;
  if (a.nrep != 2 && a.nrep != 4 && a.nrep != 8 && a.nrep != 16) a.nrep = PA_R_DEFAULT;
  const char* dbg = getenv("CWT_ADAPT_DBG");
  const int dbgv = dbg ? atoi(dbg) : 0;
  // MODE: 1 stamps (timing study), 2 latency floor (& 64), 3 side leg (& 128), 0 product
  const int mode = (dbgv & 32) ? 1 : (dbgv & 64) ? 2 : (dbgv & 128) ? 3 : 0;
  if (tail) {  // the fused tail: the product instantiation of the two-unit register form only
    if (nres != 5 || mode != 0 || E != 1 || !tail->args || !tail->wq)
      return fail(CWT_EARG, "fused tail: needs the two-unit persistent loop (nres 5), one episode, product mode");
    a.wq = tail->wq;
    hipLaunchKernelGGL((adapt_persist_tail_kernel<5>), dim3(G), dim3(PA_T), 0, st, a, *tail->args, tail->stamps);
    CWT_LAUNCH_CHECK();
    return 0;
  }
  unsigned long long* stp = nullptr;
  if (mode == 1) {  // timing study (tools/persist_stamps.py)
    const long n_st = ((long)iters + 1) * G * 10;
    if (n_st > g_adapt_stamps_n) {
      CWT_HIP(hipDeviceSynchronize());
      if (g_adapt_stamps) CWT_HIP(hipFree(g_adapt_stamps));
      CWT_HIP(hipMalloc(&g_adapt_stamps, n_st * sizeof(unsigned long long)));
      g_adapt_stamps_n = n_st;
    }
    stp = g_adapt_stamps;
  }
#define CWT_PA_LAUNCH(NR, MD) \
  hipLaunchKernelGGL((adapt_persist_kernel<NR, MD>), dim3(G), dim3(PA_T), 0, st, a, stp)
#define CWT_PA_MODES(NR)                     \
  switch (mode) {                            \
    case 1: CWT_PA_LAUNCH(NR, 1); break;     \
    case 2: CWT_PA_LAUNCH(NR, 2); break;     \
    case 3: CWT_PA_LAUNCH(NR, 3); break;     \
    default: CWT_PA_LAUNCH(NR, 0); break;    \
  }
  switch (nres) {
    case 6: CWT_PA_MODES(6); break;
    case 5: CWT_PA_MODES(5); break;
    case 4: CWT_PA_MODES(4); break;
    case 3: CWT_PA_MODES(3); break;
    case 2: CWT_PA_MODES(2); break;
    case 1: CWT_PA_MODES(1); break;
    default: CWT_PA_MODES(0); break;
  }
#undef CWT_PA_MODES
#undef CWT_PA_LAUNCH
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
  *sc = (size_t)E * (sizeof(AdaptScalars) + 2 * PREP_MAXBLK * sizeof(unsigned long long) + PREP_MAXBLK * sizeof(unsigned)) +
        64;
  *acc = (size_t)E * ADAPT_ESTRIDE * sizeof(float) + PA_CNT_WORDS * sizeof(unsigned);  // + persistent-loop counters
  *wbuf = (size_t)E * ADAPT_WSTRIDE * sizeof(float);
  *dargs = (size_t)E * sizeof(AdaptDevArgs);
  return 0;
}

// Workgroups of the persistent inner loop launch_adapt will use for this geometry (each holds a
// whole CU for the whole loop), 0 when it will use the per-step launches
int adapt_persist_workgroups(int E, int n, int h, int w, int iters, int upw) {
  int pG = 0, punits = 0, pncb = 0, pnres = 0, puc = 0;
  const char* pe = getenv("CWT_ADAPT_PERSIST");
  if (iters > 0 && !(pe && pe[0] == '0') && persist_geometry(E, n, h, w, upw, &pG, &punits, &pncb, &pnres, &puc) == 0)
    return pG;
  return 0;
}

// Which inner-loop kernel launch_adapt will use for this geometry (profile record names):
// "adapt_persist_kernel<NRES" or "adapt_step_kernel<"
const char* adapt_kernel_name(int E, int n, int h, int w, int iters, int upw) {
  int pG = 0, punits = 0, pncb = 0, pnres = 0, puc = 0;
  const char* pe = getenv("CWT_ADAPT_PERSIST");
  if (iters > 0 && !(pe && pe[0] == '0') && persist_geometry(E, n, h, w, upw, &pG, &punits, &pncb, &pnres, &puc) == 0) {
    static const char* names[7] = {"adapt_persist_kernel<0", "adapt_persist_kernel<1", "adapt_persist_kernel<2",
                                   "adapt_persist_kernel<3", "adapt_persist_kernel<4", "adapt_persist_kernel<5",
                                   "adapt_persist_kernel<6"};
    return names[pnres <= 6 ? pnres : 0];
  }
  return "adapt_step_kernel<";
}

// E episodes of n shots each: f [E][n][h][w][512], lbl64 [E][n][S][S], W [E][2][512].
int launch_adapt(const float* f, const int64_t* lbl64, int E, int n, int h, int w, int S, float lr, int iters,
                 float* W, float* f_ws /*[E][n][h][w][512]*/, uint8_t* lbl_ws, AdaptScalars* sc /*[E] + partial counts*/,
                 float* acc3 /*[E][3][R][512]*/, float* wbuf /*[E][2][2][512]*/, AdaptDevArgs* dargs /*[E]*/,
                 AdaptGraphCache* cache, int upw, unsigned* status, long spin_limit, hipStream_t st,
                 hipEvent_t ev_k0, hipEvent_t ev_k1, const FusedTail* tail) {
  const long total = (long)n * S * S;  // labels per episode
  unsigned long long* part = (unsigned long long*)(sc + E);  // [E][PREP_MAXBLK][2] after the scalars
  unsigned* fpart = (unsigned*)(part + (long)E * 2 * PREP_MAXBLK);  // [E][PREP_MAXBLK] max |f| bits
  const int pblocks = (int)std::min<long>(PREP_MAXBLK, cdiv(total, 1024));
  const long fcount = (long)n * h * w * 512;
  hipLaunchKernelGGL(adapt_prep_kernel, dim3(pblocks, E), dim3(1024), 0, st, lbl64, total, lbl_ws, part, f, fcount,
                     fpart);
  CWT_LAUNCH_CHECK();
  int pG = 0, punits = 0, pncb = 0, pnres = 0, puc = 0;
  const char* pe = getenv("CWT_ADAPT_PERSIST");
  const bool persist = iters > 0 && !(pe && pe[0] == '0') &&
                       persist_geometry(E, n, h, w, upw, &pG, &punits, &pncb, &pnres, &puc) == 0;
  unsigned* cnt = (unsigned*)(acc3 + (long)E * ADAPT_ESTRIDE);
  hipLaunchKernelGGL(adapt_setup_kernel, dim3(E), dim3(PREP_MAXBLK), 0, st, (const unsigned long long*)part, pblocks,
                     sc, lr, 0, dargs, f, (long)n * h * w * 512, (const float*)W, W, 1024,
                     iters > 0 ? acc3 : (float*)nullptr, ADAPT_ESTRIDE, persist ? 2 * ADAPT_SLOT : ADAPT_SLOT,
                     (double*)nullptr,
                     persist ? cnt : (unsigned*)nullptr, persist ? PA_CNT_WORDS : 0, (const unsigned*)fpart);
  CWT_LAUNCH_CHECK();
  if (iters <= 0) return tail ? fail(CWT_EARG, "fused tail: needs the persistent loop") : 0;
  if (tail && !persist) return fail(CWT_EARG, "fused tail: needs the persistent loop");
  if (persist) {  // one launch for all steps, f read in place (no copy, no graph)
    if (ev_k0) CWT_HIP(hipEventRecord(ev_k0, st));  // profile bracket of the kernel alone (optional)
    const int r = enqueue_adapt_persist(f, lbl_ws, sc, acc3, cnt, dargs, E, n, h, w, S, iters, pG, punits, pncb, pnres,
                                        puc, status, spin_limit, st, tail);
    if (ev_k1) CWT_HIP(hipEventRecord(ev_k1, st));
    return r;
  }
  // (the step launches: the caller records the bracket around the whole call)
  // the step graph reads f from the library's buffer (fixed address, baked into the graph)
  if (f != f_ws)
    CWT_HIP(hipMemcpyAsync(f_ws, f, (size_t)E * n * h * w * 512 * sizeof(float), hipMemcpyDeviceToDevice, st));
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
  // every query pixel ignored (sumw = 0): loss 0/0 = NaN and zero gradients, as torch's
  // CrossEntropyLoss(ignore_index=255) returns them (train.py:261-265)
  const float inv = sumw > 0.0 ? (float)(1.0 / sumw) : 0.f;
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

// The post-loop episode tail's device code (tail.hip's one-launch kernel and the persistent
// inner loop's fused tail share it): arguments, grid barrier, LDS layout and the phases.
#pragma once
#include "common.h"
#include "kernels.h"

namespace cwt {

constexpr int TL_T = 512;              // threads per workgroup (8 waves)
constexpr int TL_NW = TL_T / 64;
constexpr int TL_C = 512;
constexpr int TL_H = 4;
constexpr int TL_NR = 2 * TL_H;        // score rows per episode (query i, head h): rho = i * H + h
constexpr int TL_TPW = 4;              // tokens per wave in a chunk
constexpr int TL_TPB = TL_NW * TL_TPW; // tokens per chunk (= the module token pass's TOK_TPB)
constexpr int TL_MAXCHUNK = 512;
constexpr int TL_NBAR = 5;             // grid barriers per launch
constexpr int TL_REP = 8;              // arrival counter replicas
constexpr int TL_STRIDE = 32;          // words between counters (one per 128-B line)
constexpr int TL_MAXB = 4;

struct TailArgs {
  const float* q;        // [B][2][C] the inner loop's W
  const float* f;        // [B][hw][C] raw query features (channels-last)
  const float* M;        // [H][C][C] folded W_h^T W_h
  const float* P;        // [C][H*C] folded [fc_h W_h]
  const float* fc_b;
  const float* ln_w;
  const float* ln_b;
  const int64_t* target; // [B][S][S]
  int B, hw, h, w, S, G, nchunk;
  float sy, sx;          // align_corners scales h -> S, w -> S
  float* r;              // [B][NR][C]
  float* part_g;         // [B][nchunk][NR][C]
  float* part_ml;        // [B][nchunk][NR][2]
  float* g;              // [B][NR][C]
  float* y;              // [2B][C]
  float* inv;            // [B][hw]
  float* out;            // W' [2B][C]
  float* logits;         // [B][2][hw]
  float* logits0;        // [B][2][hw]
  unsigned* counts;      // [2][B][G][6]
  double* ce_part;       // [B][G][2]
  float* iut;            // [B][3][2]
  double* ce;            // [B][2]
  float* iut0;           // [B][3][2]
  unsigned* cnt;         // TL_REP arrival counters, the ticket, the error word (TL_STRIDE apart)
  unsigned bar_base;     // e * G * NBAR
  unsigned tick_base;    // e * G
  long spin_limit;
  unsigned* status;      // the tail's word of the context's mapped host status (word 1; the loop owns word 0)
  unsigned long long* stamps;  // timing study (ST instantiation): [G][TL_NSTAMP] s_memtime per phase edge
};
constexpr int TL_NSTAMP = 16;

__device__ __forceinline__ void st1(float* p, float v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st1(unsigned* p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st1(double* p, double v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st1x4(float* p, f32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ float ld1(const float* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ unsigned ld1(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld1(const double* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// Grid barrier: every wave's stores performed, one arrival per workgroup on its replica, wave 0
// polls the replicas' sum; returns false when the grid gave up (spin bound or another workgroup's
// abort), after setting the error word and the context's status bit.
__device__ __forceinline__ bool tail_barrier(const TailArgs& a, unsigned target, int* abort_lds) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int t = threadIdx.x, lane = t & 63;
  unsigned* err = a.cnt + (TL_REP + 1) * TL_STRIDE;
  if (t == 0) __hip_atomic_fetch_add(a.cnt + (blockIdx.x % TL_REP) * TL_STRIDE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (t < 64) {
    const unsigned* cp = a.cnt + (lane < TL_REP ? lane : 0) * TL_STRIDE;
    long spins = 0;
    while (true) {
      unsigned c = ld1(cp);
      c = lane < TL_REP ? c : 0u;
      c += __builtin_amdgcn_update_dpp(0u, c, 0x111, 0xF, 0xF, true);  // row_shr:1
      c += __builtin_amdgcn_update_dpp(0u, c, 0x112, 0xF, 0xF, true);  // row_shr:2
      c += __builtin_amdgcn_update_dpp(0u, c, 0x114, 0xF, 0xF, true);  // row_shr:4
      if ((int)((unsigned)__builtin_amdgcn_readlane((int)c, 7) - target) >= 0) break;
      if (++spins > a.spin_limit || ld1(err)) {
        if (lane == 0) {
          st1(err, 1u);
          // a plain system-scope store (PCIe atomics to host memory are not assumed)
          if (a.status) __hip_atomic_store(a.status, 2u /*CWT_STATUS_TAIL_BARRIER*/, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_SYSTEM);
          *abort_lds = 1;
        }
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  return *abort_lds == 0;
}

__device__ __forceinline__ float tl_dot8(f32x4 a0, f32x4 a1, f32x4 b0, f32x4 b1) {
  float d = a0[0] * b0[0];
  d = fmaf(a0[1], b0[1], d);
  d = fmaf(a0[2], b0[2], d);
  d = fmaf(a0[3], b0[3], d);
  d = fmaf(a1[0], b1[0], d);
  d = fmaf(a1[1], b1[1], d);
  d = fmaf(a1[2], b1[2], d);
  return fmaf(a1[3], b1[3], d);
}

// LDS of the phases (one object, carved per phase)
struct TailTok {  // P1
  float rs[TL_NR + 2][TL_C];      // score rows, then W's two rows
  float wg[2][TL_NR][TL_C];       // exp-weighted token sums, rescaled to the chunk max: two slots,
                                  // the waves adding into them two at a time (LDS ~54 KB, so a
                                  // tail workgroup co-resides with an extractor conv's)
  float wml[TL_NW][TL_NR][2];
};
struct TailComb {  // P2
  float ms[TL_MAXCHUNK], ls[TL_MAXCHUNK];
  float sg[TL_NW][64], sl[TL_NW];
};
constexpr int TL_PV = 4;  // P3: score vectors staged per pass
struct TailProj {  // P3
  float gv[TL_PV][TL_H * TL_C];
};
struct TailCls {  // P4
  float w2[2 * TL_MAXB][TL_C];
};
struct TailMet {  // P5
  unsigned c[TL_NW][12];
  double d[TL_NW][2];
  unsigned fc[12][TL_T];  // final (last workgroup): per-thread partials
  double fd[2][TL_T];
};

// The inner loop's fused tail (adapt.hip adapt_persist_tail_kernel): its arguments (q is set per
// workgroup in the kernel), the per-workgroup W copies [G][2][512] and an optional stamp slot
struct FusedTail {
  const TailArgs* args;
  float* wq;
  unsigned long long* stamps;
};

// Host: the arguments of one tail over G workgroups (launch_episode_tail's checks; tail.hip)
int fill_episode_tail_args(const float* q, const float* f, int B, int hw, int h, int w, int S, const int64_t* target,
                           const float* fold, const float* fc_b, const float* ln_w, const float* ln_b, float* out,
                           float* logits, float* logits0, float* iut, double* ce, float* iut0, float* ws,
                           unsigned* cnt, unsigned epoch, int G, long spin_limit, unsigned* status,
                           unsigned long long* stamps, TailArgs* out_args);

static_assert(sizeof(TailComb) <= sizeof(TailTok) && sizeof(TailProj) <= sizeof(TailTok) &&
                  sizeof(TailCls) <= sizeof(TailTok) && sizeof(TailMet) <= sizeof(TailTok),
              "phase LDS fits the token phase's");

// The tail's phases, run by TL_T threads of workgroup gi of the grid's a.G.  smem_raw: the
// workgroup's sizeof(TailTok) bytes of LDS; abort_flag / last_flag: two LDS ints.  The caller is
// episode_tail_kernel (its own launch) or the persistent inner loop's fused tail
// (adapt_persist_kernel<..., TAIL>: its waves past TL_T / 64 have exited before the call, so the
// workgroup barriers here wait for these TL_T threads only).
// ST: the timing-study instantiation (CWT_TAIL_STAMPS=1): thread 0 of every workgroup records
// s_memtime at each phase edge (and s_memrealtime at entry / exit) into a.stamps; never the timed one.
template <bool ST>
__device__ __forceinline__ void episode_tail_body(const TailArgs& a, const int gi, char* smem_raw, int& abort_flag,
                                                  int& last_flag) {
  constexpr int C = TL_C, H = TL_H, NR = TL_NR;
  const int t = threadIdx.x, lane = t & 63, wv = __builtin_amdgcn_readfirstlane(t >> 6);
  const int G = a.G;
  const int B = a.B, nv = 2 * B, hw = a.hw, nchunk = a.nchunk;
  if (t == 0) {
    abort_flag = 0;
    last_flag = 0;
  }
  unsigned long long* stp = (ST && t == 0) ? a.stamps + (long)gi * TL_NSTAMP : nullptr;
  auto stamp = [&](int i) {
    if (ST && stp) stp[i] = __builtin_amdgcn_s_memtime();
  };
  if (ST && stp) stp[14] = __builtin_amdgcn_s_memrealtime();
  stamp(0);
  __syncthreads();

  // this workgroup's first token chunk (f_q is an input): its loads fly under P0 and barrier 1;
  // the registers of its LAST chunk stay live into P4 (the classifier reads the same tokens)
  f32x4 fa[TL_TPW], fb[TL_TPW];
  float invs[TL_TPW];
  auto load_chunk = [&](int ci) {
    const int b = ci / nchunk, chunk = ci - b * nchunk;
    const int tok0 = chunk * TL_TPB + wv * TL_TPW;
#pragma unroll
    for (int tt = 0; tt < TL_TPW; ++tt) {
      const int p = tok0 + tt;
      if (p < hw) {
        const float* src = a.f + ((long)b * hw + p) * C + 4 * lane;
        fa[tt] = *(const f32x4*)src;
        fb[tt] = *(const f32x4*)(src + 256);
      } else {
        fa[tt] = fb[tt] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  };
  const int last_ci = gi < B * nchunk ? gi + ((B * nchunk - 1 - gi) / G) * G : -1;
  if (gi < B * nchunk) load_chunk(gi);

  // ---- P0: r[v][h*C + k] = M[h*C + k] . q[v] / sqrt(C) (rowdot_kernel<8>'s per-lane partition) ----
  {
    const float alpha = 1.0f / sqrtf((float)C);
    for (int row = gi * TL_NW + wv; row < H * C; row += G * TL_NW) {
      const float* ar = a.M + (long)row * C + lane * 4;
      const f32x4 u0 = *(const f32x4*)ar, u1 = *(const f32x4*)(ar + 256);
      for (int v = 0; v < nv; ++v) {
        const float* xr = a.q + (long)v * C + lane * 4;
        const f32x4 x0 = *(const f32x4*)xr, x1 = *(const f32x4*)(xr + 256);
        float s = 0.f;  // rowdot_kernel<8>'s order: the lane's 4 channels at +0, then at +256
#pragma unroll
        for (int c = 0; c < 4; ++c) s = fmaf(u0[c], x0[c], s);
#pragma unroll
        for (int c = 0; c < 4; ++c) s = fmaf(u1[c], x1[c], s);
        s = wave_sum(s);
        if (lane == 0) st1(a.r + (long)v * H * C + row, alpha * s);
      }
    }
  }
  stamp(1);
  if (!tail_barrier(a, a.bar_base + (unsigned)G * 1, &abort_flag)) return;
  stamp(2);

  // ---- P1: the token pass over this workgroup's chunks (attn_tokens_kernel) ----
  {
    TailTok& L = *(TailTok*)smem_raw;
    int b_loaded = -1;
    for (int ci = gi; ci < B * nchunk; ci += G) {
      const int b = ci / nchunk, chunk = ci - b * nchunk;
      __syncthreads();  // the previous chunk's LDS reads are done
      if (b != b_loaded) {
        for (int i = t; i < (NR + 2) * C; i += TL_T) {
          const int row = i / C, k = i - row * C;
          L.rs[row][k] = row < NR ? ld1(a.r + ((long)b * NR + row) * C + k) : a.q[((long)b * 2 + row - NR) * C + k];
        }
        b_loaded = b;
      }
      const int tok0 = chunk * TL_TPB + wv * TL_TPW;
      if (ci != gi) load_chunk(ci);  // the first one was loaded before P0
      __syncthreads();
      float v[64];
#pragma unroll
      for (int rho = 0; rho < NR; ++rho) {
        const f32x4 ra = *(const f32x4*)&L.rs[rho][4 * lane], rb = *(const f32x4*)&L.rs[rho][256 + 4 * lane];
#pragma unroll
        for (int tt = 0; tt < TL_TPW; ++tt) v[tt * NR + rho] = tl_dot8(ra, rb, fa[tt], fb[tt]);
      }
      {
        const f32x4 w0a = *(const f32x4*)&L.rs[NR][4 * lane], w0b = *(const f32x4*)&L.rs[NR][256 + 4 * lane];
        const f32x4 w1a = *(const f32x4*)&L.rs[NR + 1][4 * lane], w1b = *(const f32x4*)&L.rs[NR + 1][256 + 4 * lane];
#pragma unroll
        for (int tt = 0; tt < TL_TPW; ++tt) {
          v[32 + tt * 8] = tl_dot8(fa[tt], fb[tt], fa[tt], fb[tt]);
          v[32 + tt * 8 + 1] = tl_dot8(w0a, w0b, fa[tt], fb[tt]);
          v[32 + tt * 8 + 2] = tl_dot8(w1a, w1b, fa[tt], fb[tt]);
#pragma unroll
          for (int j = 3; j < 8; ++j) v[32 + tt * 8 + j] = 0.f;
        }
      }
      const float red = butterfly_sum<64>(v, lane);  // lane L: value L
      const bool score_lane = lane < 32;
      const int my_t = (lane & 31) / NR, my_rho = lane % NR;
      const int p = tok0 + my_t;
      const bool valid = score_lane && p < hw;
      const float nrm2 = __shfl(red, 32 + my_t * 8, 64);
      const float inv = 1.0f / fmaxf(sqrtf(nrm2), 1e-12f);
#pragma unroll
      for (int tt = 0; tt < TL_TPW; ++tt) invs[tt] = __shfl(inv, tt * NR, 64);  // lane tt NR: token tt
      if (ci != last_ci && valid && my_rho == 0) a.inv[(long)b * hw + p] = inv;  // read back by this workgroup only (P4)
      if (lane >= 32 && ((lane & 7) == 1 || (lane & 7) == 2)) {
        const int pt = tok0 + ((lane - 32) >> 3);
        if (pt < hw) st1(a.logits0 + ((long)b * 2 + (lane & 7) - 1) * hw + pt, red);
      }
      const float sc = valid ? red * inv : -INFINITY;
      float m = sc;
      m = fmaxf(m, __shfl_xor(m, 8, 64));
      m = fmaxf(m, __shfl_xor(m, 16, 64));
      const float e = valid ? __expf(sc - m) : 0.f;
      float l = e;
      l += __shfl_xor(l, 8, 64);
      l += __shfl_xor(l, 16, 64);
      const float wgt = e * inv;
      f32x4 ga[NR], gb[NR];
#pragma unroll
      for (int rho = 0; rho < NR; ++rho) ga[rho] = gb[rho] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int tt = 0; tt < TL_TPW; ++tt)
#pragma unroll
        for (int rho = 0; rho < NR; ++rho) {
          const float w = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wgt), tt * NR + rho));
          ga[rho] += w * fa[tt];
          gb[rho] += w * fb[tt];
        }
      if (lane < NR) {
        L.wml[wv][lane][0] = m;
        L.wml[wv][lane][1] = l;
      }
      __syncthreads();
      // rescale this wave's sums to the chunk max of each rho, then add them into slot wv & 1,
      // waves (0, 1) first, then (2, 3), ...: slot s = ((w_s + w_{s+2}) + w_{s+4}) + w_{s+6}
      float sw[NR];
#pragma unroll
      for (int rho = 0; rho < NR; ++rho) {
        float M = -INFINITY;
#pragma unroll
        for (int w = 0; w < TL_NW; ++w) M = fmaxf(M, L.wml[w][rho][0]);
        sw[rho] = (L.wml[wv][rho][0] == -INFINITY) ? 0.f : __expf(L.wml[wv][rho][0] - M);
      }
      for (int r = 0; r < TL_NW / 2; ++r) {
        if ((wv >> 1) == r) {
          const int slot = wv & 1;
#pragma unroll
          for (int rho = 0; rho < NR; ++rho) {
            f32x4* da = (f32x4*)&L.wg[slot][rho][4 * lane];
            f32x4* db = (f32x4*)&L.wg[slot][rho][256 + 4 * lane];
            const f32x4 xa = sw[rho] * ga[rho], xb = sw[rho] * gb[rho];
            *da = r ? *da + xa : xa;
            *db = r ? *db + xb : xb;
          }
        }
        __syncthreads();
      }
      for (int i = t; i < NR * (C / 4); i += TL_T) {
        const int rho = i / (C / 4), c4 = i - rho * (C / 4);
        float M = -INFINITY;
#pragma unroll
        for (int w = 0; w < TL_NW; ++w) M = fmaxf(M, L.wml[w][rho][0]);
        const f32x4 Gs = *(const f32x4*)&L.wg[0][rho][c4 * 4] + *(const f32x4*)&L.wg[1][rho][c4 * 4];
        float Ls = 0.f;
#pragma unroll
        for (int w = 0; w < TL_NW; ++w) {
          const float s = (L.wml[w][rho][0] == -INFINITY) ? 0.f : __expf(L.wml[w][rho][0] - M);
          Ls = fmaf(s, L.wml[w][rho][1], Ls);
        }
        st1x4(a.part_g + (((long)b * nchunk + chunk) * NR + rho) * C + c4 * 4, Gs);
        if (c4 == 0) {
          st1(a.part_ml + (((long)b * nchunk + chunk) * NR + rho) * 2, M);
          st1(a.part_ml + (((long)b * nchunk + chunk) * NR + rho) * 2 + 1, Ls);
        }
      }
    }
  }
  stamp(3);
  if (!tail_barrier(a, a.bar_base + (unsigned)G * 2, &abort_flag)) return;
  stamp(4);

  // ---- P2: combine the chunk partials: g[b][rho][k] (items: b, rho, 64-channel block) ----
  {
    TailComb& L = *(TailComb*)smem_raw;
    for (int item = gi; item < B * NR * (C / 64); item += G) {
      const int b = item / (NR * (C / 64)), rem = item - b * NR * (C / 64);
      const int rho = rem / (C / 64), kb = rem - rho * (C / 64);
      const int k = kb * 64 + lane;
      __syncthreads();
      for (int c = t; c < nchunk; c += TL_T) {
        L.ms[c] = ld1(a.part_ml + (((long)b * nchunk + c) * NR + rho) * 2);
        L.ls[c] = ld1(a.part_ml + (((long)b * nchunk + c) * NR + rho) * 2 + 1);
      }
      __syncthreads();
      float M = -INFINITY;
      for (int c = lane; c < nchunk; c += 64) M = fmaxf(M, L.ms[c]);
      M = wave_max(M);
      const float* pg = a.part_g + ((long)b * nchunk * NR + rho) * C + k;
      float Gs = 0.f, Ls = 0.f;
      for (int c0 = wv; c0 < nchunk; c0 += 16 * TL_NW) {  // 16 chunks per round, all loads in flight
        float gc[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) gc[u] = ld1(pg + (long)min(c0 + TL_NW * u, nchunk - 1) * NR * C);
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int c = c0 + TL_NW * u;
          if (c >= nchunk) break;
          const float s = (L.ms[c] == -INFINITY) ? 0.f : __expf(L.ms[c] - M);
          Gs = fmaf(s, gc[u], Gs);
          Ls = fmaf(s, L.ls[c], Ls);
        }
      }
      L.sg[wv][lane] = Gs;
      if (lane == 0) L.sl[wv] = Ls;
      __syncthreads();
      if (wv == 0) {
        const float Gt = ((L.sg[0][lane] + L.sg[1][lane]) + (L.sg[2][lane] + L.sg[3][lane])) +
                         ((L.sg[4][lane] + L.sg[5][lane]) + (L.sg[6][lane] + L.sg[7][lane]));
        const float Lt = ((L.sl[0] + L.sl[1]) + (L.sl[2] + L.sl[3])) + ((L.sl[4] + L.sl[5]) + (L.sl[6] + L.sl[7]));
        st1(a.g + ((long)b * NR + rho) * C + k, Gt / Lt);
      }
    }
  }
  stamp(5);
  if (!tail_barrier(a, a.bar_base + (unsigned)G * 3, &abort_flag)) return;
  stamp(6);

  // ---- P3: y[v][j] = P[j] . g_v + fc_b[j] + q_v[j] (rowdot_kernel<32>'s per-lane partition) ----
  {
    TailProj& L = *(TailProj*)smem_raw;
    for (int v0 = 0; v0 < nv; v0 += TL_PV) {
    const int npv = min(TL_PV, nv - v0);
    __syncthreads();  // the previous pass's reads are done
    for (int i = t; i < npv * H * C; i += TL_T) L.gv[i / (H * C)][i % (H * C)] = ld1(a.g + (long)v0 * H * C + i);
    __syncthreads();
    for (int row = gi * TL_NW + wv; row < C; row += G * TL_NW) {
      float av[32];
      const float* ar = a.P + (long)row * H * C + lane * 4;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const f32x4 u = *(const f32x4*)(ar + c * 256);
        av[4 * c] = u[0];
        av[4 * c + 1] = u[1];
        av[4 * c + 2] = u[2];
        av[4 * c + 3] = u[3];
      }
      for (int vi = 0; vi < npv; ++vi) {
        const int v = v0 + vi;
        float s = 0.f;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          const f32x4 u = *(const f32x4*)&L.gv[vi][c * 256 + lane * 4];
          s = fmaf(av[4 * c], u[0], s);
          s = fmaf(av[4 * c + 1], u[1], s);
          s = fmaf(av[4 * c + 2], u[2], s);
          s = fmaf(av[4 * c + 3], u[3], s);
        }
        s = wave_sum(s);
        if (lane == 0) st1(a.y + (long)v * C + row, s + a.fc_b[row] + a.q[(long)v * C + row]);
      }
    }
    }
  }
  stamp(7);
  if (!tail_barrier(a, a.bar_base + (unsigned)G * 4, &abort_flag)) return;
  stamp(8);

  // ---- P4: LayerNorm (each workgroup its own copy of W'), then pred_q over this workgroup's
  // token chunks: (W' . f_p) / ||f_p|| (classify_scaled_kernel) ----
  {
    TailCls& L = *(TailCls*)smem_raw;
    if (wv < nv) {  // layernorm_kernel: wave v normalises row v
      float x[8];
      float s = 0.f;
#pragma unroll
      for (int qq = 0; qq < 8; ++qq) {
        x[qq] = ld1(a.y + (long)wv * C + lane + 64 * qq);
        s += x[qq];
      }
      const float mean = wave_sum(s) / (float)C;
      float ss = 0.f;
#pragma unroll
      for (int qq = 0; qq < 8; ++qq) {
        const float d = x[qq] - mean;
        ss = fmaf(d, d, ss);
      }
      const float var = wave_sum(ss) / (float)C;
      const float rstd = 1.0f / sqrtf(var + 1e-5f);
#pragma unroll
      for (int qq = 0; qq < 8; ++qq) {
        const int k = lane + 64 * qq;
        const float o = (x[qq] - mean) * rstd * a.ln_w[k] + a.ln_b[k];
        L.w2[wv][k] = o;
        if (gi == 0) a.out[(long)wv * C + k] = o;
      }
    }
    __syncthreads();
    for (int ci = last_ci; ci >= 0; ci -= G) {  // the last token chunk first: its tokens are in registers
      const int b = ci / nchunk, chunk = ci - b * nchunk;
      const bool regs = ci == last_ci;
      const f32x4 w0a = *(const f32x4*)&L.w2[2 * b][lane * 4], w0b = *(const f32x4*)&L.w2[2 * b][256 + lane * 4];
      const f32x4 w1a = *(const f32x4*)&L.w2[2 * b + 1][lane * 4], w1b = *(const f32x4*)&L.w2[2 * b + 1][256 + lane * 4];
#pragma unroll
      for (int tt = 0; tt < TL_TPW; ++tt) {
        const int p = chunk * TL_TPB + wv * TL_TPW + tt;
        if (p >= hw) break;
        const float* src = a.f + ((long)b * hw + p) * C + lane * 4;
        const f32x4 u = regs ? fa[tt] : *(const f32x4*)src, vv = regs ? fb[tt] : *(const f32x4*)(src + 256);
        float s0 = 0.f, s1 = 0.f;
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          s0 = fmaf(w0a[qq], u[qq], s0);
          s0 = fmaf(w0b[qq], vv[qq], s0);
          s1 = fmaf(w1a[qq], u[qq], s1);
          s1 = fmaf(w1b[qq], vv[qq], s1);
        }
        s0 = wave_sum_dpp(s0);
        s1 = wave_sum_dpp(s1);
        if (lane == 0) {
          const float iv = regs ? invs[tt] : ld1(a.inv + (long)b * hw + p);
          st1(a.logits + (long)b * 2 * hw + p, s0 * iv);
          st1(a.logits + (long)b * 2 * hw + hw + p, s1 * iv);
        }
      }
    }
  }
  stamp(9);
  if (!tail_barrier(a, a.bar_base + (unsigned)G * 5, &abort_flag)) return;
  stamp(10);

  // ---- P5: upsample (align_corners) + argmax + counts + CE (seg_metrics_kernel's per-pixel
  // math) of pred_q and pred_q0; per-workgroup partials, summed by the last arriver ----
  {
    TailMet& L = *(TailMet*)smem_raw;
    const long npix = (long)a.S * a.S, plane = (long)a.h * a.w;
    // this workgroup's pixels: one contiguous range of the S x S image per episode; the low-res
    // rows its bilinear footprint touches (four planes: pred_q, pred_q0) are staged in LDS when
    // they fit beside the partials -- the per-pixel reads then hit LDS, not sixteen sc1 loads
    const long p0 = npix * gi / G, p1 = npix * (gi + 1) / G;
    const int Y0 = (int)(p0 / a.S), Y1 = (int)((p1 > p0 ? p1 - 1 : p0) / a.S);
    const int ylo = lerp_coord(Y0, a.h, a.sy).i0, yhi = lerp_coord(Y1, a.h, a.sy).i1;
    const long nrow = (long)(yhi - ylo + 1) * a.w;  // staged floats per plane
    float* lg = (float*)(smem_raw + sizeof(TailMet));
    const bool in_lds = 4 * nrow * (long)sizeof(float) <= (long)(sizeof(TailTok) - sizeof(TailMet));
    for (int b = 0; b < B; ++b) {
      const float* L0 = a.logits + (long)b * 2 * plane;
      const float* L1 = L0 + plane;
      const float* K0 = a.logits0 + (long)b * 2 * plane;
      const float* K1 = K0 + plane;
      long obase = 0;  // subtracted from every plane offset when staged
      if (in_lds) {
        __syncthreads();  // the previous episode's reads of lg are done
        const long r0 = (long)ylo * a.w;
        for (long i = t; i < nrow; i += TL_T) {
          lg[i] = ld1(L0 + r0 + i);
          lg[nrow + i] = ld1(L1 + r0 + i);
          lg[2 * nrow + i] = ld1(K0 + r0 + i);
          lg[3 * nrow + i] = ld1(K1 + r0 + i);
        }
        __syncthreads();
        L0 = lg;
        L1 = lg + nrow;
        K0 = lg + 2 * nrow;
        K1 = lg + 3 * nrow;
        obase = r0;
      }
      auto rd = [&](const float* pp, long o) { return in_lds ? pp[o - obase] : ld1(pp + o); };
      unsigned c[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
      double nll = 0.0;
      unsigned nvalid = 0;
      for (long i = p0 + t; i < p1; i += TL_T) {
        const int Y = (int)(i / a.S), X = (int)(i - (long)Y * a.S);
        const Lerp ly = lerp_coord(Y, a.h, a.sy), lx = lerp_coord(X, a.w, a.sx);
        const long o00 = ly.i0 * a.w + lx.i0, o01 = ly.i0 * a.w + lx.i1, o10 = ly.i1 * a.w + lx.i0,
                   o11 = ly.i1 * a.w + lx.i1;
        const float l0 = ly.l0 * (lx.l0 * rd(L0, o00) + lx.l1 * rd(L0, o01)) +
                         ly.l1 * (lx.l0 * rd(L0, o10) + lx.l1 * rd(L0, o11));
        const float l1 = ly.l0 * (lx.l0 * rd(L1, o00) + lx.l1 * rd(L1, o01)) +
                         ly.l1 * (lx.l0 * rd(L1, o10) + lx.l1 * rd(L1, o11));
        const float k0 = ly.l0 * (lx.l0 * rd(K0, o00) + lx.l1 * rd(K0, o01)) +
                         ly.l1 * (lx.l0 * rd(K0, o10) + lx.l1 * rd(K0, o11));
        const float k1 = ly.l0 * (lx.l0 * rd(K1, o00) + lx.l1 * rd(K1, o01)) +
                         ly.l1 * (lx.l0 * rd(K1, o10) + lx.l1 * rd(K1, o11));
        const int64_t tg = a.target[(long)b * npix + i];
        if (tg == 255) continue;
        const int pred = (l1 > l0) ? 1 : 0, pred0 = (k1 > k0) ? 1 : 0;  // torch.argmax: first index on ties
        // every counter by a constant index (a dynamic index would put c[] in scratch, which the
        // compiler then promotes to 48 KB of LDS per 1024-thread workgroup)
        c[2] += pred == 0;
        c[3] += pred == 1;
        c[8] += pred0 == 0;
        c[9] += pred0 == 1;
        if (tg == 0 || tg == 1) {
          c[4] += tg == 0;
          c[5] += tg == 1;
          c[10] += tg == 0;
          c[11] += tg == 1;
          c[0] += pred == tg && pred == 0;
          c[1] += pred == tg && pred == 1;
          c[6] += pred0 == tg && pred0 == 0;
          c[7] += pred0 == tg && pred0 == 1;
          const float m = fmaxf(l0, l1);
          const float lse = m + logf(expf(l0 - m) + expf(l1 - m));
          nll += (double)(lse - (tg == 1 ? l1 : l0));
          nvalid++;
        }
      }
#pragma unroll
      for (int k = 0; k < 12; ++k)
        for (int o = 32; o > 0; o >>= 1) c[k] += __shfl_xor(c[k], o, 64);
      for (int o = 32; o > 0; o >>= 1) {
        nll += __shfl_xor(nll, o, 64);
        nvalid += __shfl_xor(nvalid, o, 64);
      }
      __syncthreads();  // the previous episode's LDS partials are read
      if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 12; ++k) L.c[wv][k] = c[k];
        L.d[wv][0] = nll;
        L.d[wv][1] = (double)nvalid;
      }
      __syncthreads();
      if (t < 12) {
        unsigned s = 0;
#pragma unroll
        for (int w = 0; w < TL_NW; ++w) s += L.c[w][t];
        st1(a.counts + (((long)(t / 6) * B + b) * G + gi) * 6 + (t % 6), s);
      } else if (t < 14) {
        const int q = t - 12;
        const double s = ((L.d[0][q] + L.d[1][q]) + (L.d[2][q] + L.d[3][q])) +
                         ((L.d[4][q] + L.d[5][q]) + (L.d[6][q] + L.d[7][q]));
        st1(a.ce_part + ((long)b * G + gi) * 2 + q, s);
      }
    }
    // ticket: the last workgroup to arrive sums the partials in workgroup order (deterministic)
    stamp(11);
    if (ST && stp) stp[15] = __builtin_amdgcn_s_memrealtime();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
      const unsigned old = __hip_atomic_fetch_add(a.cnt + TL_REP * TL_STRIDE, 1u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
      last_flag = (old == a.tick_base + (unsigned)G - 1u) ? 1 : 0;
    }
    __syncthreads();
    if (!last_flag) return;
    for (int b = 0; b < B; ++b) {
      const bool have = t < G;
#pragma unroll
      for (int q = 0; q < 12; ++q)
        L.fc[q][t] = have ? ld1(a.counts + (((long)(q / 6) * B + b) * G + t) * 6 + (q % 6)) : 0u;
      L.fd[0][t] = have ? ld1(a.ce_part + ((long)b * G + t) * 2) : 0.0;
      L.fd[1][t] = have ? ld1(a.ce_part + ((long)b * G + t) * 2 + 1) : 0.0;
      __syncthreads();
      for (int o = TL_T / 2; o > 0; o >>= 1) {
        if (t < o) {
#pragma unroll
          for (int q = 0; q < 12; ++q) L.fc[q][t] += L.fc[q][t + o];
          L.fd[0][t] += L.fd[0][t + o];
          L.fd[1][t] += L.fd[1][t + o];
        }
        __syncthreads();
      }
      if (t < 2) {
        a.iut[b * 6 + t] = (float)L.fc[t][0];                                   // intersection
        a.iut[b * 6 + 2 + t] = (float)(L.fc[2 + t][0] + L.fc[4 + t][0] - L.fc[t][0]);  // union
        a.iut[b * 6 + 4 + t] = (float)L.fc[4 + t][0];                           // target
        a.iut0[b * 6 + t] = (float)L.fc[6 + t][0];
        a.iut0[b * 6 + 2 + t] = (float)(L.fc[8 + t][0] + L.fc[10 + t][0] - L.fc[6 + t][0]);
        a.iut0[b * 6 + 4 + t] = (float)L.fc[10 + t][0];
        a.ce[b * 2 + t] = L.fd[t][0];
      }
      __syncthreads();
    }
  }
}

}  // namespace cwt

// The LDS-DMA implicit-GEMM conv body shared by conv_x3s.hip (bf16x3, plain bf16, exact fp32)
// and conv_x6.hip (fp32 width on the bf16 matrix cores); the design notes are at the top of
// conv_x3s.hip (S-layout, main loop, epilogue) and above split3_bf16 (PREC 6).
#pragma once
#include "common.h"
#include "kernels.h"

namespace cwt {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

#define CWT_LDS __attribute__((address_space(3)))
#define CWT_GLB __attribute__((address_space(1)))

__device__ __forceinline__ void glds16(const void* src, char* lds_dst) {
  __builtin_amdgcn_global_load_lds((const CWT_GLB void*)src, (CWT_LDS void*)lds_dst, 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// vmcnt(n * LPT) for a runtime n in [0, 5]
template <int LPT>
__device__ __forceinline__ void wait_tiles(int n) {
  if (n <= 0)
    wait_vmcnt<0>();
  else if (n == 1)
    wait_vmcnt<LPT>();
  else if (n == 2)
    wait_vmcnt<2 * LPT>();
  else if (n == 3)
    wait_vmcnt<3 * LPT>();
  else if (n == 4)
    wait_vmcnt<4 * LPT>();
  else
    wait_vmcnt<5 * LPT>();
}

__device__ __forceinline__ void block_sync_lds() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Residual of 8 consecutive channels [co, co + 8) of output row m (0 without a residual).
struct Res8 {
  f32x4 a, b;  // fp32 residual, or the S-layout hi / lo halves (PREC 1: a = 8 bf16) reinterpreted
};
template <int PREC>
__device__ __forceinline__ Res8 load_res8(const ConvSArgs& a, int m, int co) {
  Res8 r;
  if (a.res) {
    const f32x4* rp = (const f32x4*)(a.res + (long)m * a.res_ld + co);
    r.a = rp[0];
    r.b = rp[1];
  } else if (a.res_s) {
    if (PREC == 1) {
      r.a = *(const f32x4*)(a.res_s + (long)m * a.Co + co);
      r.b = f32x4{0.f, 0.f, 0.f, 0.f};
    } else {
      const __bf16* rp = a.res_s + ((long)m * (a.Co >> 5) + (co >> 5)) * 64 + (co & 31);
      r.a = *(const f32x4*)rp;
      r.b = *(const f32x4*)(rp + 32);
    }
  } else {
    r.a = r.b = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  return r;
}

// 8 consecutive channels [co, co + 8) of output row m: BN, residual, ReLU, stores.
template <int PREC>
__device__ __forceinline__ void store_out8(const ConvSArgs& a, int m, int co, const float* v, const float* sc,
                                           const float* sh, const Res8& rs) {
  float o[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = fmaf(v[i], sc[i], sh[i]);
  if (a.res) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      o[i] += rs.a[i];
      o[4 + i] += rs.b[i];
    }
  } else if (a.res_s) {
    const bf16x8 rh = __builtin_bit_cast(bf16x8, rs.a), rl = __builtin_bit_cast(bf16x8, rs.b);
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] += PREC == 1 ? (float)rh[i] : (float)rh[i] + (float)rl[i];
  }
  if (a.relu) {
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = fmaxf(o[i], 0.f);
  }
  if (a.y) {
    f32x4* yp = (f32x4*)(a.y + (long)m * a.y_ld + a.y_off + co);
    yp[0] = f32x4{o[0], o[1], o[2], o[3]};
    yp[1] = f32x4{o[4], o[5], o[6], o[7]};
  }
  if (a.ys) {
    bf16x8 hi, lo;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      hi[i] = (__bf16)o[i];
      lo[i] = (__bf16)(o[i] - (float)hi[i]);
    }
    if (PREC == 1) {
      *(bf16x8*)(a.ys + (long)m * a.Co + co) = hi;
    } else {
      __bf16* sp = a.ys + ((long)m * (a.Co >> 5) + (co >> 5)) * 64 + (co & 31);
      *(bf16x8*)sp = hi;
      *(bf16x8*)(sp + 32) = lo;
    }
  }
}

// PREC = 6 (conv_igemm_x6, the fp32-width path on the bf16 matrix cores): every fp32 operand is
// split EXACTLY into three bf16 terms x = hi + mid + lo: hi = bf16_rne(x), mid = bf16_rne(x - hi),
// lo = x - hi - mid (|lo| <= 2^-16 |x|, at most 8 significant bits, so its bf16 conversion is
// exact).  a.b is summed from the six products whose size is >= 2^-24 |a||b| (hi.hi, hi.mid,
// mid.hi, mid.mid, hi.lo, lo.hi) with fp32 accumulation; the three dropped (mid.lo, lo.mid, lo.lo)
// total < 2^-23 |a||b|, the size of one fp32 rounding.  One v_mfma_f32_16x16x32_bf16 covers the
// whole 32-deep K-tile, so a fragment pair costs 6 x 16 cycles against the f32 MFMA's 8 x 32.
// The activations stay fp32 NHWC (conv_igemm_f32d's bytes) and are split in registers after the
// fragment read; the weights, static, are split once at load: the S-layout line [32 hi | 32 mid]
// (the bf16x3 kernel's own packed weights) plus a lo plane [Co][K/32][32 lo] (64-B rows), both
// moved to LDS by LDS-DMA, so the main loop's VALU splits only the A fragments.
__device__ __forceinline__ void split3_bf16(const f32x4& x0, const f32x4& x1, bf16x8& h, bf16x8& m, bf16x8& l) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float v = i < 4 ? x0[i] : x1[i - 4];
    const __bf16 hv = (__bf16)v;
    const float r = v - (float)hv;
    const __bf16 mv = (__bf16)r;
    h[i] = hv;
    m[i] = mv;
    l[i] = (__bf16)(r - (float)mv);
  }
}

// PF = 0: fragments of tile t are read after the barrier that publishes it, then its MFMAs.
// PF = 1: fragments of tile t+1 are read (into a second register set) right after the barrier
// that publishes it, BEFORE the MFMAs of tile t, so their LDS latency hides under the MFMAs;
// the slot tile t occupied is refilled (tile t + NSTG) as soon as every wave has passed that
// barrier, so the ring keeps NSTG - 1 tiles in flight either way.
// PF bits: 1 fragment prefetch; 2 / 4 timing studies (no MFMAs / no operand DMA); 8 buffer
// addressing of the operand DMA (every production instantiation sets it); 16 timing study of the
// x6 WN = 128 forms without the A split (wrong numbers, same data movement and MFMAs); 32 timing
// study without the epilogue; 64 timing study: every workgroup returns at once (the launch alone).
template <int BM, int BN, int WAVES_M, int WAVES_N, int NSTG, int PREC, int PF>
__device__ __forceinline__ void conv_s_body(const ConvSArgs& a) {
  static_assert(PREC == 0 || PREC == 1 || PREC == 3 || PREC == 6,
                "PREC: 3 = bf16x3 over the S-layout, 1 = plain bf16, 0 = exact fp32 (f32 MFMA), "
                "6 = fp32 operands split three ways in registers (bf16x6)");
  constexpr int NW = WAVES_M * WAVES_N;
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  constexpr int FM = WM / 16, FN = WN / 16;
  constexpr int LA = BM / (8 * NW), LB = BN / (8 * NW);  // LDS-DMA pieces (8 rows x 128 B) per wave per tile
  // PREC 6: the weights' lo plane, pieces of 16 rows x 64 B; with fewer pieces than waves the
  // surplus waves repeat one (identical bytes to the same LDS slot), so every wave issues the same
  // count per tile (the vmcnt accounting)
  constexpr int NLO = PREC == 6 ? BN / 16 : 0;
  constexpr int LBL = PREC == 6 ? (NLO + NW - 1) / NW : 0;
  constexpr int LPT = LA + LB + LBL;
  constexpr int LO_OFF = (BM + BN) * 128;  // the lo plane's place in a stage
  constexpr int STG_BYTES = (BM + BN) * 128 + (PREC == 6 ? BN * 64 : 0);
  static_assert(LA * 8 * NW == BM && LB * 8 * NW == BN, "tile rows must split into 8-row pieces per wave");
  static_assert(NSTG >= 2 && NSTG <= 6, "ring depth");
  constexpr int EP_ROWS = WM < 32 ? WM : 32;
  constexpr int EP_LD = WN + 4;  // floats per row of a wave's epilogue tile
  constexpr int EP_BYTES = NW * EP_ROWS * EP_LD * 4;
  constexpr int SMEM = NSTG * STG_BYTES > EP_BYTES ? NSTG * STG_BYTES : EP_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];  // the one LDS object (ring + epilogue)

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wv / WAVES_N, wn = wv % WAVES_N;
  int mt, nt, ks;
  conv_tile_coords(mt, nt, ks);
  // batched GEMMs (PREC 6, the Winograd products): grid.z = batch, one whole K range each
  const bool batched = PREC == 6 && a.batch > 1;
  const int bidx = batched ? ks : 0;
  if (batched) ks = 0;
  const char* xs_b = (const char*)a.xs + (batched ? bidx * a.xs_bstride : 0L);
  const __bf16* ws_b = a.ws + (batched ? bidx * a.ws_bstride : 0L);
  const __bf16* wl_b = a.ws_lo + (batched ? bidx * a.wl_bstride : 0L);
  float* part_b = a.part + (batched ? (long)bidx * a.M * a.Co : 0L);
  const int m0 = mt * BM, n0 = nt * BN;
  const int kt_begin = ks * a.kt_per_split;
  const int kt_end = min(a.ktiles, kt_begin + a.kt_per_split);
  const int T = kt_end - kt_begin;
  if constexpr ((PF & 64) != 0) {  // timing study (x6 var 18): the launch alone (every workgroup returns here)
    asm volatile("" ::"s"(T));
    return;
  }


  // ---- LDS-DMA source geometry (constant over K) ----
  const int lrow = lane >> 3, lslot = lane & 7;
  const int cblocks = a.Ci >> (PREC == 1 ? 6 : 5);  // 128-B lines per pixel
  int a_ih0[LA], a_iw0[LA], a_pix0[LA], a_ch[LA];
  const int HoWo = a.Ho * a.Wo;
#pragma unroll
  for (int j = 0; j < LA; ++j) {
    const int r = (wv * LA + j) * 8 + lrow;
    a_ch[j] = (lslot ^ ((r >> 1) & 7)) * 8;
    const int m = m0 + r;
    if (m < a.M) {
      const int n = m / HoWo;
      const int rem = m - n * HoWo;
      const int oh = rem / a.Wo;
      const int ow = rem - oh * a.Wo;
      a_ih0[j] = oh * a.stride - a.pad;
      a_iw0[j] = ow * a.stride - a.pad;
      a_pix0[j] = (n * a.Hi + a_ih0[j]) * a.Wi + a_iw0[j];
    } else {
      a_ih0[j] = -(1 << 28);
      a_iw0[j] = 0;
      a_pix0[j] = 0;
    }
  }
  const int b_rowlen = a.ktiles_total * 64;  // bf16 per packed weight row
  int b_off[LB];
#pragma unroll
  for (int j = 0; j < LB; ++j) {
    const int r = (wv * LB + j) * 8 + lrow;
    b_off[j] = (n0 + r) * b_rowlen + (lslot ^ ((r >> 1) & 7)) * 8;
  }

  // next tile to issue: (channel block, ky, kx) walked incrementally (packed_k order)
  int i_cb, i_ky, i_kx;
  {
    const int taps = a.kh * a.kw;
    i_cb = kt_begin / taps;
    const int tap = kt_begin - i_cb * taps;
    i_ky = tap / a.kw;
    i_kx = tap - i_ky * a.kw;
  }
  int i_kt = kt_begin;
  // PF & 8: buffer addressing (buffer_load_dwordx4 ... lds).  A piece's 32-bit byte offset is its
  // row's constant part plus ONE uniform per-tap / per-channel-block term; an out-of-image tap or
  // a row past M gets an offset past the buffer's end, which the hardware reads as zeros (no zero
  // line, no 64-bit address math, no exec-masked branch per piece).  The weights' K offset goes in
  // the uniform soffset.
  __amdgpu_buffer_rsrc_t rsA, rsB, rsL;
  int a_roff[LA], b_voff[LB], l_voff[LBL > 0 ? LBL : 1];
#if defined(__HIP_DEVICE_COMPILE__)  // the buffer builtins exist for the device pass only
  if constexpr ((PF & 8) != 0) {
    const int cbl = a.Ci >> (PREC == 1 ? 6 : 5);
    const long a_bytes = (long)a.N * a.Hi * a.Wi * cbl * 128;
    rsA = __builtin_amdgcn_make_buffer_rsrc((void*)xs_b, (short)0, (int)a_bytes, 0x00020000);
    rsB = __builtin_amdgcn_make_buffer_rsrc((void*)ws_b, (short)0, (int)((long)a.Co * a.ktiles_total * 128), 0x00020000);
#pragma unroll
    for (int j = 0; j < LA; ++j) a_roff[j] = (a_pix0[j] * cbl * 64 + a_ch[j]) * 2;
#pragma unroll
    for (int j = 0; j < LB; ++j) b_voff[j] = b_off[j] * 2;
    if constexpr (PREC == 6) {
      // lo plane: piece q covers tile rows 16 q .. 16 q + 15; lane -> (row lane >> 2, LDS slot lane & 3)
      // holding 16-B chunk slot ^ ((row >> 2) & 3) (conflict-free fragment reads, see read_frags)
      rsL = __builtin_amdgcn_make_buffer_rsrc((void*)wl_b, (short)0, (int)((long)a.Co * a.ktiles_total * 64),
                                              0x00020000);
#pragma unroll
      for (int j = 0; j < LBL; ++j) {
        const int q = (wv * LBL + j) % NLO;
        const int r = q * 16 + (lane >> 2);
        l_voff[j] = (n0 + r) * a.ktiles_total * 64 + (((lane & 3) ^ ((r >> 2) & 3)) << 4);
      }
    }
  }
#endif
  auto issue = [&](int stg) {
    if (PF & 4) return;  // timing study: no operand traffic
    char* sb = smem + stg * STG_BYTES;
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr ((PF & 8) != 0) {
      const int dy = i_ky * a.dil, dx = i_kx * a.dil;
      const int uni = ((dy * a.Wi + dx) * cblocks + i_cb) * 128;
#pragma unroll
      for (int j = 0; j < LA; ++j) {
        const int ih = a_ih0[j] + dy, iw = a_iw0[j] + dx;
        const bool in = (unsigned)ih < (unsigned)a.Hi && (unsigned)iw < (unsigned)a.Wi;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (CWT_LDS void*)(sb + (wv * LA + j) * 1024), 16,
                                                 in ? a_roff[j] + uni : (int)0x80000000, 0, 0, 0);
      }
#pragma unroll
      for (int j = 0; j < LB; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (CWT_LDS void*)(sb + BM * 128 + (wv * LB + j) * 1024), 16,
                                                 b_voff[j], i_kt * 128, 0, 0);
      if constexpr (PREC == 6) {
#pragma unroll
        for (int j = 0; j < LBL; ++j)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rsL, (CWT_LDS void*)(sb + LO_OFF + ((wv * LBL + j) % NLO) * 1024), 16,
                                                   l_voff[j], i_kt * 64, 0, 0);
      }
      ++i_kt;
      if (++i_kx == a.kw) {
        i_kx = 0;
        if (++i_ky == a.kh) {
          i_ky = 0;
          ++i_cb;
        }
      }
      return;
    }
#endif
    const int dy = i_ky * a.dil, dx = i_kx * a.dil;
    const int shift = dy * a.Wi + dx;
#pragma unroll
    for (int j = 0; j < LA; ++j) {
      const int ih = a_ih0[j] + dy, iw = a_iw0[j] + dx;
      const bool in = (unsigned)ih < (unsigned)a.Hi && (unsigned)iw < (unsigned)a.Wi;
      const __bf16* src = in ? a.xs + ((a_pix0[j] + shift) * cblocks + i_cb) * 64 + a_ch[j] : a.zero;
      glds16(src, sb + (wv * LA + j) * 1024);
    }
#pragma unroll
    for (int j = 0; j < LB; ++j) glds16(a.ws + b_off[j] + i_kt * 64, sb + BM * 128 + (wv * LB + j) * 1024);
    ++i_kt;
    if (++i_kx == a.kw) {
      i_kx = 0;
      if (++i_ky == a.kh) {
        i_ky = 0;
        ++i_cb;
      }
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment read geometry: lane -> row (lane & 15) of a 16-row block, k-chunk (lane >> 4)
  const int fr = lane & 15, fk = lane >> 4;
  const int swz = (fr >> 1) & 7;
  const int off_hi = fr * 128 + ((fk ^ swz) << 4);
  const int off_lo = fr * 128 + (((4 + fk) ^ swz) << 4);
  // PREC 6: an A lane's 8 fp32 k-values are 16-B chunks 2fk and 2fk+1 (k = 8fk .. 8fk+7, the k slots
  // of its bf16 fragment and of the weights' hi / mid chunks fk, 4 + fk); conflict-free like the
  // others (rows fr, fr^1 share a swizzle but sit 128 B apart).  The lo plane's 64-B rows: chunk fk
  // of row fr sits in slot fk ^ ((fr >> 2) & 3), so a 16-lane group reads 16 distinct 16-B slots
  const int off_a0 = PREC == 6 ? fr * 128 + (((2 * fk) ^ swz) << 4) : off_hi;
  const int off_a1 = PREC == 6 ? fr * 128 + (((2 * fk + 1) ^ swz) << 4) : off_lo;
  const int off_l = fr * 64 + ((fk ^ ((fr >> 2) & 3)) << 4);
  const int a_row0 = wm * WM, b_row0 = BM + wn * WN;

  // PREC 6 without fragment prefetch: the B fragments (three pre-split terms each) are read from the
  // stage inside the MFMA loop, one fragment column at a time, after all A fragments are split --
  // the live set is FM x 3 split A terms + one B column instead of every B fragment (8 columns in
  // the WN = 128 forms); the stage is stable until the next barrier
  constexpr bool LAZY_B = PREC == 6 && (PF & 3) == 0 && FN >= 8;  // the WN = 128 forms (conv_x6.hip var 3, 5)
  struct Frags {
    bf16x8 ah[FM], al[FM], bh[LAZY_B ? 1 : FN], bl[LAZY_B ? 1 : FN];
    bf16x8 bo[PREC == 6 && !LAZY_B ? FN : 1];  // PREC 6: the weights' lo term
  };
  auto read_frags = [&](Frags& F, int stg) {
    const char* sb = smem + stg * STG_BYTES;
#pragma unroll
    for (int j = 0; j < (LAZY_B ? 0 : FN); ++j) {
      const char* p = sb + (b_row0 + j * 16) * 128;
      F.bh[j] = *(const bf16x8*)(p + off_hi);
      F.bl[j] = *(const bf16x8*)(p + off_lo);
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const char* p = sb + (a_row0 + i * 16) * 128;
      F.ah[i] = *(const bf16x8*)(p + off_a0);
      F.al[i] = *(const bf16x8*)(p + off_a1);
    }
    if constexpr (PREC == 6 && !LAZY_B) {
#pragma unroll
      for (int j = 0; j < FN; ++j) F.bo[j] = *(const bf16x8*)(sb + LO_OFF + (wn * WN + j * 16) * 64 + off_l);
    }
  };
  auto mfmas = [&](const Frags& F, int stg) {
    if (PF & 2) {  // timing study: no MFMAs (keep the fragments live)
#pragma unroll
      for (int i = 0; i < FM; ++i) asm volatile("" ::"v"(F.ah[i]), "v"(F.al[i]));
#pragma unroll
      for (int j = 0; j < (LAZY_B ? 1 : FN); ++j)
        asm volatile("" ::"v"(F.bh[j]), "v"(F.bl[j]), "v"(F.bo[j < (PREC == 6 && !LAZY_B ? FN : 1) ? j : 0]));
      return;
    }
    if constexpr (LAZY_B) {  // split every A fragment, then one B column at a time from the stage
      const char* sb = smem + stg * STG_BYTES;
      bf16x8 as[FM][3];
#pragma unroll
      for (int i = 0; i < FM; ++i)
        if constexpr ((PF & 16) != 0) {  // timing study (x6 var 12, 13): no A split, the raw bits as the terms
          as[i][0] = F.ah[i];
          as[i][1] = F.al[i];
          as[i][2] = F.ah[i];
        } else {
          split3_bf16(__builtin_bit_cast(f32x4, F.ah[i]), __builtin_bit_cast(f32x4, F.al[i]), as[i][0], as[i][1],
                      as[i][2]);
        }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const char* p = sb + (b_row0 + j * 16) * 128;
        const bf16x8 bh = *(const bf16x8*)(p + off_hi), bm = *(const bf16x8*)(p + off_lo);
        const bf16x8 bl = *(const bf16x8*)(sb + LO_OFF + (wn * WN + j * 16) * 64 + off_l);
#pragma unroll
        for (int i = 0; i < FM; ++i) {  // smallest products first
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as[i][1], bm, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as[i][2], bh, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as[i][0], bl, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as[i][1], bh, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as[i][0], bm, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as[i][0], bh, acc[i][j], 0, 0, 0);
        }
      }
    } else if constexpr (PREC == 6) {  // B: hi = bh, mid = bl, lo = bo (pre-split); A split here
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        bf16x8 ah, am, al;
        split3_bf16(__builtin_bit_cast(f32x4, F.ah[i]), __builtin_bit_cast(f32x4, F.al[i]), ah, am, al);
#pragma unroll
        for (int j = 0; j < FN; ++j) {  // smallest products first
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, F.bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, F.bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, F.bo[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, F.bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, F.bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, F.bh[j], acc[i][j], 0, 0, 0);
        }
      }
    } else {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        if (PREC == 0) {
          // exact fp32: a 16-B chunk is 4 consecutive k of one row; lane (row fr, chunk fk)
          // supplies k = 4 fk + s to MFMA s (A and B permuted alike: the k order of a sum is
          // free), 16-B chunks fk and 4 + fk cover the 32-deep tile in 8 v_mfma_f32_16x16x4_f32
          const f32x4 a0 = __builtin_bit_cast(f32x4, F.ah[i]), a1 = __builtin_bit_cast(f32x4, F.al[i]);
          const f32x4 b0 = __builtin_bit_cast(f32x4, F.bh[j]), b1 = __builtin_bit_cast(f32x4, F.bl[j]);
#pragma unroll
          for (int s = 0; s < 4; ++s) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[s], b0[s], acc[i][j], 0, 0, 0);
#pragma unroll
          for (int s = 0; s < 4; ++s) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[s], b1[s], acc[i][j], 0, 0, 0);
        } else if (PREC == 1) {  // "hi" / "lo" = first / second 32 k of the 64-deep tile
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(F.ah[i], F.bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(F.al[i], F.bl[j], acc[i][j], 0, 0, 0);
        } else {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(F.al[i], F.bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(F.ah[i], F.bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(F.ah[i], F.bh[j], acc[i][j], 0, 0, 0);
        }
      }
    }
  };

  if constexpr ((PF & 1) == 0) {
#pragma unroll
    for (int s = 0; s < NSTG - 1; ++s)
      if (s < T) issue(s);

    for (int t = 0; t < T; ++t) {
      wait_tiles<LPT>(min(NSTG - 2, T - 1 - t));
      block_sync_lds();
      if (t + NSTG - 1 < T) issue((t + NSTG - 1) % NSTG);
      Frags F;
      read_frags(F, t % NSTG);
      mfmas(F, t % NSTG);
    }
  } else {
    // prologue: tiles 0 .. NSTG-1 fill every slot; tile 0's fragments
#pragma unroll
    for (int s = 0; s < NSTG; ++s)
      if (s < T) issue(s);
    Frags F0, F1;
    if (T > 0) {
      wait_tiles<LPT>(min(NSTG - 1, T - 1));
      block_sync_lds();
      read_frags(F0, 0);
    }
    // step t: publish tile t+1 (issued: min(T, NSTG + t) tiles, so min(T-t-2, NSTG-2) may stay
    // in flight), refill tile t's slot with tile t+NSTG, read tile t+1's fragments, MFMAs of t
    auto step = [&](int t, Frags& cur, Frags& nxt) {
      if (t + 1 < T) {
        wait_tiles<LPT>(min(T - t - 2, NSTG - 2));
        block_sync_lds();
        if (t + NSTG < T) issue(t % NSTG);
        read_frags(nxt, (t + 1) % NSTG);
      }
      mfmas(cur, -1);
    };
    for (int t = 0; t < T; t += 2) {
      step(t, F0, F1);
      if (t + 1 < T) step(t + 1, F1, F0);
    }
  }

  // ---- epilogue through a per-wave LDS tile ----
  wait_vmcnt<0>();
  if constexpr ((PF & 32) != 0) {  // timing study (x6 var 17): no epilogue (the accumulators kept live)
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) asm volatile("" ::"v"(acc[i][j]));
    return;
  }
  block_sync_lds();
  float* ep = (float*)smem + wv * (EP_ROWS * EP_LD);
  constexpr int LPR = WN / 8;    // lanes per output row (8 channels each)
  constexpr int RPR = 64 / LPR;  // rows per round
  static_assert(LPR * 8 == WN && RPR * LPR == 64 && EP_ROWS % RPR == 0, "epilogue geometry");
  const int er = lane / LPR, eg = lane - er * LPR;
  const int co = n0 + wn * WN + eg * 8;
  float sc[8], sh[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    sc[i] = a.part ? 1.f : a.scale[co + i];
    sh[i] = a.part ? 0.f : a.shift[co + i];
  }
  const int fq = lane >> 4;
  constexpr int NPASS = WM / EP_ROWS, RR = EP_ROWS / RPR;
  const int mrow = m0 + wm * WM + er;  // output row of round rr of pass p: mrow + p*EP_ROWS + rr*RPR
  // residuals of pass p+1 are loaded while pass p is stored (double buffer; rows past M clamp)
  Res8 resb[2][RR];
  const bool fused = !a.part;
#pragma unroll
  for (int rr = 0; rr < RR; ++rr)
    if (fused) resb[0][rr] = load_res8<PREC>(a, min(mrow + rr * RPR, a.M - 1), co);
#pragma unroll
  for (int pass = 0; pass < NPASS; ++pass) {
#pragma unroll
    for (int fi = 0; fi < EP_ROWS / 16; ++fi)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) ep[(fi * 16 + fq * 4 + q) * EP_LD + j * 16 + fr] = acc[pass * (EP_ROWS / 16) + fi][j][q];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    f32x4 v0[RR], v1[RR];
#pragma unroll
    for (int rr = 0; rr < RR; ++rr) {
      const int r = rr * RPR + er;
      v0[rr] = *(const f32x4*)(ep + r * EP_LD + eg * 8);
      v1[rr] = *(const f32x4*)(ep + r * EP_LD + eg * 8 + 4);
    }
    if (pass + 1 < NPASS && fused) {
#pragma unroll
      for (int rr = 0; rr < RR; ++rr)
        resb[(pass + 1) & 1][rr] = load_res8<PREC>(a, min(mrow + (pass + 1) * EP_ROWS + rr * RPR, a.M - 1), co);
    }
#pragma unroll
    for (int rr = 0; rr < RR; ++rr) {
      const int m = mrow + pass * EP_ROWS + rr * RPR;
      if (m < a.M) {
        if (!fused) {
          f32x4* pp = (f32x4*)(part_b + ((long)ks * a.M + m) * a.Co + co);
          pp[0] = v0[rr];
          pp[1] = v1[rr];
        } else {
          const float v[8] = {v0[rr][0], v0[rr][1], v0[rr][2], v0[rr][3], v1[rr][0], v1[rr][1], v1[rr][2], v1[rr][3]};
          store_out8<PREC>(a, m, co, v, sc, sh, resb[pass & 1][rr]);
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}

// the automatic tile / split-K plan of a GEMM shape (conv_x3s.hip)
ConvPlan plan_heuristic_s(int M, int Co, int ktiles);
void launch_tiles_x6(int stage, const ConvSArgs& a, const ConvPlan& p, dim3 grid, hipStream_t st);
}  // namespace cwt

// Shared device/host helpers for libcwt (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace cwt {

void set_error(const std::string& msg);
int fail(int code, const std::string& msg);

#define CWT_HIP(expr)                                                                         \
  do {                                                                                        \
    hipError_t e_ = (expr);                                                                   \
    if (e_ != hipSuccess)                                                                     \
      return ::cwt::fail((int)e_, std::string(#expr " -> ") + hipGetErrorString(e_));         \
  } while (0)

#define CWT_CHECK(cond, msg)                                                                  \
  do {                                                                                        \
    if (!(cond)) return ::cwt::fail(CWT_EARG, std::string("bad argument: ") + (msg));         \
  } while (0)

#define CWT_LAUNCH_CHECK()                                                                    \
  do {                                                                                        \
    hipError_t e_ = hipGetLastError();                                                        \
    if (e_ != hipSuccess)                                                                     \
      return ::cwt::fail((int)e_, std::string("kernel launch: ") + hipGetErrorString(e_));    \
  } while (0)

static inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// DPP lane exchanges (VALU modifiers, no LDS round trip): quad_perm xor 1 / xor 2, and the
// 8- / 16-lane mirrors.  After xor1, xor2, half-mirror every lane of an aligned octet holds
// the octet's sum; a further row-mirror gives the 16-lane row sum.
template <int CTRL>
__device__ __forceinline__ float dpp_add(float v) {
  return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float octet_sum(float v) {
  return dpp_add<0x141>(dpp_add<0x4E>(dpp_add<0xB1>(v)));
}
// Full 64-lane sum, wave-uniform result: row sums by DPP, then four readlanes.
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v = dpp_add<0x140>(octet_sum(v));
  const int i = __float_as_int(v);
  return (__int_as_float(__builtin_amdgcn_readlane(i, 0)) + __int_as_float(__builtin_amdgcn_readlane(i, 16))) +
         (__int_as_float(__builtin_amdgcn_readlane(i, 32)) + __int_as_float(__builtin_amdgcn_readlane(i, 48)));
}

// Transposing 64-lane reduction of NV per-lane values v[0..NV) (NV = 64 or 32): every halving
// step pairs lanes that differ in one lane bit (bit 5: v_permlane32_swap, bit 4:
// v_permlane16_swap -- whole halves / rows exchanged, so both partners just add; bits 3, 2:
// DPP row / half-row mirror; bits 1, 0: DPP quad perms), the lane with the bit set keeping the
// upper half of the values.  Returns, summed over the 64 lanes: NV = 64 -> value L in lane L;
// NV = 32 -> value L >> 1 in lanes L (pairs).  NV reductions for the price of ~NV adds.
template <int CTRL>
__device__ __forceinline__ float dpp_get(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int NV>
__device__ __forceinline__ float butterfly_sum(float (&v)[NV], int lane) {
  static_assert(NV == 64 || NV == 32, "64 or 32 values");
  constexpr int H0 = NV / 2, H1 = H0 / 2, H2 = H1 / 2, H3 = H2 / 2;
#pragma unroll
  for (int j = 0; j < H0; ++j) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[j]), __float_as_uint(v[j + H0]), false, false);
    v[j] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
#pragma unroll
  for (int j = 0; j < H1; ++j) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[j]), __float_as_uint(v[j + H1]), false, false);
    v[j] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  {
    const bool up = (lane & 8) != 0;
#pragma unroll
    for (int j = 0; j < H2; ++j) {
      const float send = up ? v[j] : v[j + H2], keep = up ? v[j + H2] : v[j];
      v[j] = keep + dpp_get<0x140>(send);
    }
  }
  {
    const bool up = (lane & 4) != 0;
#pragma unroll
    for (int j = 0; j < H3; ++j) {
      const float send = up ? v[j] : v[j + H3], keep = up ? v[j + H3] : v[j];
      v[j] = keep + dpp_get<0x141>(send);
    }
  }
  if constexpr (NV == 64) {
    {
      const bool up = (lane & 2) != 0;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const float send = up ? v[j] : v[j + 2], keep = up ? v[j + 2] : v[j];
        v[j] = keep + dpp_get<0x4E>(send);
      }
    }
    const bool up = (lane & 1) != 0;
    const float send = up ? v[0] : v[1], keep = up ? v[1] : v[0];
    return keep + dpp_get<0xB1>(send);
  } else {
    const bool up = (lane & 2) != 0;
    const float send = up ? v[0] : v[1], keep = up ? v[1] : v[0];
    const float x = keep + dpp_get<0x4E>(send);
    return x + dpp_get<0xB1>(x);
  }
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Bilinear source coordinate, PyTorch upsample_bilinear2d(align_corners=True) CPU semantics
// (aten/src/ATen/native/UpSample.h area_pixel_compute_scale / source index): scale is a float
// (in-1)/(out-1), src = scale*dst, i0 = (int)src, i1 = i0 + (i0 < in-1), l1 = src - i0.
struct Lerp {
  int i0, i1;
  float l0, l1;
};
__device__ __forceinline__ Lerp lerp_coord(int dst, int in_size, float scale) {
  Lerp r;
  float src = scale * (float)dst;
  r.i0 = (int)src;
  r.i1 = r.i0 + ((r.i0 < in_size - 1) ? 1 : 0);
  r.l1 = src - (float)r.i0;
  r.l0 = 1.0f - r.l1;
  return r;
}
__host__ __device__ static inline float align_corners_scale(int in_size, int out_size) {
  return out_size > 1 ? (float)(in_size - 1) / (float)(out_size - 1) : 0.0f;
}

// Counter-based dropout draw (the CWT's training-mode dropouts): a splitmix64 finaliser of
// (seed, stream, index) -> u in [0, 1) with 24 random bits; an element is kept iff u >= p and
// then scaled by 1 / (1 - p), as nn.Dropout does.  The same function regenerates the mask in the
// backward pass (nothing is stored) and in the tests (tests/dropout_ref.py restates it).
// Streams: 1 = attention probabilities [B][2H][hw], 2 = fc output [2B][512].
__host__ __device__ __forceinline__ float dropout_uniform(unsigned long long seed, unsigned stream,
                                                         unsigned long long idx) {
  unsigned long long z = seed + 0x9E3779B97F4A7C15ull * (idx + 1) + 0xD1B54A32D192ED03ull * (stream + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (float)(z >> 40) * (1.0f / 16777216.0f);
}
__host__ __device__ __forceinline__ float dropout_scale(float p, unsigned long long seed, unsigned stream,
                                                       unsigned long long idx) {
  return dropout_uniform(seed, stream, idx) >= p ? 1.0f / (1.0f - p) : 0.0f;
}

}  // namespace cwt

#ifndef CWT_EARG
#define CWT_EARG 1001
#define CWT_ESTATE 1002
#define CWT_ENOFG 1003
#endif

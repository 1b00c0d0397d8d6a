// DeTr head of the transformer variants (src/model/detr.py:13-151),
// forward only, on tokens [B][hw][C] (channels last):
//  * linear epilogue: bias, ReLU and an accumulated second product after the exact-fp32 GEMM
//    (launch_gemm_abt), for nn.Linear / 1x1 nn.Conv2d (detr.py:22, ms_deform_attn.py:56-59);
//  * the sine position embedding of SinePositionalEncoding(256, normalize=True)
//    (positional_encoding.py:44-74) added to the query tokens (detr.py:94);
//  * the deformable attention core: per (query, head) a softmax over the n_points attention
//    logits, sampling locations reference + offset / (W, H), and the bilinear grid_sample
//    (align_corners False, zero padding) of the head's value channels at each of them, summed
//    with the attention weights (ms_deform_attn.py:84-117, ms_deform_attn_func.py:41-61), one
//    level (DeformAtt n_levels = 1, detr.py:32,78-110);
//  * the blend F.normalize(a) + F.normalize(b) * att_wt (detr.py:41,45).
#include "common.h"
#include "kernels.h"

namespace cwt {

// out[p][n] = act(tmp[p][n] + bias[n] (+ acc[p][n]))
__global__ void linear_epilogue_kernel(const float* __restrict__ tmp, const float* __restrict__ bias,
                                       const float* __restrict__ acc, long total, int N, int relu,
                                       float* __restrict__ out) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    float v = tmp[i];
    if (acc) v = acc[i] + v;
    if (bias) v += bias[i % N];
    out[i] = relu ? fmaxf(v, 0.f) : v;
  }
}

int launch_linear_epilogue(const float* tmp, const float* bias, const float* acc, long P, int N, int relu, float* out,
                           hipStream_t st) {
  const long total = P * N;
  hipLaunchKernelGGL(linear_epilogue_kernel, dim3((unsigned)std::min<long>(4096, cdiv(total, 256))), dim3(256), 0, st,
                     tmp, bias, acc, total, N, relu, out);
  CWT_LAUNCH_CHECK();
  return 0;
}

// x + pos for SinePositionalEncoding(num_feats = C/2, temperature, normalize, scale, eps) of
// the mask DeformAtt passes (detr.py:135: torch.zeros(...).long(), so ~mask is -1 everywhere):
// y_embed = cumsum over rows of -1 = -(i + 1), x_embed = -(j + 1); normalize divides by the last
// row / column plus eps, in fp32 as the reference does.  Channel c < C/2: the y part, k = c;
// c >= C/2: the x part, k = c - C/2; dim_t[k] = temperature^(2 (k / 2) / num_feats); even k sin,
// odd k cos (the stack + flatten interleave).  One thread per (token, channel).
__global__ void sine_pos_add_kernel(const float* __restrict__ x, int B, int h, int w, int C, float temperature,
                                    int normalize, float scale, float eps, float* __restrict__ out) {
#pragma clang fp contract(off)
  const int nf = C / 2;
  const long total = (long)B * h * w * C;
  for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int c = (int)(idx % C);
    const long pix = idx / C;
    const int j = (int)(pix % w);
    const int i = (int)((pix / w) % h);
    const bool ypart = c < nf;
    const int k = ypart ? c : c - nf;
    float e = ypart ? -(float)(i + 1) : -(float)(j + 1);
    if (normalize) {
      const float last = ypart ? -(float)h : -(float)w;
      e = e / (last + eps) * scale;
    }
    const float dt = powf(temperature, (2.f * (float)(k / 2)) / (float)nf);
    const float a = e / dt;
    const float pv = (k & 1) ? cosf(a) : sinf(a);
    out[idx] = x[idx] + pv;
  }
}

int launch_sine_pos_add(const float* x, int B, int h, int w, int C, float temperature, int normalize, float scale,
                        float eps, float* out, hipStream_t st) {
  const long total = (long)B * h * w * C;
  hipLaunchKernelGGL(sine_pos_add_kernel, dim3((unsigned)std::min<long>(4096, cdiv(total, 256))), dim3(256), 0, st, x,
                     B, h, w, C, temperature, normalize, scale, eps, out);
  CWT_LAUNCH_CHECK();
  return 0;
}

// One wave per (batch, query, head); lane d < D holds value channel head*D + d.  The offsets and
// logits of the (query, head) are wave-uniform loads.  grid_sample's source index (align_corners
// False): ix = ((g + 1) W - 1) / 2 with g = 2 loc - 1, loc = ref + off / W, ref = (j + 0.5) / W,
// evaluated in that order (fp contraction off); corners outside the map contribute 0.
constexpr int DA_MAXP = 16;
__global__ __launch_bounds__(256) void deform_attn_kernel(const float* __restrict__ value,
                                                          const float* __restrict__ offsets,
                                                          const float* __restrict__ logits, int B, int H, int W,
                                                          int M, int P, int D, float* __restrict__ out) {
#pragma clang fp contract(off)
  const int lane = threadIdx.x & 63;
  const long L = (long)H * W;
  const long nw = (long)B * L * M;
  const long wid = (long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (wid >= nw) return;
  const int m = (int)(wid % M);
  const long bq = wid / M;
  const int q = (int)(bq % L);
  const int b = (int)(bq / L);
  const int qy = q / W, qx = q - qy * W;
  const float* lg = logits + (bq * M + m) * P;
  const float* of = offsets + (bq * M + m) * P * 2;
  float mx = -INFINITY;
  for (int p = 0; p < P; ++p) mx = fmaxf(mx, lg[p]);
  float s = 0.f;
  for (int p = 0; p < P; ++p) s += expf(lg[p] - mx);
  const float ref_x = ((float)qx + 0.5f) / (float)W, ref_y = ((float)qy + 0.5f) / (float)H;
  const float* vb = value + (long)b * L * (M * D) + m * D + lane;
  const bool act = lane < D;
  float acc = 0.f;
  for (int p = 0; p < P; ++p) {
    const float lx = ref_x + of[2 * p] / (float)W, ly = ref_y + of[2 * p + 1] / (float)H;
    const float gx = 2.f * lx - 1.f, gy = 2.f * ly - 1.f;
    const float ix = ((gx + 1.f) * (float)W - 1.f) / 2.f, iy = ((gy + 1.f) * (float)H - 1.f) / 2.f;
    const float fx = floorf(ix), fy = floorf(iy);
    const int x0 = (int)fx, y0 = (int)fy, x1 = x0 + 1, y1 = y0 + 1;
    const float wx1 = ix - fx, wx0 = (fx + 1.f) - ix, wy1 = iy - fy, wy0 = (fy + 1.f) - iy;
    const float w00 = wx0 * wy0, w01 = wx1 * wy0, w10 = wx0 * wy1, w11 = wx1 * wy1;  // nw, ne, sw, se
    float v = 0.f;
    if (act) {
      if ((unsigned)y0 < (unsigned)H && (unsigned)x0 < (unsigned)W) v += vb[((long)y0 * W + x0) * (M * D)] * w00;
      if ((unsigned)y0 < (unsigned)H && (unsigned)x1 < (unsigned)W) v += vb[((long)y0 * W + x1) * (M * D)] * w01;
      if ((unsigned)y1 < (unsigned)H && (unsigned)x0 < (unsigned)W) v += vb[((long)y1 * W + x0) * (M * D)] * w10;
      if ((unsigned)y1 < (unsigned)H && (unsigned)x1 < (unsigned)W) v += vb[((long)y1 * W + x1) * (M * D)] * w11;
    }
    acc += v * (expf(lg[p] - mx) / s);
  }
  if (act) out[bq * (M * D) + m * D + lane] = acc;
}

int launch_deform_attn(const float* value, const float* offsets, const float* logits, int B, int H, int W, int M,
                       int P, int D, float* out, hipStream_t st) {
  if (P > DA_MAXP || D > 64) return fail(CWT_EARG, "deform_attn: n_points <= 16 and d_model / n_heads <= 64");
  const long nw = (long)B * H * W * M;
  hipLaunchKernelGGL(deform_attn_kernel, dim3((unsigned)cdiv(nw, 4)), dim3(256), 0, st, value, offsets, logits, B, H,
                     W, M, P, D, out);
  CWT_LAUNCH_CHECK();
  return 0;
}

// Backward of deform_attn_kernel (ms_deform_attn.py:99-117 under autograd; the reference's CUDA
// op backpropagates the same quantities), one wave per (batch, query, head) as the forward:
//   v_p = bilinear(value, ix_p, iy_p), a = softmax(logits), out = sum_p a_p v_p;
//   d a_p = <d_out, v_p>, d logits_p = a_p (d a_p - sum_q a_q d a_q),
//   d offset_p = a_p <d_out, dv_p / d(ix, iy)> (ix = loc W - 1/2 and loc = ref + off / W, so
//   d ix / d off_x = 1; zero-padded corners carry no value and no slope),
//   d value[corner] += w_corner a_p d_out.  One value position is sampled by many queries (the
//   reference's CUDA backward scatters with float atomics, whose sum order -- and so result --
//   changes from run to run); here every contribution is rounded once to a 64-bit fixed-point
//   integer, rint(c 2^sh) with 2^sh chosen from max|d_out| so no sum can overflow (|c| <= |d_out|,
//   at most H W P contributions per position), and added with integer atomics, which are exactly
//   associative: the result is deterministic, within 2^-sh per contribution (~2^-45 max|d_out| at
//   60^2 positions and 4 points) of the exact sum.  dv64 must be zeroed first;
//   deform_attn_dv_finish_kernel converts it back.
__global__ void absmax_bits_kernel(const float* __restrict__ x, long n, unsigned* __restrict__ out) {
  float m = 0.f;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float v = fabsf(x[i]);
    if (v <= 3.4028235e38f) m = fmaxf(m, v);  // finite values only (NaN / Inf take the float path below)
  }
  for (int o = 32; o; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) atomicMax(out, __float_as_uint(m));  // order-free: deterministic
}

__device__ __forceinline__ double dv_scale(const unsigned* gmax_bits, int headroom) {
  const float gm = __uint_as_float(*gmax_bits);
  const int e = gm > 0.f ? ilogbf(gm) : 0;  // |c| < 2^(e+1)
  return ldexp(1.0, 62 - headroom - (e + 1));
}

__global__ __launch_bounds__(256) void deform_attn_bwd_kernel(const float* __restrict__ value,
                                                              const float* __restrict__ offsets,
                                                              const float* __restrict__ logits, int B, int H, int W,
                                                              int M, int P, int D, const float* __restrict__ d_out,
                                                              unsigned long long* dv64, const unsigned* gmax_bits,
                                                              int headroom, float* d_value, float* __restrict__ d_offsets,
                                                              float* __restrict__ d_logits) {
#pragma clang fp contract(off)
  const int lane = threadIdx.x & 63;
  const long L = (long)H * W;
  const long nw = (long)B * L * M;
  const long wid = (long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (wid >= nw) return;
  const int m = (int)(wid % M);
  const long bq = wid / M;
  const int q = (int)(bq % L);
  const int b = (int)(bq / L);
  const int qy = q / W, qx = q - qy * W;
  const float* lg = logits + (bq * M + m) * P;
  const float* of = offsets + (bq * M + m) * P * 2;
  float mx = -INFINITY;
  for (int p = 0; p < P; ++p) mx = fmaxf(mx, lg[p]);
  float s = 0.f;
  for (int p = 0; p < P; ++p) s += expf(lg[p] - mx);
  const float ref_x = ((float)qx + 0.5f) / (float)W, ref_y = ((float)qy + 0.5f) / (float)H;
  const long vs = (long)M * D;
  const float* vb = value + (long)b * L * vs + m * D + lane;
  unsigned long long* dvb = dv64 + (long)b * L * vs + m * D + lane;
  float* dvf = d_value + (long)b * L * vs + m * D + lane;
  const double S = dv_scale(gmax_bits, headroom);
  const bool act = lane < D;
  const float g = act ? d_out[bq * vs + m * D + lane] : 0.f;
  float da[DA_MAXP], dox[DA_MAXP], doy[DA_MAXP], ap[DA_MAXP];
  float sad = 0.f;
  for (int p = 0; p < P; ++p) {
    const float a = expf(lg[p] - mx) / s;
    const float lx = ref_x + of[2 * p] / (float)W, ly = ref_y + of[2 * p + 1] / (float)H;
    const float gx = 2.f * lx - 1.f, gy = 2.f * ly - 1.f;
    const float ix = ((gx + 1.f) * (float)W - 1.f) / 2.f, iy = ((gy + 1.f) * (float)H - 1.f) / 2.f;
    const float fx = floorf(ix), fy = floorf(iy);
    const int x0 = (int)fx, y0 = (int)fy, x1 = x0 + 1, y1 = y0 + 1;
    const float wx1 = ix - fx, wx0 = (fx + 1.f) - ix, wy1 = iy - fy, wy0 = (fy + 1.f) - iy;
    const float w00 = wx0 * wy0, w01 = wx1 * wy0, w10 = wx0 * wy1, w11 = wx1 * wy1;
    const bool i00 = act && (unsigned)y0 < (unsigned)H && (unsigned)x0 < (unsigned)W;
    const bool i01 = act && (unsigned)y0 < (unsigned)H && (unsigned)x1 < (unsigned)W;
    const bool i10 = act && (unsigned)y1 < (unsigned)H && (unsigned)x0 < (unsigned)W;
    const bool i11 = act && (unsigned)y1 < (unsigned)H && (unsigned)x1 < (unsigned)W;
    const float v00 = i00 ? vb[((long)y0 * W + x0) * vs] : 0.f, v01 = i01 ? vb[((long)y0 * W + x1) * vs] : 0.f;
    const float v10 = i10 ? vb[((long)y1 * W + x0) * vs] : 0.f, v11 = i11 ? vb[((long)y1 * W + x1) * vs] : 0.f;
    float v = 0.f;
    v += v00 * w00;
    v += v01 * w01;
    v += v10 * w10;
    v += v11 * w11;
    const float dvx = wy0 * (v01 - v00) + wy1 * (v11 - v10), dvy = wx0 * (v10 - v00) + wx1 * (v11 - v01);
    da[p] = wave_sum_dpp(g * v);
    dox[p] = a * wave_sum_dpp(g * dvx);
    doy[p] = a * wave_sum_dpp(g * dvy);
    ap[p] = a;
    sad += a * da[p];
    const float gv = a * g;
    // a non-finite contribution (NaN / Inf in d_out or the logits) goes to d_value itself as a float
    // atomic, as the reference's CUDA op adds it, so it propagates to exactly the positions it reaches;
    // the finish kernel adds the fixed-point sum to it (0 elsewhere)
    auto add = [&](long pos, float c) {
      if (fabsf(c) <= 3.4028235e38f)
        atomicAdd(&dvb[pos], (unsigned long long)(long long)rint((double)c * S));
      else
        atomicAdd(&dvf[pos], c);
    };
    if (i00) add(((long)y0 * W + x0) * vs, w00 * gv);
    if (i01) add(((long)y0 * W + x1) * vs, w01 * gv);
    if (i10) add(((long)y1 * W + x0) * vs, w10 * gv);
    if (i11) add(((long)y1 * W + x1) * vs, w11 * gv);
  }
  if (lane == 0) {
    float* dl = d_logits + (bq * M + m) * P;
    float* dof = d_offsets + (bq * M + m) * P * 2;
    for (int p = 0; p < P; ++p) {
      dl[p] = ap[p] * (da[p] - sad);
      dof[2 * p] = dox[p];
      dof[2 * p + 1] = doy[p];
    }
  }
}

__global__ void deform_attn_dv_finish_kernel(const unsigned long long* __restrict__ dv64, long n,
                                             const unsigned* __restrict__ gmax_bits, int headroom,
                                             float* __restrict__ d_value) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  d_value[i] += (float)((double)(long long)dv64[i] / dv_scale(gmax_bits, headroom));  // + the non-finite part
}

size_t deform_attn_bwd_ws_bytes(int B, int H, int W, int M, int D) { return 256 + (size_t)B * H * W * M * D * 8; }

// ws: deform_attn_bwd_ws_bytes bytes of device scratch
int launch_deform_attn_bwd(const float* value, const float* offsets, const float* logits, int B, int H, int W, int M,
                           int P, int D, const float* d_out, float* d_value, float* d_offsets, float* d_logits,
                           void* ws, hipStream_t st) {
  if (P > DA_MAXP || D > 64) return fail(CWT_EARG, "deform_attn: n_points <= 16 and d_model / n_heads <= 64");
  const long nw = (long)B * H * W * M;
  const long n = nw * D;
  unsigned* gmax = (unsigned*)ws;
  unsigned long long* dv64 = (unsigned long long*)((char*)ws + 256);
  int headroom = 1;  // bits for the number of contributions per position (<= H W P) and the sign
  while ((1L << headroom) < (long)H * W * P * 2) ++headroom;
  if (hipMemsetAsync(ws, 0, 256 + (size_t)n * 8, st) != hipSuccess ||
      hipMemsetAsync(d_value, 0, (size_t)n * 4, st) != hipSuccess)
    return fail(CWT_ESTATE, "deform_attn_bwd: memset");
  hipLaunchKernelGGL(absmax_bits_kernel, dim3((unsigned)std::min<long>(1024, cdiv(n, 256))), dim3(256), 0, st, d_out, n,
                     gmax);
  CWT_LAUNCH_CHECK();
  hipLaunchKernelGGL(deform_attn_bwd_kernel, dim3((unsigned)cdiv(nw, 4)), dim3(256), 0, st, value, offsets, logits, B, H,
                     W, M, P, D, d_out, dv64, (const unsigned*)gmax, headroom, d_value, d_offsets, d_logits);
  CWT_LAUNCH_CHECK();
  hipLaunchKernelGGL(deform_attn_dv_finish_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, st,
                     (const unsigned long long*)dv64, n, (const unsigned*)gmax, headroom, d_value);
  CWT_LAUNCH_CHECK();
  return 0;
}

// norm_blend's backward: d_a = (d - a_hat (a_hat . d)) / |a| (d / eps where |a| <= eps), d_b the
// same for b scaled by wt; one wave per token
__global__ __launch_bounds__(256) void norm_blend_bwd_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                             const float* __restrict__ d, long T, int C, float wt,
                                                             float* __restrict__ d_a, float* __restrict__ d_b) {
  const float eps = 1e-12f;
  const int lane = threadIdx.x & 63;
  for (long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6); r < T; r += (long)gridDim.x * 4) {
    const float* ar = a + r * C;
    const float* br = b + r * C;
    const float* dr = d + r * C;
    float sa = 0.f, sb = 0.f, pa = 0.f, pb = 0.f;
    for (int c = lane; c < C; c += 64) {
      sa = fmaf(ar[c], ar[c], sa);
      sb = fmaf(br[c], br[c], sb);
      pa = fmaf(ar[c], dr[c], pa);
      pb = fmaf(br[c], dr[c], pb);
    }
    const float na = sqrtf(wave_sum_dpp(sa)), nb = sqrtf(wave_sum_dpp(sb));
    pa = wave_sum_dpp(pa);
    pb = wave_sum_dpp(pb);
    for (int c = lane; c < C; c += 64) {
      if (d_a) d_a[r * C + c] = na > eps ? (dr[c] - (ar[c] / na) * (pa / na)) / na : dr[c] / eps;
      if (d_b) d_b[r * C + c] = wt * (nb > eps ? (dr[c] - (br[c] / nb) * (pb / nb)) / nb : dr[c] / eps);
    }
  }
}

int launch_norm_blend_bwd(const float* a, const float* b, const float* d, long T, int C, float wt, float* d_a,
                          float* d_b, hipStream_t st) {
  hipLaunchKernelGGL(norm_blend_bwd_kernel, dim3((unsigned)std::min<long>(2048, (T + 3) / 4)), dim3(256), 0, st, a, b, d,
                     T, C, wt, d_a, d_b);
  CWT_LAUNCH_CHECK();
  return 0;
}

// dst[r][c] = src[r][c] (row strides lds / ldd)
__global__ void copy_2d_kernel(const float* __restrict__ src, long R, int Cc, long lds, float* __restrict__ dst,
                               long ldd) {
  const long total = R * Cc;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long r = i / Cc;
    const int c = (int)(i - r * Cc);
    dst[r * ldd + c] = src[r * lds + c];
  }
}

int launch_copy_2d(const float* src, long R, int Cc, long lds, float* dst, long ldd, hipStream_t st) {
  hipLaunchKernelGGL(copy_2d_kernel, dim3((unsigned)std::min<long>(65536, cdiv(R * Cc, 256))), dim3(256), 0, st, src, R,
                     Cc, lds, dst, ldd);
  CWT_LAUNCH_CHECK();
  return 0;
}

// out[t] = a[t] / max(|a[t]|, 1e-12) + b[t] / max(|b[t]|, 1e-12) * wt, one wave per token
__global__ __launch_bounds__(256) void norm_blend_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                         long T, int C, float wt, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  for (long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6); r < T; r += (long)gridDim.x * 4) {
    const float* ar = a + r * C;
    const float* br = b + r * C;
    float sa = 0.f, sb = 0.f;
    for (int c = lane; c < C; c += 64) {
      sa = fmaf(ar[c], ar[c], sa);
      sb = fmaf(br[c], br[c], sb);
    }
    const float na = fmaxf(sqrtf(wave_sum_dpp(sa)), 1e-12f), nb = fmaxf(sqrtf(wave_sum_dpp(sb)), 1e-12f);
    for (int c = lane; c < C; c += 64) out[r * C + c] = ar[c] / na + br[c] / nb * wt;
  }
}

int launch_norm_blend(const float* a, const float* b, long T, int C, float wt, float* out, hipStream_t st) {
  hipLaunchKernelGGL(norm_blend_kernel, dim3((unsigned)std::min<long>(2048, (T + 3) / 4)), dim3(256), 0, st, a, b, T, C,
                     wt, out);
  CWT_LAUNCH_CHECK();
  return 0;
}

}  // namespace cwt

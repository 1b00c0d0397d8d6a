// Episode preprocessing on the device (the loader's transforms):
// transform.py Resize (aspect-preserving, both sides floored to a multiple of 8, top-left
// placement, pad 0 / mean*255 for the image and 255 for the label), ToTensor (/255) and
// Normalize ((x - mean) / std), plus the episode label remap of dataset.py:222-228,261-266
// (chosen class -> 1, 255 kept, everything else 0) and the optional hor/vert flips of the
// training augmentations (applied to the source, as cv2.flip before the resize).
//
// cv2.resize semantics restated (OpenCV resize.cpp, no cv2 in this image -- parity unpinned
// against cv2 itself, pinned against oracle/data_oracle.py):
//   INTER_LINEAR, float32 source: scale = src / dst (double); fx = (float)((dx + 0.5) * scale
//   - 0.5); sx = floor(fx); fx -= sx; sx < 0 -> (sx, fx) = (0, 0); sx >= src - 1 ->
//   (sx, fx) = (src - 1, 0); weights (1 - fx, fx); horizontal pass per source row, then the
//   vertical blend of the two rows, each as two products and one sum in fp32.
//   INTER_NEAREST: sx = min(floor(dx * scale), src - 1).
// One thread per destination pixel; the S x S outputs are written coalesced (NCHW planes).
#include "common.h"
#include "kernels.h"

// every product and sum of this file rounds on its own, as plain C / numpy evaluate them
// (-ffp-contract=fast would fuse them; the __f*_rn helpers do not help: they are inline
// operators compiled under the header's contraction state)
#pragma clang fp contract(off)

namespace cwt {

struct LinTap {
  int i0, i1;
  float w0, w1;
};

__device__ __forceinline__ LinTap cv2_linear_tap(int d, double scale, int src) {
  float f = (float)(((double)d + 0.5) * scale - 0.5);
  int s = (int)floorf(f);
  f -= (float)s;
  if (s < 0) {
    s = 0;
    f = 0.f;
  }
  if (s >= src - 1) {
    s = src - 1;
    f = 0.f;
  }
  LinTap t;
  t.i0 = s;
  t.i1 = min(s + 1, src - 1);
  t.w0 = 1.f - f;
  t.w1 = f;
  return t;
}

template <typename T>
__device__ __forceinline__ float ld_px(const T* src, int W, int y, int x, int c) {
  return (float)src[((long)y * W + x) * 3 + c];
}

// src: device HWC RGB (uint8 or fp32) H x W; dst: [3][S][S] fp32.  new_h / new_w: the Resize
// target (find_new_hw); pixels outside it take pad[c].
template <typename T>
__global__ __launch_bounds__(256) void episode_image_kernel(const T* __restrict__ src, int H, int W, int new_h,
                                                            int new_w, int S, double sy, double sx, int flip_h,
                                                            int flip_v, float m0, float m1, float m2, float s0,
                                                            float s1, float s2, float p0, float p1, float p2,
                                                            float* __restrict__ dst) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  const int y = blockIdx.y;
  if (x >= S) return;
  const float mean[3] = {m0, m1, m2}, stdv[3] = {s0, s1, s2}, pad[3] = {p0, p1, p2};
  float v[3];
  if (y < new_h && x < new_w) {
    const LinTap ty = cv2_linear_tap(y, sy, H), tx = cv2_linear_tap(x, sx, W);
    // flips act on the source (cv2.flip before the resize)
    const int y0 = flip_v ? H - 1 - ty.i0 : ty.i0, y1 = flip_v ? H - 1 - ty.i1 : ty.i1;
    const int x0 = flip_h ? W - 1 - tx.i0 : tx.i0, x1 = flip_h ? W - 1 - tx.i1 : tx.i1;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float r0 = ld_px(src, W, y0, x0, c) * tx.w0 + ld_px(src, W, y0, x1, c) * tx.w1;
      const float r1 = ld_px(src, W, y1, x0, c) * tx.w0 + ld_px(src, W, y1, x1, c) * tx.w1;
      v[c] = r0 * ty.w0 + r1 * ty.w1;
    }
  } else {
#pragma unroll
    for (int c = 0; c < 3; ++c) v[c] = pad[c];
  }
#pragma unroll
  for (int c = 0; c < 3; ++c)
    dst[((long)c * S + y) * S + x] = (v[c] / 255.f - mean[c]) / stdv[c];
}

// src: device uint8 H x W label; dst: int64 [S][S].  Remap, nearest resize, pad 255.
__global__ __launch_bounds__(256) void episode_label_kernel(const unsigned char* __restrict__ src, int H, int W,
                                                            int new_h, int new_w, int S, double sy, double sx,
                                                            int flip_h, int flip_v, int cls,
                                                            long long* __restrict__ dst) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  const int y = blockIdx.y;
  if (x >= S) return;
  long long out = 255;
  if (y < new_h && x < new_w) {
    int iy = min((int)floor(y * sy), H - 1), ix = min((int)floor(x * sx), W - 1);
    if (flip_v) iy = H - 1 - iy;
    if (flip_h) ix = W - 1 - ix;
    const int v = src[(long)iy * W + ix];
    out = v == 255 ? 255 : (cls < 0 ? v : (v == cls ? 1 : 0));
  }
  dst[(long)y * S + x] = out;
}

// transform.py Resize.find_new_hw: the longer side -> S, the other scaled by int(), then both
// floored to a multiple of 8
void find_new_hw(int h, int w, int S, int* nh, int* nw) {
  int new_h, new_w;
  if (h >= w) {
    const double ratio = S * 1.0 / h;
    new_h = S;
    new_w = (int)(w * ratio);
  } else {
    const double ratio = S * 1.0 / w;
    new_h = (int)(h * ratio);
    new_w = S;
  }
  if (new_h % 8 != 0) new_h = (new_h / 8) * 8;
  if (new_w % 8 != 0) new_w = (new_w / 8) * 8;
  *nh = new_h;
  *nw = new_w;
}

int launch_episode_image(const void* src, int src_f32, int H, int W, int S, const float* mean, const float* stdv,
                         const float* pad, int flip_h, int flip_v, float* dst, hipStream_t st) {
  int nh, nw;
  find_new_hw(H, W, S, &nh, &nw);
  if (nh < 1 || nw < 1) return fail(CWT_EARG, "preprocess: image too thin for the Resize target");
  // cv2: inv_scale = dsize / ssize, scale = 1 / inv_scale (double)
  const float p[3] = {pad ? pad[0] : 0.f, pad ? pad[1] : 0.f, pad ? pad[2] : 0.f};
  const dim3 grid(cdiv(S, 256), S);
  if (src_f32)
    hipLaunchKernelGGL(episode_image_kernel<float>, grid, dim3(256), 0, st, (const float*)src, H, W, nh, nw, S,
                       1.0 / ((double)nh / H), 1.0 / ((double)nw / W), flip_h, flip_v, mean[0], mean[1], mean[2],
                       stdv[0], stdv[1], stdv[2], p[0], p[1], p[2], dst);
  else
    hipLaunchKernelGGL(episode_image_kernel<unsigned char>, grid, dim3(256), 0, st, (const unsigned char*)src, H, W,
                       nh, nw, S, 1.0 / ((double)nh / H), 1.0 / ((double)nw / W), flip_h, flip_v, mean[0], mean[1],
                       mean[2], stdv[0], stdv[1], stdv[2], p[0], p[1], p[2], dst);
  CWT_LAUNCH_CHECK();
  return 0;
}

int launch_episode_label(const unsigned char* src, int H, int W, int S, int cls, int flip_h, int flip_v,
                         long long* dst, hipStream_t st) {
  int nh, nw;
  find_new_hw(H, W, S, &nh, &nw);
  if (nh < 1 || nw < 1) return fail(CWT_EARG, "preprocess: label too thin for the Resize target");
  const dim3 grid(cdiv(S, 256), S);
  hipLaunchKernelGGL(episode_label_kernel, grid, dim3(256), 0, st, src, H, W, nh, nw, S, 1.0 / ((double)nh / H),
                     1.0 / ((double)nw / W), flip_h, flip_v, cls, dst);
  CWT_LAUNCH_CHECK();
  return 0;
}

}  // namespace cwt

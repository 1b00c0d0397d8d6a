// Kernel-side argument structs and launcher declarations shared by the .hip units.
#pragma once
#include <vector>

#include "common.h"

namespace cwt {

struct ConvArgs {
  const float* x;      // NHWC input, pixel stride x_ld floats
  const float* w;      // packed [Co][K], K = kh*kw*Ci (tap-major)
  const float* scale;  // [Co] folded BN scale
  const float* shift;  // [Co] folded BN shift
  const float* res;    // optional residual, NHWC, pixel stride res_ld
  float* y;            // output NHWC, pixel stride y_ld, channel offset y_off
  float* part;         // split-K partials [nsplit][M][Co] (set by launch_conv)
  int N, Hi, Wi, Ci, x_ld;
  int Ho, Wo, Co, kh, kw, stride, pad, dil;
  int M, K, ktiles, kt_per_split;
  int y_ld, y_off, res_ld;
  int relu;
};

// Conv on split activations (conv_x3s.hip): input and weights in the S-layout
// [row][C/32][hi 32 | lo 32] bf16; output fp32 NHWC and/or S-layout.
struct ConvSArgs {
  const __bf16* xs;     // input, S-layout [N*Hi*Wi][Ci/32][64]
  const __bf16* ws;     // weights, S-layout [Co][K/32][64] (K in packed_k order)
  const __bf16* ws_lo;  // x6 (prec 6): the weights' lo plane [Co][K/32][32] (ws holds hi | mid)
  const __bf16* zero;   // >= 128 B of zeros (padding taps, rows past M)
  const float* scale;   // [Co] folded BN scale
  const float* shift;   // [Co] folded BN shift
  const float* res;     // optional fp32 residual NHWC, pixel stride res_ld
  const __bf16* res_s;  // optional S-layout residual [M][Co/32][64]
  float* y;             // optional fp32 output NHWC, pixel stride y_ld, channel offset y_off
  __bf16* ys;           // optional S-layout output [M][Co/32][64]
  float* part;          // split-K partials [nsplit][M][Co] (set by launch_conv_x3s)
  int N, Hi, Wi, Ci;
  int Ho, Wo, Co, kh, kw, stride, pad, dil;
  int M, K, ktiles, ktiles_total, kt_per_split;
  int y_ld, y_off, res_ld;
  int relu;
  // batched GEMMs (x6 only; the Winograd path's 16 products): grid.z = batch, GEMM b reads
  // xs + b * xs_bstride BYTES, ws / ws_lo + b * ws_bstride / wl_bstride elements and writes its raw
  // sums to part + b * M * Co (no epilogue); batch <= 1: off
  int batch;
  long xs_bstride, ws_bstride, wl_bstride;
};

// Conv weights are packed [Co][K] with K ordered (32-channel block, tap, channel in block):
// a 3x3 conv's workgroup walks its 9 taps over one 32-channel slab of its input window
// before the next slab, so the slab (~40 KB for 256 output pixels) is re-read from L1/L2
// 9 times back to back instead of once per pass over all channels (an L2-missing
// 9-fold re-stream of the window).  For 1x1 convs this is the plain channel order.
__host__ __device__ __forceinline__ long packed_k(int ci, int tap, int taps) {
  return (long)(ci >> 5) * (taps * 32) + tap * 32 + (ci & 31);
}
// The same with 64-channel blocks: the K order of the plain-bf16 conv (one 128-B line = 64 k).
__host__ __device__ __forceinline__ long packed_k64(int ci, int tap, int taps) {
  return (long)(ci >> 6) * (taps * 64) + tap * 64 + (ci & 63);
}

// Tile of this workgroup.  Blocks b and b+8 are observed to land on the same XCD (speed
// only, MI355X_MICROARCH.md §Workgroup dispatch); the linear block id is remapped so that
// each XCD gets one contiguous run of (split, m-tile, n-tile) with n fastest: its
// workgroups share A rows across n-tiles and B columns across m-tiles in their L2.
__device__ __forceinline__ void conv_tile_coords(int& mt, int& nt, int& ks) {
  const int T = gridDim.x * gridDim.y * gridDim.z;
  const int lin = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  const int q = T >> 3, r = T & 7;
  const int xcd = lin & 7, slot = lin >> 3;
  const int L = (xcd < r) ? xcd * (q + 1) + slot : r * (q + 1) + (xcd - r) * q + slot;
  nt = L % gridDim.y;
  const int rest = L / gridDim.y;
  mt = rest % gridDim.x;
  ks = rest / gridDim.x;
}

// Epilogue of one 32x32 MFMA accumulator fragment of the implicit-GEMM conv (C/D layout:
// col = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5)): BN scale/shift, residual, ReLU, or
// the raw split-K partial.  All 16 residual loads are issued (at clamped, always-valid
// addresses) before the first store: res and y are not known not to alias, so loads
// interleaved with stores would each wait a full memory round trip.
__device__ __forceinline__ void conv_store_fragment(const ConvArgs& a, const f32x16& acc, int mbase, int co, int h,
                                                    int ks, float sc, float sh) {
  if (a.part) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = mbase + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (m < a.M) a.part[((long)ks * a.M + m) * a.Co + co] = acc[r];
    }
    return;
  }
  float rv[16];
  if (a.res) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = min(mbase + (r & 3) + 8 * (r >> 2) + 4 * h, a.M - 1);
      rv[r] = a.res[(long)m * a.res_ld + co];
    }
  } else {
#pragma unroll
    for (int r = 0; r < 16; ++r) rv[r] = 0.f;
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = mbase + (r & 3) + 8 * (r >> 2) + 4 * h;
    float v = fmaf(acc[r], sc, sh) + rv[r];
    if (a.relu) v = fmaxf(v, 0.f);
    if (m < a.M) a.y[(long)m * a.y_ld + a.y_off + co] = v;
  }
}

struct ConvPlan {
  int bm = 128, bn = 128, kt_per_split = 1, nsplit = 1;
  int var = 0;  // S-layout convs: 0 base main loop, 1 fragment prefetch, 2 prefetch with 8 waves (conv_x3s.hip)
};

ConvPlan plan_conv(int M, int Co, int K);
int launch_conv(ConvArgs a, const ConvPlan& p, int stage, float* part_ws, size_t part_ws_floats, hipStream_t st);
int launch_splitk_epilogue(const ConvArgs& a, int nsplit, hipStream_t st);
// split-activation variant (conv_x3s.hip)
ConvPlan plan_conv_x3s(int M, int Co, int K);
ConvPlan plan_conv_b16(int M, int Co, int K);
ConvPlan plan_conv_f32d(int M, int Co, int K);
ConvPlan plan_conv_x6(int M, int Co, int K);
ConvPlan plan_conv_x6_batched(int M, int Co, int K, int batch);  // the Winograd forms' GEMMs
// Winograd F(2x2, 3x3) and F(4x4, 3x3) for the x6 path's stride-1 3x3 convs (wino.hip)
struct WinoGeom {
  int N, H, W, d;  // image, dilation (= padding)
  int m;           // output tile edge: 2 (F(2x2,3x3), 16 positions) or 4 (F(4x4,3x3), 36)
  int P;           // transformed positions (m + 2)^2 = the batched GEMMs' count
  int TY, TX;      // m x m output tiles per dilation sub-grid
  long T;          // N * d * d * TY * TX
};
WinoGeom wino_geom(int N, int H, int W, int d, int m = 2);
int launch_wino_weights(const float* w_packed, int Co, int Ci, float* U, hipStream_t st, int m = 2);
int launch_wino_in(const float* x, const WinoGeom& g, int Ci, float* V, hipStream_t st);
int launch_wino_out(const float* Mb, const WinoGeom& g, int Co, const float* scale, const float* shift, const float* res,
                    int res_ld, int relu, float* y, int y_ld, int y_off, hipStream_t st);
// prec 3: bf16x3 (S-layout operands); prec 1: plain bf16 (NHWC bf16 activations, [Co][K]
// bf16 weights with K ordered (64-channel block, tap, channel): packed_k64); prec 0: exact fp32
// (f32 MFMA) and prec 6: fp32 width on the bf16 MFMA (three-way register split), both over fp32
// NHWC activations and the fp32 packed weights
int launch_conv_x3s(ConvSArgs a, const ConvPlan& p, int stage, float* part_ws, size_t part_ws_floats,
                    hipStream_t st, int prec = 3);
int launch_split_act(const float* x, long P, int C, int ld, __bf16* out, hipStream_t st);
int launch_split_w3(const float* w, long R, int K, __bf16* ws, __bf16* wl, hipStream_t st);
int launch_occupy(int nwg, int us, hipStream_t st);  // timing study (cwt_debug_occupy)
int launch_unsplit_act(const __bf16* s, long P, int C, float* out, int ld, hipStream_t st);

// inner loop (adapt.hip): cache of instantiated graphs of the 200-step launch sequence
struct AdaptGraphCache {
  struct Entry {
    int E, n, h, w, S, iters;
    const void *fws, *lbl, *sc, *acc, *wbuf, *dargs;
    hipGraphExec_t exec;
    bool same(const Entry& o) const {
      return E == o.E && n == o.n && h == o.h && w == o.w && S == o.S && iters == o.iters && fws == o.fws &&
             lbl == o.lbl && sc == o.sc && acc == o.acc && wbuf == o.wbuf && dargs == o.dargs;
    }
  };
  std::vector<Entry> entries;
  hipStream_t cap_stream = nullptr;
  ~AdaptGraphCache();
};

// backbone helpers (backbone.hip).  Activation storage of the conv stack:
enum ActLayout { ACT_F32 = 0, ACT_SPLIT = 1, ACT_BF16 = 2 };  // fp32 NHWC, S-layout, bf16 NHWC
int launch_stem_conv1(const float* img, int N, int S, const float* w27x64, const float* scale,
                      const float* shift, float* out, int Ho, hipStream_t st, int layout = ACT_F32,
                      int relu = 1);
// Training-mode BatchNorm over a raw conv output (bn_train.hip): batch statistics of the M
// rows, running-statistic update (momentum, unbiased variance), eval fold rewritten from the
// new running statistics, then y = [relu](bn(y) [+ res]) [* Dropout2d mask] in place.
struct BnTrainArgs {
  void* y;          // activation in `layout` (ACT_F32 rows of ld floats; S-layout / bf16: ld = C)
  int layout, ld;
  long M;           // rows (N * H * W)
  int C;
  const void* res;  // optional residual, same layout as y
  int res_ld;
  int relu;
  float* bn;        // device [4][C]: gamma, beta, running_mean, running_var (updated)
  float* scale;     // eval fold gamma / sqrt(rv + eps) and beta - rm * scale (rewritten)
  float* shift;
  float eps, momentum;
  float drop_p;     // Dropout2d over (image, channel), stream 3 of dropout_scale
  unsigned long long seed;
  long rows_per_image;
};
size_t bn_train_part_floats(long M, int C);
int launch_bn_train(const BnTrainArgs& a, float* part, size_t part_floats, float* batch_sc, hipStream_t st);
// dst[i] = src[i] * sc[i % period] (the PPM fold of the bottleneck BN scale)
int launch_scale_cols(const float* src, float* dst, long n, int period, const float* sc, hipStream_t st);
// Episode preprocessing (preprocess.hip): Resize + ToTensor + Normalize of one HWC RGB image
// into [3][S][S] fp32, and the remapped / resized / padded int64 label
void find_new_hw(int h, int w, int S, int* nh, int* nw);
int launch_episode_image(const void* src, int src_f32, int H, int W, int S, const float* mean, const float* stdv,
                         const float* pad, int flip_h, int flip_v, float* dst, hipStream_t st);
int launch_episode_label(const unsigned char* src, int H, int W, int S, int cls, int flip_h, int flip_v,
                         long long* dst, hipStream_t st);
int launch_maxpool3s2_s(const __bf16* in, int N, int H, int W, int C, __bf16* out, int Ho, int Wo, hipStream_t st);
int launch_maxpool3s2_b16(const __bf16* in, int N, int H, int W, int C, __bf16* out, int Ho, int Wo, hipStream_t st);
int launch_maxpool3s2(const float* in, int N, int H, int W, int C, float* out, int Ho, int Wo,
                      hipStream_t st);
int launch_ppm(const float* x, int N, int h, int w, int ld, const int* bins, int nbins, float* ws,
               float* pooled, hipStream_t st, int layout = ACT_F32);
int launch_repack_cblock(const float* src, float* dst, int Co, int taps, int Ci, hipStream_t st);
int launch_smallm_gemm(const float* A, int lda, const float* const* Bt, const int* M, int np, int N, int K, int kc,
                       float* part, size_t part_floats, const float* const* scale, const float* const* shift,
                       float* out, hipStream_t st);
// Few-row form of the two PPM GEMMs (K = 512 or 2048) on the f32 MFMA; cells <= kPpmGemmMaxRows.
constexpr int kPpmGemmMaxRows = 200;
int launch_ppm_gemm(const float* A, int lda, const float* const* Bt, const int* M, int np, int N, int K,
                    const float* const* scale, const float* const* shift, float* part, size_t part_floats,
                    float* out, hipStream_t st);
int launch_ppm_field(const float* Q, int N, int h, int w, const int* bins, float* R, float* F, hipStream_t st);
// its adjoint: dQ [cells][9 * 512] from dF [N][h][w][512] (dR: R's shape, scratch)
int launch_ppm_field_bwd(const float* dF, int N, int h, int w, const int* bins, float* dR, float* dQ, hipStream_t st);

// ---- MatchNet / MMN backward (match_bwd.hip; launch_cp4d_dgrad in match.hip) ----
struct MmBwdWs {  // MutualMatching backward scratch, per (b, c): rows NA, columns NB, row blocks of 16
  float* rowmax;
  int* rowarg;
  float* colpv;  // [B*C][nrb][NB] column partial maxima, then the partial column sums
  int* colpi;
  float* colmax;
  int* colarg;
  float* srow;
  float* scol;
};
int launch_mutual_matching_bwd(const float* x, const float* dy, int B, int NA, int NB, int C, float* dx,
                               const MmBwdWs& ws, hipStream_t st);
int launch_relu_mask(const float* g, const float* out, long n, float* gm, hipStream_t st);
int cp4d_wgrad_part_floats(int cin, int cout);
int launch_cp4d_wgrad_mfma(const float* x, const float* gm, int B, int hA, int wA, int hB, int wB, int cin, int cout,
                           int G, float* part, hipStream_t st);
int launch_cp4d_wgrad(const float* x, const float* gm, int B, int hA, int wA, int hB, int wB, int cin, int cout,
                      float* part, size_t part_floats, float* dWa, float* dWb, float* db1, float* db2, hipStream_t st);
int launch_cp4d_dgrad(const float* g, int B, int hA, int wA, int hB, int wB, int gin, int gout, const float* Wa,
                      const float* Wb, float* dx, int accum, hipStream_t st);
int launch_match_softmax_bwd(const float* P, int ldp, const float* dA, int rows, int NB, float temp, int accum,
                             float* g, hipStream_t st);
int launch_token_norm(const float* x, long T, int C, float eps, float* xn, float* nrm, hipStream_t st);
int launch_token_norm_bwd(const float* xn, const float* nrm, const float* dxn, long T, int C, int ld_d, float eps,
                          int accum, float* dx, hipStream_t st);
int launch_wa_bwd(const float* tpg, int N, int h, int w, int co, const float* bt, const float* bp, const float* bg,
                  const float* dwavg, float* coef, float* dtpg, hipStream_t st);
size_t colsum_ws_floats(long R, int Cc);
int launch_colsum(const float* X, long R, int Cc, long ld, int accum, float* out, float* ws, size_t ws_floats,
                  hipStream_t st);
int launch_to_channels_first(const float* x, int B, int C, long P, float* y, hipStream_t st);
int launch_copy_pad(const float* X, long R, int Cc, int ld, float* out, hipStream_t st);
size_t deform_attn_bwd_ws_bytes(int B, int H, int W, int M, int D);
int launch_deform_attn_bwd(const float* value, const float* offsets, const float* logits, int B, int H, int W, int M,
                           int P, int D, const float* d_out, float* d_value, float* d_offsets, float* d_logits,
                           void* ws, hipStream_t st);
int launch_norm_blend_bwd(const float* a, const float* b, const float* d, long T, int C, float wt, float* d_a,
                          float* d_b, hipStream_t st);
int launch_copy_2d(const float* src, long R, int Cc, long lds, float* dst, long ldd, hipStream_t st);
int launch_mmn_blend_bwd(const float* d_fq, const float* d_mean, int B, long n, float att_wt, float* d_att,
                         float* d_fq_in, hipStream_t st);

}  // namespace cwt

// Kernel argument structs and launchers of the stage-1 pretraining step (pretrain_kernels.hip,
// driven by pretrain.hip).
#pragma once
#include "common.h"

namespace cwt {

struct WgradArgs {
  const float* dy;  // output gradient [M][Co] (row stride dy_ld)
  const float* x;   // conv input NHWC (pixel stride x_ld)
  float* out;       // set by launch_conv_wgrad: the slab base or gw
  long M;           // N * Ho * Wo
  int N, Hi, Wi, Ho, Wo, Co, K, kh, kw, stride, pad, dil;
  int x_ld, dy_ld;
  int chunks_per_split;
};
int launch_conv_wgrad(WgradArgs a, float* gw, float* ws, size_t ws_floats, hipStream_t st);
int launch_slab_reduce(const float* slabs, int nsplit, long n, float* dst, hipStream_t st);
int launch_wt_transpose(const float* w, float* wt, int Co, int Ci, int taps, hipStream_t st);
int launch_zero_insert(const float* dy, int N, int Ho, int Wo, int C, float* z, int Hi, int Wi, hipStream_t st);
int launch_stem1_wgrad(const float* img, int N, int S, const float* dy, int Ho, float* gw, float* ws,
                       size_t ws_floats, hipStream_t st);

// training-mode BN: stats [2][C] = mean, 1/sqrt(var + eps); run [2][C] = running mean, var
size_t ptbn_part_floats(long M, int C);
int launch_ptbn_fwd(const float* y, int ld, long M, int C, float* run, float eps, float momentum, int train,
                    float* stats, float* part, size_t part_floats, hipStream_t st);
struct PtBnApply {
  const float* y;  // raw conv output
  int y_ld;
  long M;
  int C;
  const float *gamma, *beta, *stats;
  const float* res;  // optional residual (raw conv output when res_stats != null)
  int res_ld;
  const float *res_gamma, *res_beta, *res_stats;
  int relu;
  float drop_p;  // Dropout2d over (image, channel) after the ReLU
  unsigned long long seed;
  long rows_per_image;
  float* out;      // activation (after dropout)
  float* out_pre;  // optional: the activation before dropout (the ReLU mask)
  int out_ld;
};
int launch_ptbn_apply(const PtBnApply& a, hipStream_t st);
struct PtBnBwd {
  const float* dout;  // gradient at the activation (after dropout / ReLU)
  int dout_ld;
  const float* act;   // activation before dropout (ReLU mask), or null
  int act_ld;
  int relu_from_y;    // act == null: the ReLU mask recomputed from y (gamma x_hat + beta > 0, no residual)
  const float* beta;
  float drop_p;
  unsigned long long seed;
  long rows_per_image;
  const float* y;     // raw conv output
  int y_ld;
  const float *gamma, *stats;
  long M;
  int C;
  float* dy;          // gradient at the raw conv output
  int dy_ld;
  float* g_out;       // optional: the gradient at the BN output (identity residual branch)
  int g_ld;
};
int launch_ptbn_bwd(const PtBnBwd& a, float* dgamma, float* dbeta, float* part, size_t part_floats, float* sums,
                    hipStream_t st);

int launch_maxpool_idx(const float* in, int N, int H, int C, float* out, uint8_t* idx, int Ho, hipStream_t st);
int launch_maxpool_bwd(const float* dout, const uint8_t* idx, int N, int H, int C, int Ho, float* din, hipStream_t st);
int launch_avgpool_bwd(const float* dpool, int N, int h, int C, const int* bins, float* dx, int ld, hipStream_t st);

struct PtGemm {
  const float* A;  // A(i, k) = A[i * sai + k * sak]
  const float* B;  // B(k, j) = B[k * sbk + j * sbj]
  float* C;        // C[i * ldc + j]
  long sai, sak, sbk, sbj, ldc;
  int M, N;
  long K;
  int k_per_split;
  float* slab;
};
int launch_pt_gemm(PtGemm g, float* ws, size_t ws_floats, hipStream_t st);
// bottleneck weights' PPM-branch columns <-> GEMM form wq[4][512 ci][9 * 512] (dir 0: w -> wq, 1: wq -> w)
int launch_ppm_wq(float* w, long w_ld, float* wq, int dir, hipStream_t st);

struct PtLoss {
  const float* logits;    // [N][h][w][nc]
  const int64_t* target;  // [N][S][S]
  float* dlogits;         // [N][h][w][nc]
  float* Rr;              // workspace (set by the launcher)
  int N, S, h, w, nc, ignore;
  float on, off;          // smoothed one-hot values
};
size_t seg_ce_ws_bytes(int N, int S, int w, int nc);
int launch_seg_ce_smooth(PtLoss a, void* ws, size_t ws_bytes, float* loss, hipStream_t st);
// evaluation: out[0] mean CE (plain one-hot), out[1] valid pixels; iu [3][nc] intersection / union / target
size_t seg_eval_ws_bytes(int N, int S, int w, int nc);
int launch_seg_eval(PtLoss a, void* ws, size_t ws_bytes, float* out, float* iu, hipStream_t st);

// torch.optim.SGD step over a flat buffer (seg.hip)
int launch_sgd(float* p, const float* g, float* buf, long n, float lr, float mom, float wd, int nesterov, int first,
               hipStream_t st);

}  // namespace cwt

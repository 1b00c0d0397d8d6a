// C ABI of libcwt.so (declared in include/cwt.h): context, weight loading, workspace pool
// and the frozen-extractor orchestration.  See include/cwt.h for the contract of each
// entry point and the reference call site it replaces.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/cwt.h"
#include "../../include/cwt_debug.h"
#include "common.h"
#include "kernels.h"
#include "tail_body.h"

namespace cwt {

static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }
int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

// launchers defined in the other units
struct AdaptScalars;
struct AdaptDevArgs;
int launch_adapt(const float* f, const int64_t* lbl64, int E, int n, int h, int w, int S, float lr, int iters,
                 float* W, float* f_ws, uint8_t* lbl_ws, AdaptScalars* sc, float* acc3, float* wbuf,
                 AdaptDevArgs* dargs, AdaptGraphCache* cache, int upw, unsigned* status, long spin_limit,
                 hipStream_t st, hipEvent_t ev_k0, hipEvent_t ev_k1, const FusedTail* tail = nullptr);
const char* adapt_kernel_name(int E, int n, int h, int w, int iters, int upw);
int adapt_persist_workgroups(int E, int n, int h, int w, int iters, int upw);
extern unsigned long long* g_adapt_stamps;
extern long g_adapt_stamps_n;
size_t adapt_ws_sizes(int E, int n, int h, int w, int S, size_t* fws, size_t* lbl, size_t* sc, size_t* acc,
                      size_t* wbuf, size_t* dargs);
int launch_seg_ce(const float* logits, const int64_t* target, int B, int h, int w, int S, float* loss_out,
                  float* dlogits, uint8_t* lbl_ws, AdaptScalars* sc, double* loss_num, hipStream_t st);
int launch_normalize(const float* f, int B, int Pb, float* out, const float* W0, float* logits0, hipStream_t st);
int launch_classify(const float* W, const float* f, int B, int Pb, float* logits, hipStream_t st);
int launch_classify_scaled(const float* W, const float* f, const float* inv, int B, int Pb, float* logits,
                           hipStream_t st);
size_t attention_fold_floats(int C, int H);
int attention_fold(const float* w_qkvs, const float* fc_w, int C, int H, float* fold, float* ws, size_t ws_floats,
                   hipStream_t st);
size_t attention_infer_ws_floats(int B, int hw, int C, int H);
size_t episode_tail_ws_floats(int B, int hw, int G);
size_t episode_tail_cnt_words();
unsigned episode_tail_max_epoch(int G);
int launch_episode_tail(const float* q, const float* f, int B, int hw, int h, int w, int S, const int64_t* target,
                        const float* fold, const float* fc_b, const float* ln_w, const float* ln_b, float* out,
                        float* logits, float* logits0, float* iut, double* ce, float* iut0, float* ws,
                        unsigned* cnt, unsigned epoch, int G, long spin_limit, unsigned* status, hipStream_t st,
                        unsigned long long* stamps);
int attention_infer(const float* q, const float* f, int B, int hw, int C, int H, const float* fold, const float* fc_b,
                    const float* ln_w, const float* ln_b, float* out, float* inv_norm, float* logits0, float* ws,
                    hipStream_t st);
int launch_classify_bwd(const float* dl, const float* f, int B, int Pb, float* dW, hipStream_t st);
// variant heads (heads.hip)
int launch_cos_weight(float* v, const float* g, int n, int C, int mode, float* w_eff, float* vnorm, hipStream_t st);
int launch_cos_cls_fwd(const float* x, long P, int B, int n, const float* w_eff, const float* bias, const float* scale,
                       float* out, hipStream_t st);
int cos_cls_bwd_blocks(long total);
int launch_cos_cls_bwd(const float* x, long P, int B, int n, const float* w_eff, const float* bias, const float* scale,
                       const float* G, float* part, float* part_s, int mode, const float* v, const float* g,
                       const float* vnorm, float* dv, float* dg, float* db, float* dscale, hipStream_t st);
int launch_corr(const float* q, const float* k, int B, int Pq, int Pk, int C, float* qn, float* kn, float* sim,
                hipStream_t st);
int launch_unsplit_act(const __bf16* s, long P, int C, float* out, int ld, hipStream_t st);
int launch_widen_bf16(const __bf16* x, long n, float* y, hipStream_t st);
int launch_gemm_abt(const float* A, const float* Bm, int B, int M, int N, int K, float* Cm, hipStream_t st);
int launch_mutual_matching(const float* x, int B, int NA, int NB, int C, float* y, float* rowmax, float* colpart,
                           float* colmax, hipStream_t st);
int launch_mutual_matching_sum(const float* x, const float* x2, int B, int NA, int NB, float* y, float* rowmax,
                               float* colpart, float* colmax, hipStream_t st);
int launch_mutual_matching_planar2(const float* x, int B, int NA, int NB, float* y, float* rowmax, float* colpart,
                                   float* colmax, hipStream_t st);
int launch_cp4d_layer(const float* x, int B, int hA, int wA, int hB, int wB, int cin, int cout, const float* Wa,
                      const float* ba, const float* Wb, const float* bb, float* y, hipStream_t st);
int launch_cp4d_layer_variant(const float* x, int B, int hA, int wA, int hB, int wB, int cin, int cout,
                              const float* Wa, const float* ba, const float* Wb, const float* bb, float* y, int variant,
                              hipStream_t st);
int launch_to_channels_last(const float* x, int B, int C, long P, float* y, hipStream_t st);
int launch_add_inplace(float* y, const float* x, long n, hipStream_t st);
int launch_match_softmax(const float* corr, int B, int NA, int NB, float temp, int ldp, float* P, hipStream_t st);
int launch_match_vt(const float* v, int B, int NB, int C, int ldp, float* vt, hipStream_t st);
int launch_cv4d_layer(const float* x, int B, int hA, int wA, int hB, int wB, int cin, int cout, const float* W,
                      const float* bias, int swap, float* y, hipStream_t st);
int launch_sce_descriptor(const float* x, int B, int h, int w, int C, int k, int ldg, float* g, hipStream_t st);
int launch_channel_sum(const float* x, int B, int L, long P, float* y, hipStream_t st);
int launch_match_masks(float* corr, int B, int NA, int NB, const uint8_t* ig, const int64_t* s_mask, float* incons,
                       int* q2k, float* pv, int* pi, hipStream_t st, float drop_p = 0.f, unsigned long long seed = 0);
int launch_match_zero_ig_cols(float* g, const uint8_t* ig, int B, int NA, int NB, hipStream_t st);
int launch_wa_attn(const float* tpg, int N, int h, int w, int co, const float* bt, const float* bp, const float* bg,
                   float* wavg, hipStream_t st);
int launch_wa_residual(const float* x, const float* back, const float* b, long n, int C, float* out, hipStream_t st);
int launch_linear_epilogue(const float* tmp, const float* bias, const float* acc, long P, int N, int relu, float* out,
                           hipStream_t st);
int launch_sine_pos_add(const float* x, int B, int h, int w, int C, float temperature, int normalize, float scale,
                        float eps, float* out, hipStream_t st);
int launch_deform_attn(const float* value, const float* offsets, const float* logits, int B, int H, int W, int M,
                       int P, int D, float* out, hipStream_t st);
int launch_norm_blend(const float* a, const float* b, long T, int C, float wt, float* out, hipStream_t st);
int launch_mmn_blend(const float* fq_in, const float* att, int B, long n, float att_wt, float* att_mean, float* fq_out,
                     hipStream_t st);
int launch_seg_metrics(const float* logits, const int64_t* target, int B, int h, int w, int S, float* iut,
                       double* ce, unsigned* counts_ws, hipStream_t st, const float* logits2 = nullptr,
                       float* iut2 = nullptr);
int launch_iou_preds(const int64_t* preds, const int64_t* target, long n, int K, int ignore, float* iut,
                     unsigned* counts_ws, hipStream_t st);
int launch_sgd(float* p, const float* g, float* buf, long n, float lr, float mom, float wd, int nesterov, int first,
               hipStream_t st);
size_t attention_saved_floats(int B, int hw, int C, int H);
size_t attention_ws_floats(int B, int hw, int C, int H);
int attention_fwd(const float* q, const float* f, int B, int hw, int C, int H, const float* w_qkvs,
                  const float* fc_w, const float* fc_b, const float* ln_w, const float* ln_b, float* out,
                  float* saved, float* ws, hipStream_t st, float p_attn, float p_out, unsigned long long seed);
int attention_bwd(const float* q, const float* f, int B, int hw, int C, int H, const float* w_qkvs,
                  const float* fc_w, const float* fc_b, const float* ln_w, const float* ln_b, const float* saved,
                  const float* d_out, float* g_w_qkvs, float* g_fc_w, float* g_fc_b, float* g_ln_w, float* g_ln_b,
                  float* ws, hipStream_t st, float p_attn, float p_out, unsigned long long seed);
size_t attention_bwd_ws_floats(int B, int hw, int C, int H);

// ------------------------------------------------------------------------------------------
struct ConvLayer {
  int Ci = 0, Co = 0, k = 1, stride = 1, pad = 0, dil = 1;
  float* w = nullptr;  // device, packed [Co][k][k][Ci] (stem conv1: [ci][ky][kx][co])
  __bf16* w_s = nullptr;   // S-layout [Co][K/32][hi 32 | lo 32] of the same split (conv_x3s.hip)
  __bf16* w_l = nullptr;   // x6: the third term w - hi - lo, [Co][K/32][32] (exact in bf16)
  // x6 Winograd forms (stride-1 3x3, Ci >= 256; wino.hip): U = G g G^T per transformed
  // position, [P][Co][Ci] split like w_s / w_l; wino_s / wino_l F(2x2,3x3) (P = 16), wino4_s /
  // wino4_l F(4x4,3x3) (P = 36)
  __bf16* wino_s = nullptr;
  __bf16* wino_l = nullptr;
  __bf16* wino4_s = nullptr;
  __bf16* wino4_l = nullptr;
  __bf16* w_b = nullptr;   // plain bf16 [Co][K], K in packed_k64 order (bf16 conv stack; Ci % 64 == 0)
  float* scale = nullptr;
  float* shift = nullptr;
  float* bn = nullptr;  // [4][Co] gamma, beta, running_mean, running_var (training-mode BN)
};

struct Block {
  ConvLayer c1, c2, c3, down;
  bool has_down = false;
};

struct Backbone {  // the opaque cwt_backbone of the C ABI
  int layers = 0;
  int device = 0;
  int precision = CWT_CONV_FP32;  // cwt_backbone_set_precision
  ConvLayer stem[3];
  std::vector<Block> blocks[4];
  ConvLayer ppm[4];     // PPM 1x1 convs (scale/shift used; weights below)
  float* ppm_wt[4] = {};  // their weights K-major [2048][512] for the small-M GEMM
  ConvLayer bott;       // bottleneck conv over the 2048 layer4 channels only
  float* ppm_q[4] = {};   // bottleneck weights of PPM bin b, K-major [512][9 * 512], BN scale folded in
  float* ppm_q_raw[4] = {};  // the same without the BN scale (training-mode BN; ppm_q is refolded)
  float* ones = nullptr;     // [2048] scale / shift of a raw conv (training-mode BN)
  float* zeros = nullptr;
  float eps = 1e-5f;
  std::map<std::string, std::pair<float*, int>> bn_by_name;  // BN prefix -> (device [4][C], C)
  std::vector<void*> allocs;
};

struct WsBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

}  // namespace cwt

struct cwt_ctx {
  int device = 0;
  std::map<std::string, cwt::WsBuf> ws;
  size_t ws_total = 0;
  // optional per-launch profiling: events recorded on the caller's stream around each
  // instrumented launch (cwt_profile_enable); read back after a sync
  int prof_level = 0;  // 0 off, 1 phases + the bottleneck conv, 2 every launch
  struct Rec {
    std::string name;
    double flops, bytes;
    hipEvent_t e0, e1;
    int fslot = -1;  // a fused loop + tail launch: its slot in fstamps, and which part (0 loop, 1 tail)
    int fpart = 0;
  };
  // the fused loop + tail launches' realtime stamps ({start, loop end, tail end} per slot, a ring)
  unsigned long long* fstamps = nullptr;
  int fstamp_next = 0;
  std::vector<Rec> recs;
  std::vector<hipEvent_t> evpool;
  size_t ev_used = 0;
  // inner loop: captured graphs of the step sequence (disable with CWT_ADAPT_GRAPH=0)
  cwt::AdaptGraphCache adapt_graphs;
  bool use_graph = true;
  // conv arithmetic (CWT_CONV_ARITH_*): fp32 width on the bf16 matrix cores, operands split three
  // ways in registers (default, CWT_CONV=x6); bf16x3 over S-layout activations (CWT_CONV=x3s,
  // ~16-bit operands: a declared approximation); exact fp32 MFMA (CWT_CONV=f32)
  int conv_arith = CWT_CONV_ARITH_BF16X6;
  // persistent inner loop: units per workgroup (0 automatic, 1, 2), cwt_ctx_set_adapt_units
  int adapt_upw = 0;
  // asynchronous status word (cwt_ctx_status): mapped, coherent host memory the kernels OR
  // CWT_STATUS_* bits into (system-scope stores; written only on failure)
  unsigned* status_host = nullptr;
  unsigned* status_dev = nullptr;
  long adapt_spin_limit = 0;  // 0: the persistent loop's default bound (cwt_debug_adapt_spin_limit)
  // cwt_episode_tail's counters: this context's next launch number on them; ~0u = re-zero first
  unsigned tail_epoch = ~0u;
  int tail_G = 0;
  int tail_stamp_G = 0;  // workgroups of the last stamped tail launch (CWT_TAIL_STAMPS)
  // folded CWT weights of cwt_attention_infer (M_h = W_h^T W_h, P = [fc_h W_h]) and the
  // parameter identity they were folded from (buffers + the caller's version counter)
  const float* fold_w = nullptr;
  const float* fold_fc = nullptr;
  int64_t fold_ver = -1;
  int fold_H = 0;
  // a second stream for independent work inside one call (the symmetric NeighConsensus
  // branches), forked from and joined back into the caller's stream by events
  hipStream_t aux = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
};

namespace cwt {

// Profiling bracket: Prof p(ctx, st, name, flops, bytes); ... launches ...; p.end();
struct Prof {
  cwt_ctx* c;
  hipStream_t st;
  int idx = -1;
  Prof(cwt_ctx* ctx, hipStream_t s, const std::string& name, double flops, double bytes, int level = 2)
      : c(ctx), st(s) {
    if (c->prof_level < level) return;
    hipEvent_t ev[2];
    for (int k = 0; k < 2; ++k) {
      if (c->ev_used == c->evpool.size()) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return;
        c->evpool.push_back(e);
      }
      ev[k] = c->evpool[c->ev_used++];
    }
    c->recs.push_back({name, flops, bytes, ev[0], ev[1]});
    idx = (int)c->recs.size() - 1;
    (void)hipEventRecord(ev[0], st);
  }
  void end() {
    if (idx >= 0) (void)hipEventRecord(c->recs[idx].e1, st);
    idx = -1;
  }
  // deferred form: the record's two events, for a callee to record around one launch
  // (Prof(..., level, true)); recorded in place of the constructor / end() when used
  hipEvent_t ev0() const { return idx >= 0 ? c->recs[idx].e0 : nullptr; }
  hipEvent_t ev1() const { return idx >= 0 ? c->recs[idx].e1 : nullptr; }
  Prof(cwt_ctx* ctx, hipStream_t s, const std::string& name, double flops, double bytes, int level, bool deferred)
      : Prof(ctx, s, name, flops, bytes, deferred ? 1 << 30 : level) {
    if (!deferred || c->prof_level < level) return;
    hipEvent_t ev[2];
    for (int k = 0; k < 2; ++k) {
      if (c->ev_used == c->evpool.size()) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return;
        c->evpool.push_back(e);
      }
      ev[k] = c->evpool[c->ev_used++];
    }
    c->recs.push_back({name, flops, bytes, ev[0], ev[1]});
    idx = (int)c->recs.size() - 1;
  }
};

static int ensure_ws(cwt_ctx* ctx, const std::string& name, size_t bytes, void** out) {
  WsBuf& b = ctx->ws[name];
  if (b.bytes < bytes) {
    if (b.p) {
      CWT_HIP(hipDeviceSynchronize());  // the old buffer may still be in use by queued work
      CWT_HIP(hipFree(b.p));
      ctx->ws_total -= b.bytes;
      b.p = nullptr;
      b.bytes = 0;
    }
    size_t nb = (bytes + 255) & ~(size_t)255;
    CWT_HIP(hipMalloc(&b.p, nb));
    b.bytes = nb;
    ctx->ws_total += nb;
  }
  *out = b.p;
  return 0;
}

// 256 B of zeros on the device (the LDS-DMA source of zero-padding taps in conv_x3s)
static int zero_line(cwt_ctx* ctx, const __bf16** out) {
  const bool fresh = ctx->ws.find("zero") == ctx->ws.end();
  void* p;
  int rc;
  if ((rc = ensure_ws(ctx, "zero", 256, &p))) return rc;
  if (fresh) CWT_HIP(hipMemset(p, 0, 256));
  *out = (const __bf16*)p;
  return 0;
}

// C = A . Bm^T (+ bias[N]) (+ res, pixel stride res_ld) in exact fp32 on the LDS-DMA conv body:
// conv_igemm_f32d as a 1x1 conv over M "pixels" (A's [M][K] rows) with the [N][K] weights Bm (a
// 1x1 conv's fp32 packing is plain row-major [Co][Ci]); the epilogue is fmaf(acc, 1, bias) then
// + res, the order of the separate bias / residual passes it replaces.  Shapes: K % 32 == 0,
// N % 64 == 0, 16-B aligned operands (gemm_f32d_ok); the rest stay on corr_gemm_kernel.
// Used for MatchNet's readout, cwt_linear and (with the measured plans of the heads' GEMM shapes,
// conv_plans_f32d.inc from tools/conv_s_sweep.py --configs 0:60:1, profiles/r4/sweeps) the
// WeightAverage GEMMs -- with the heuristic plans those measured slower than corr_gemm_kernel
// (0.72 against 0.66 ms for the layer-4 module, profiles/r4/run_i).  CWT_GEMM_F32D=0 keeps
// every GEMM on corr_gemm_kernel.
static int gemm_f32d_mode() {
  static const int m = getenv("CWT_GEMM_F32D") ? atoi(getenv("CWT_GEMM_F32D")) : 1;
  return m;
}
static bool gemm_f32d_ok(int M, int N, int K, const void* A, const void* Bm, const void* Cm, const void* res) {
  const bool on = gemm_f32d_mode() != 0;
  const uintptr_t al = (uintptr_t)A | (uintptr_t)Bm | (uintptr_t)Cm | (uintptr_t)res;
  return on && M >= 1 && K % 32 == 0 && N % 64 == 0 && N <= 8192 && (al & 15) == 0;
}
static int zero_line(cwt_ctx* ctx, const __bf16** out);
static int gemm_f32d(cwt_ctx* ctx, const float* A, const float* Bm, int M, int N, int K, float* Cm, const float* bias,
                     const float* res, int res_ld, hipStream_t st, int relu = 0) {
  const bool fresh = ctx->ws.find("gemm.one") == ctx->ws.end();
  void *one, *zer, *part;
  const __bf16* zero;
  int rc;
  if ((rc = ensure_ws(ctx, "gemm.one", 8192 * 4, &one)) || (rc = ensure_ws(ctx, "gemm.zero", 8192 * 4, &zer)) ||
      (rc = zero_line(ctx, &zero)))
    return rc;
  if (fresh) {
    CWT_HIP(hipMemsetD32((hipDeviceptr_t)one, 0x3f800000u, 8192));  // 1.0f
    CWT_HIP(hipMemset(zer, 0, 8192 * 4));
  }
  const ConvPlan pl = plan_conv_f32d(M, N, K);
  const size_t part_floats = pl.nsplit > 1 ? (size_t)pl.nsplit * M * N : 1;
  if ((rc = ensure_ws(ctx, "gemm.part", part_floats * 4, &part))) return rc;
  ConvSArgs a;
  memset(&a, 0, sizeof(a));
  a.xs = (const __bf16*)A;
  a.ws = (const __bf16*)Bm;
  a.zero = zero;
  a.scale = (const float*)one;
  a.shift = bias ? bias : (const float*)zer;
  a.res = res;
  a.res_ld = res_ld;
  a.y = Cm;
  a.y_ld = N;
  a.N = 1;
  a.Hi = M;
  a.Wi = 1;
  a.Ci = K;
  a.Ho = M;
  a.Wo = 1;
  a.Co = N;
  a.kh = a.kw = 1;
  a.stride = 1;
  a.dil = 1;
  a.M = M;
  a.K = K;
  a.relu = relu;
  return launch_conv_x3s(a, pl, 0, (float*)part, part_floats, st, 0);
}

// MatchNet's readout weighted_v[b] = attn[b] . v[b] as tokens [B][NA][Cv] = P[b] . vt[b]^T
static int readout_gemm(cwt_ctx* ctx, const float* P, const float* vt, int B, int NA, int Cv, int ldp, float* out,
                        hipStream_t st) {
  if (!gemm_f32d_ok(NA, Cv, ldp, P, vt, out, nullptr)) return launch_gemm_abt(P, vt, B, NA, Cv, ldp, out, st);
  for (int b = 0; b < B; ++b) {
    int rc = gemm_f32d(ctx, P + (long)b * NA * ldp, vt + (long)b * Cv * ldp, NA, Cv, ldp, out + (long)b * NA * Cv,
                       nullptr, nullptr, 0, st);
    if (rc) return rc;
  }
  return 0;
}

struct HostParams {
  std::map<std::string, std::pair<const float*, int64_t>> m;
  const float* get(const std::string& k, int64_t numel, std::string* err) const {
    auto it = m.find(k);
    if (it == m.end() || it->second.first == nullptr) {
      *err = "missing tensor '" + k + "'";
      return nullptr;
    }
    if (it->second.second != numel) {
      *err = "tensor '" + k + "' has " + std::to_string(it->second.second) + " elements, expected " +
             std::to_string(numel);
      return nullptr;
    }
    return it->second.first;
  }
};

static int upload(Backbone* bb, const std::vector<float>& v, float** out) {
  void* p = nullptr;
  CWT_HIP(hipMalloc(&p, v.size() * sizeof(float)));
  CWT_HIP(hipMemcpy(p, v.data(), v.size() * sizeof(float), hipMemcpyHostToDevice));
  bb->allocs.push_back(p);
  *out = (float*)p;
  return 0;
}

static uint16_t bf16_rne(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7F800000u) == 0x7F800000u) return (uint16_t)(u >> 16);  // inf / nan pass through
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

static float bf16_to_float(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

static int upload_u16(Backbone* bb, const std::vector<uint16_t>& v, __bf16** out) {
  void* p = nullptr;
  CWT_HIP(hipMalloc(&p, v.size() * sizeof(uint16_t)));
  CWT_HIP(hipMemcpy(p, v.data(), v.size() * sizeof(uint16_t), hipMemcpyHostToDevice));
  bb->allocs.push_back(p);
  *out = (__bf16*)p;
  return 0;
}

// BN eval folding as PyTorch's CPU inference kernel: alpha = w / sqrt(var + eps), beta = b - mean * alpha.
// ci_total / ci_off: the stored weight has ci_total input channels; this layer takes
// [ci_off, ci_off + Ci) of them (the bottleneck's layer4 half).
static int load_conv(Backbone* bb, const HostParams& hp, const std::string& wname, const std::string& bnp, int Ci,
                     int Co, int k, int stride, int pad, int dil, float eps, bool stem1, ConvLayer* L,
                     int ci_total = -1, int ci_off = 0) {
  if (ci_total < 0) ci_total = Ci;
  std::string err;
  const float* w = hp.get(wname, (int64_t)Co * ci_total * k * k, &err);
  if (!w) return fail(CWT_EARG, err);
  const float* g = hp.get(bnp + ".weight", Co, &err);
  const float* b = g ? hp.get(bnp + ".bias", Co, &err) : nullptr;
  const float* rm = b ? hp.get(bnp + ".running_mean", Co, &err) : nullptr;
  const float* rv = rm ? hp.get(bnp + ".running_var", Co, &err) : nullptr;
  if (!rv) return fail(CWT_EARG, err);
  L->Ci = Ci;
  L->Co = Co;
  L->k = k;
  L->stride = stride;
  L->pad = pad;
  L->dil = dil;
  const int K = k * k * Ci;
  std::vector<float> packed((size_t)Co * K);
  for (int co = 0; co < Co; ++co)
    for (int ci = 0; ci < Ci; ++ci)
      for (int ky = 0; ky < k; ++ky)
        for (int kx = 0; kx < k; ++kx) {
          const float v = w[(((size_t)co * ci_total + ci_off + ci) * k + ky) * k + kx];
          if (stem1)
            packed[((size_t)(ci * 9 + ky * 3 + kx)) * Co + co] = v;
          else
            packed[(size_t)co * K + packed_k(ci, ky * k + kx, k * k)] = v;
        }
  std::vector<float> sc(Co), sh(Co);
  for (int c = 0; c < Co; ++c) {
    const float invstd = 1.0f / std::sqrt(rv[c] + eps);
    sc[c] = g[c] * invstd;
    sh[c] = b[c] - rm[c] * sc[c];
  }
  int rc;
  if ((rc = upload(bb, packed, &L->w))) return rc;
  if (!stem1) {  // bf16x3 operands: hi = bf16_rne(w), lo = bf16_rne(w - hi)
    std::vector<uint16_t> hi(packed.size()), lo(packed.size()), lo3(packed.size());
    for (size_t i = 0; i < packed.size(); ++i) {
      const float v = packed[i];
      hi[i] = bf16_rne(v);
      const float r = v - bf16_to_float(hi[i]);
      lo[i] = bf16_rne(r);
      lo3[i] = bf16_rne(r - bf16_to_float(lo[i]));  // exact: at most 8 significant bits remain
    }
    std::vector<uint16_t> sl(2 * packed.size());
    for (size_t r = 0; r < (size_t)Co; ++r)
      for (int kb = 0; kb < K / 32; ++kb)
        for (int i = 0; i < 32; ++i) {
          const size_t src = r * K + kb * 32 + i, dst = (r * (K / 32) + kb) * 64 + i;
          sl[dst] = hi[src];
          sl[dst + 32] = lo[src];
        }
    if ((rc = upload_u16(bb, sl, &L->w_s))) return rc;
    if (K % 32 == 0 && (rc = upload_u16(bb, lo3, &L->w_l))) return rc;  // [Co][K] = [Co][K/32][32]
    // the Winograd form's transformed weights: stride-1 3x3 layers with Ci >= 256 (at Ci = 128 the
    // 16 thin GEMMs and the transforms measured slower than the direct conv: 35.9 vs 29.1 us,
    // profiles/r5/sweeps)
    // F(4x4,3x3) only on request (CWT_WINO=4 at load): faster in the pipeline but ~20x the
    // rounding error of F(2x2) / the fp32 conv (DESIGN.md §3 "Measured and not kept")
    static const bool wino4 = getenv("CWT_WINO") && getenv("CWT_WINO")[0] == '4';
    if (k == 3 && stride == 1 && Ci >= 128 && Ci % 32 == 0) {
      for (const int m : {2, 4}) {
        if ((m == 2 && Ci < 256) || (m == 4 && !wino4)) continue;
        const int P = (m + 2) * (m + 2);
        const size_t n = (size_t)P * Co * Ci;
        void *U = nullptr, *us = nullptr, *ul = nullptr;
        CWT_HIP(hipMalloc(&us, n * 4));
        bb->allocs.push_back(us);
        CWT_HIP(hipMalloc(&ul, n * 2));
        bb->allocs.push_back(ul);
        CWT_HIP(hipMalloc(&U, n * 4));
        rc = launch_wino_weights(L->w, Co, Ci, (float*)U, nullptr, m);
        if (!rc) rc = launch_split_w3((const float*)U, (long)P * Co, Ci, (__bf16*)us, (__bf16*)ul, nullptr);
        const hipError_t e = hipDeviceSynchronize();
        (void)hipFree(U);
        if (rc) return rc;
        if (e != hipSuccess) return fail((int)e, "winograd weight transform");
        (m == 2 ? L->wino_s : L->wino4_s) = (__bf16*)us;
        (m == 2 ? L->wino_l : L->wino4_l) = (__bf16*)ul;
      }
    }
    if (Ci % 64 == 0) {  // plain bf16 operand of the bf16 conv stack, K in packed_k64 order
      std::vector<uint16_t> b16(packed.size());
      for (int co = 0; co < Co; ++co)
        for (int ci = 0; ci < Ci; ++ci)
          for (int tap = 0; tap < k * k; ++tap)
            b16[(size_t)co * K + packed_k64(ci, tap, k * k)] = hi[(size_t)co * K + packed_k(ci, tap, k * k)];
      if ((rc = upload_u16(bb, b16, &L->w_b))) return rc;
    }
  }
  if ((rc = upload(bb, sc, &L->scale))) return rc;
  if ((rc = upload(bb, sh, &L->shift))) return rc;
  std::vector<float> bnp4((size_t)4 * Co);
  for (int c = 0; c < Co; ++c) {
    bnp4[c] = g[c];
    bnp4[Co + c] = b[c];
    bnp4[2 * Co + c] = rm[c];
    bnp4[3 * Co + c] = rv[c];
  }
  if ((rc = upload(bb, bnp4, &L->bn))) return rc;
  bb->bn_by_name[bnp] = {L->bn, Co};
  return 0;
}

// Weights of the folded PPM branch (backbone.hip, PPM section): the PPM 1x1 conv weights
// transposed to [2048][512], and per bin b the bottleneck taps over that bin's 512 concat
// channels as Wq_b[ci][tap * 512 + co] = W[co][2048 + 512 b + ci][tap] * bn_scale[co].
static int load_ppm_fold(Backbone* bb, const HostParams& hp, float eps) {
  std::string err;
  for (int b = 0; b < 4; ++b) {
    const float* w = hp.get("ppm.features." + std::to_string(b) + ".1.weight", (int64_t)512 * 2048, &err);
    if (!w) return fail(CWT_EARG, err);
    std::vector<float> t((size_t)2048 * 512);
    for (int co = 0; co < 512; ++co)
      for (int ci = 0; ci < 2048; ++ci) t[(size_t)ci * 512 + co] = w[(size_t)co * 2048 + ci];
    int rc;
    if ((rc = upload(bb, t, &bb->ppm_wt[b]))) return rc;
  }
  const float* w = hp.get("bottleneck.0.weight", (int64_t)512 * 4096 * 9, &err);
  const float* g = w ? hp.get("bottleneck.1.weight", 512, &err) : nullptr;
  const float* rv = g ? hp.get("bottleneck.1.running_var", 512, &err) : nullptr;
  if (!rv) return fail(CWT_EARG, err);
  for (int b = 0; b < 4; ++b) {
    std::vector<float> q((size_t)512 * 4608), qr((size_t)512 * 4608);
    for (int co = 0; co < 512; ++co) {
      const float sc = g[co] * (1.0f / std::sqrt(rv[co] + eps));  // as load_conv's BN fold
      for (int ci = 0; ci < 512; ++ci)
        for (int tap = 0; tap < 9; ++tap) {
          const float v = w[((size_t)co * 4096 + 2048 + 512 * b + ci) * 9 + tap];
          qr[(size_t)ci * 4608 + tap * 512 + co] = v;
          q[(size_t)ci * 4608 + tap * 512 + co] = v * sc;
        }
    }
    int rc;
    if ((rc = upload(bb, q, &bb->ppm_q[b])) || (rc = upload(bb, qr, &bb->ppm_q_raw[b]))) return rc;
  }
  return 0;
}

static const int kBlocks50[4] = {3, 4, 6, 3};
static const int kBlocks101[4] = {3, 4, 23, 3};
static const int kBins[4] = {1, 2, 3, 6};

static int load_backbone(int layers, const HostParams& hp, float eps, Backbone** out) {
  if (layers != 50 && layers != 101) return fail(CWT_EARG, "layers must be 50 or 101");
  Backbone* bb = new Backbone();
  bb->layers = layers;
  bb->eps = eps;
  int rc = 0;
  auto cleanup = [&]() {
    for (void* p : bb->allocs) (void)hipFree(p);
    delete bb;
  };
  // layer0: deep-base stem (resnet.py:110-118)
  if ((rc = load_conv(bb, hp, "layer0.0.weight", "layer0.1", 3, 64, 3, 2, 1, 1, eps, true, &bb->stem[0])) ||
      (rc = load_conv(bb, hp, "layer0.3.weight", "layer0.4", 64, 64, 3, 1, 1, 1, eps, false, &bb->stem[1])) ||
      (rc = load_conv(bb, hp, "layer0.6.weight", "layer0.7", 64, 128, 3, 1, 1, 1, eps, false, &bb->stem[2]))) {
    cleanup();
    return rc;
  }
  const int* nb = (layers == 50) ? kBlocks50 : kBlocks101;
  int inplanes = 128;
  const int planes_of[4] = {64, 128, 256, 512};
  for (int li = 0; li < 4; ++li) {
    const int planes = planes_of[li];
    for (int bi = 0; bi < nb[li]; ++bi) {
      Block B;
      // dilation surgery (pspnet.py:103-112): layer3 conv2 d2 s1, layer4 conv2 d4 s1, downsample s1
      int s2 = 1, d2 = 1, sd = 1;
      if (li == 1 && bi == 0) {
        s2 = 2;
        sd = 2;
      }
      if (li == 2) d2 = 2;
      if (li == 3) d2 = 4;
      const std::string p = "layer" + std::to_string(li + 1) + "." + std::to_string(bi);
      if ((rc = load_conv(bb, hp, p + ".conv1.weight", p + ".bn1", inplanes, planes, 1, 1, 0, 1, eps, false, &B.c1)) ||
          (rc = load_conv(bb, hp, p + ".conv2.weight", p + ".bn2", planes, planes, 3, s2, d2, d2, eps, false, &B.c2)) ||
          (rc = load_conv(bb, hp, p + ".conv3.weight", p + ".bn3", planes, planes * 4, 1, 1, 0, 1, eps, false,
                          &B.c3))) {
        cleanup();
        return rc;
      }
      if (bi == 0) {
        B.has_down = true;
        if ((rc = load_conv(bb, hp, p + ".downsample.0.weight", p + ".downsample.1", inplanes, planes * 4, 1, sd, 0, 1,
                            eps, false, &B.down))) {
          cleanup();
          return rc;
        }
      }
      inplanes = planes * 4;
      bb->blocks[li].push_back(B);
    }
  }
  for (int i = 0; i < 4; ++i) {
    const std::string p = "ppm.features." + std::to_string(i);
    if ((rc = load_conv(bb, hp, p + ".1.weight", p + ".2", 2048, 512, 1, 1, 0, 1, eps, false, &bb->ppm[i]))) {
      cleanup();
      return rc;
    }
  }
  if ((rc = load_conv(bb, hp, "bottleneck.0.weight", "bottleneck.1", 2048, 512, 3, 1, 1, 1, eps, false, &bb->bott,
                      4096, 0)) ||
      (rc = load_ppm_fold(bb, hp, eps)) || (rc = upload(bb, std::vector<float>(2048, 1.0f), &bb->ones)) ||
      (rc = upload(bb, std::vector<float>(2048, 0.0f), &bb->zeros))) {
    cleanup();
    return rc;
  }
  *out = bb;
  return 0;
}

static inline int down2(int x) { return (x - 1) / 2 + 1; }  // 3x3 s2 p1 conv / maxpool output size

struct ConvCall {
  int stage;  // 0 stem, 1-4 layer1-4, 5 PPM, 6 bottleneck (kernel symbol tag)
  const ConvLayer* L;
  const float* x;
  int N, Hi, Wi, x_ld;
  float* y;
  int y_ld, y_off;
  const float* res;
  int res_ld;
  int relu;
  bool out_f32;  // S-layout mode: this call writes fp32 (and takes an fp32 residual)
};

static ConvArgs make_args(const ConvCall& c) {
  ConvArgs a;
  memset(&a, 0, sizeof(a));
  const ConvLayer& L = *c.L;
  a.x = c.x;
  a.w = L.w;
  a.scale = L.scale;
  a.shift = L.shift;
  a.res = c.res;
  a.y = c.y;
  a.N = c.N;
  a.Hi = c.Hi;
  a.Wi = c.Wi;
  a.Ci = L.Ci;
  a.x_ld = c.x_ld;
  a.Ho = (c.Hi + 2 * L.pad - L.dil * (L.k - 1) - 1) / L.stride + 1;
  a.Wo = (c.Wi + 2 * L.pad - L.dil * (L.k - 1) - 1) / L.stride + 1;
  a.Co = L.Co;
  a.kh = a.kw = L.k;
  a.stride = L.stride;
  a.pad = L.pad;
  a.dil = L.dil;
  a.M = c.N * a.Ho * a.Wo;
  a.K = L.k * L.k * L.Ci;
  a.y_ld = c.y_ld;
  a.y_off = c.y_off;
  a.res_ld = c.res_ld;
  a.relu = c.relu;
  return a;
}

// The Winograd output tile the x6 stack takes for a stride-1 3x3 conv by default (0 = the direct
// conv): F(2x2,3x3) for Ci >= 256 (at Ci = 128 the direct conv measured faster).  F(4x4,3x3)
// only on request (CWT_WINO=4): its rounding error is ~20x F(2x2)'s (4e-6 .. 1.2e-5 of max |y|
// per conv against 2-6e-7; the fp32 GEMM's accumulation error, amplified by the transforms), for
// +8 % pipelined throughput (profiles/r5/wino4/)
static int wino_tile_default(int Ci, int Co, int d, int Ho) {
  (void)Co;
  (void)d;
  (void)Ho;
  return Ci >= 256 ? 2 : 0;
}

// One stride-1 3x3 conv (dilation d = padding) in the Winograd form F(m x m, 3x3) on the x6
// matrix-core arithmetic (wino.hip): input transform -> P = (m+2)^2 batched GEMMs
// (conv_igemm_x6, batch P) -> output transform with the conv's BN / residual / ReLU.  us / ul: the
// layer's wino_s / wino_l (m = 2) or wino4_s / wino4_l (m = 4); bm > 0 overrides the GEMMs' tile
// (bm = 1000 * variant + rows, as cwt_debug_conv_s).
static int run_wino_conv(cwt_ctx* ctx, const float* x, int N, int H, int W, int Ci, int Co, int d, int m,
                         const __bf16* us, const __bf16* ul, const float* scale, const float* shift, const float* res,
                         int res_ld, int relu, float* y, int y_ld, int y_off, int stage, hipStream_t st, int bm = 0,
                         int bn = 0) {
  if (m != 2 && m != 4) return fail(CWT_EARG, "winograd: output tile must be 2 or 4");
  const WinoGeom g = wino_geom(N, H, W, d, m);
  if (g.T * Ci * 4 >= (1L << 31) || g.T * Co * 4 >= (1L << 31)) return fail(CWT_EARG, "winograd: plane too large");
  void *V, *Mb;
  const __bf16* zero = nullptr;
  int rc;
  if ((rc = ensure_ws(ctx, "wino.V", (size_t)g.P * g.T * Ci * 4, &V)) ||
      (rc = ensure_ws(ctx, "wino.M", (size_t)g.P * g.T * Co * 4, &Mb)) || (rc = zero_line(ctx, &zero)))
    return rc;
  // sub-records (the executed work of the form): the transforms' algorithmic bytes
  // and the batched GEMMs' executed FLOPs, at profile level 3 only (their event pairs would add
  // ~10 us of gaps to each Winograd conv's own bracket at levels 1 and 2)
  const int plev = 3;
  (void)stage;
  const double vb = 4.0 * g.P * g.T * Ci, mb = 4.0 * g.P * g.T * Co;
  Prof pin(ctx, st, "wino_in " + std::to_string(Ci) + "@" + std::to_string(H), 0.0,
           4.0 * N * H * W * Ci + vb, plev);
  rc = launch_wino_in(x, g, Ci, (float*)V, st);
  pin.end();
  if (rc) return rc;
  ConvSArgs a;
  memset(&a, 0, sizeof(a));
  a.xs = (const __bf16*)V;
  a.ws = us;
  a.ws_lo = ul;
  a.zero = zero;
  a.scale = scale;
  a.shift = shift;
  a.N = 1;
  a.Hi = (int)g.T;
  a.Wi = 1;
  a.Ci = Ci;
  a.Ho = (int)g.T;
  a.Wo = 1;
  a.Co = Co;
  a.kh = a.kw = 1;
  a.stride = 1;
  a.pad = 0;
  a.dil = 1;
  a.M = (int)g.T;
  a.K = Ci;
  a.part = (float*)Mb;
  a.batch = g.P;
  a.xs_bstride = g.T * Ci * 4;
  a.ws_bstride = (long)Co * Ci * 2;
  a.wl_bstride = (long)Co * Ci;
  ConvPlan p = plan_conv_x6_batched(a.M, Co, Ci, g.P);
  if (bm > 0) {
    p.var = bm / 1000;
    p.bm = bm % 1000;
    p.bn = bn;
    if (Co % p.bn) return fail(CWT_EARG, "winograd GEMM tile: Co % bn");
  }
  // the batched GEMMs are the stage-7 (F(2x2)) / stage-8 (F(4x4)) instantiations, the
  // bottleneck's (stage 6) its own: their own rocprofv3 statistics
  Prof pg(ctx, st, "wino_gemm " + std::to_string(Ci) + "x" + std::to_string(Co) + "@" + std::to_string(H),
          2.0 * g.P * g.T * Ci * Co, vb + 6.0 * g.P * Co * Ci + mb, plev);
  rc = launch_conv_x3s(a, p, m == 4 ? 8 : stage == 6 ? 6 : 7, nullptr, 0, st, 6);
  pg.end();
  if (rc) return rc;
  const double ob = 4.0 * N * H * W * Co * (res ? 2.0 : 1.0);
  Prof pout(ctx, st, "wino_out " + std::to_string(Co) + "@" + std::to_string(H), 0.0, mb + ob, plev);
  rc = launch_wino_out((const float*)Mb, g, Co, scale, shift, res, res_ld, relu, y, y_ld, y_off, st);
  pout.end();
  return rc;
}

// Training-mode BN of one extraction (cwt_extract_features_train_bn; bn_train.hip)
struct TrainBn {
  float momentum, drop_p;
  unsigned long long seed;
};

// The whole extractor as a list of conv calls + byte kernels.  dry_run sizes the split-K workspace.
// tb != null: every BN on batch statistics with running-statistic update, Dropout2d on the
// bottleneck output (train.py:184 model.train() before the first support extraction).
// mid (optional, eval mode only): fp32 NHWC copies of the outputs of layer2, layer3 and layer4
// ([N][h][h][512 / 1024 / 2048]; get_feat_list's per-layer features, pspnet.py:272-287)
static int run_extract(cwt_ctx* ctx, const Backbone* bb, const float* img, int N, int S, float* feat,
                       hipStream_t st, const TrainBn* tb = nullptr, float* const* mid = nullptr) {
  // conv arithmetic / activation storage: plain bf16 (cwt_backbone_set_precision), else the
  // context's fp32-accurate mode (S-layout bf16x3 by default)
  const bool b16 = bb->precision == CWT_CONV_BF16;
  // the training-mode BN pass (once per epoch) amplifies conv rounding ~100x through its
  // batch statistics: in fp32 precision it runs the exact-fp32 conv path
  const bool conv_split = ctx->conv_arith == CWT_CONV_ARITH_BF16X3 && !(tb && !b16);
  const bool s_path = b16 || conv_split;  // S-layout / bf16 activations
  const int layout = b16 ? ACT_BF16 : conv_split ? ACT_SPLIT : ACT_F32;
  // the exact-fp32 path (eval mode) runs on the same LDS-DMA conv body (conv_igemm_f32d: fp32
  // NHWC activations, f32 MFMA); CWT_CONV_F32D=0 selects the register-staged conv_igemm_f32
  static const bool f32d_env = !(getenv("CWT_CONV_F32D") && getenv("CWT_CONV_F32D")[0] == '0');
  // fp32 width on the bf16 matrix cores (conv_igemm_x6): f32d's operands, split in registers
  const bool x6 = !s_path && !tb && ctx->conv_arith == CWT_CONV_ARITH_BF16X6;
  const bool f32d = !s_path && !tb && !x6 && f32d_env;
  const bool f32ops = f32d || x6;  // fp32 NHWC operands on the LDS-DMA body
  const bool dma = s_path || f32ops;  // conv_x3s.hip kernels
  const int prec = b16 ? 1 : conv_split ? 3 : x6 ? 6 : 0;
  const int Hs = down2(S), H1 = down2(Hs), h = down2(H1);
  const long sA = std::max({(long)N * Hs * Hs * 128, (long)N * H1 * H1 * 256, (long)N * h * h * 2048});
  const long sT1 = std::max((long)N * H1 * H1 * 128, (long)N * h * h * 512);
  const long sT2 = std::max((long)N * H1 * H1 * 64, (long)N * h * h * 512);
  const long sD = std::max((long)N * H1 * H1 * 256, (long)N * h * h * 2048);
  const long sCol = (long)N * h * 16 * 2048 + (long)N * 16 * 16 * 2048;  // PPM row-segment + block sums
  const long sPool = (long)N * 50 * 2048;
  const long sPpm = (long)N * 50 * 512;
  const long sQ = (long)N * 50 * 4608;
  const long sR = (long)N * 12 * h * 3 * 512;
  const long sF = (long)N * h * h * 512;
  constexpr int kKcPpm = 32, kKcQ = 64;  // K chunk of the two small-M GEMMs
  const long sPartS = std::max((long)(2048 / kKcPpm) * N * 50 * 512, (long)(512 / kKcQ) * N * 50 * 4608);

  // collect every conv call first (to size split-K scratch), then run
  float *A, *B, *T1, *T2, *D, *COL, *POOL, *PPM, *QB, *RB, *FB, *PARTS;
  void* p;
  int rc;
  if ((rc = ensure_ws(ctx, "bb.A", sA * 4, &p))) return rc;
  A = (float*)p;
  if ((rc = ensure_ws(ctx, "bb.B", sA * 4, &p))) return rc;
  B = (float*)p;
  if ((rc = ensure_ws(ctx, "bb.T1", sT1 * 4, &p))) return rc;
  T1 = (float*)p;
  if ((rc = ensure_ws(ctx, "bb.T2", sT2 * 4, &p))) return rc;
  T2 = (float*)p;
  if ((rc = ensure_ws(ctx, "bb.D", sD * 4, &p))) return rc;
  D = (float*)p;
  if ((rc = ensure_ws(ctx, "bb.COL", sCol * 4, &p))) return rc;
  COL = (float*)p;
  if ((rc = ensure_ws(ctx, "bb.POOL", sPool * 4, &p))) return rc;
  POOL = (float*)p;
  if ((rc = ensure_ws(ctx, "bb.PPM", sPpm * 4, &p))) return rc;
  PPM = (float*)p;
  if ((rc = ensure_ws(ctx, "bb.Q", sQ * 4, &p))) return rc;
  QB = (float*)p;
  if ((rc = ensure_ws(ctx, "bb.R", sR * 4, &p))) return rc;
  RB = (float*)p;
  if ((rc = ensure_ws(ctx, "bb.F", sF * 4, &p))) return rc;
  FB = (float*)p;
  if ((rc = ensure_ws(ctx, "bb.PARTS", sPartS * 4, &p))) return rc;
  PARTS = (float*)p;

  std::vector<ConvCall> calls;
  int stage = 0;
  auto cc = [&](const ConvLayer* L, const float* x, int n, int Hi, int Wi, int x_ld, float* y, int y_ld, int y_off,
                const float* res, int res_ld, int relu) {
    ConvCall c{stage, L, x, n, Hi, Wi, x_ld, y, y_ld, y_off, res, res_ld, relu, stage == 6};
    calls.push_back(c);
  };
  // stem conv2/conv3 (conv1 and maxpool are separate kernels, ordered below by index)
  cc(&bb->stem[1], A, N, Hs, Hs, 64, B, 64, 0, nullptr, 0, 1);
  cc(&bb->stem[2], B, N, Hs, Hs, 64, A, 128, 0, nullptr, 0, 1);
  const size_t n_stem_calls = calls.size();
  size_t last_of_layer[4] = {0, 0, 0, 0};  // call index of each layer's last block (mid features)
  float* cur = B;  // maxpool output
  float* other = A;
  int H = H1;
  for (int li = 0; li < 4; ++li) {
    stage = li + 1;
    const int nbk = (int)bb->blocks[li].size();
    for (int bi = 0; bi < nbk; ++bi) {
      const Block& blk = bb->blocks[li][bi];
      const int Cin = blk.c1.Ci;
      const int Ho = (blk.c2.stride == 2) ? down2(H) : H;
      cc(&blk.c1, cur, N, H, H, Cin, T1, blk.c1.Co, 0, nullptr, 0, 1);
      cc(&blk.c2, T1, N, H, H, blk.c2.Ci, T2, blk.c2.Co, 0, nullptr, 0, 1);
      const float* res = cur;
      int res_ld = Cin;
      if (blk.has_down) {
        cc(&blk.down, cur, N, H, H, Cin, D, blk.down.Co, 0, nullptr, 0, 0);
        res = D;
        res_ld = blk.down.Co;
      }
      cc(&blk.c3, T2, N, Ho, Ho, blk.c3.Ci, other, blk.c3.Co, 0, res, res_ld, 1);
      if (bi == nbk - 1) last_of_layer[li] = calls.size() - 1;
      std::swap(cur, other);
      H = Ho;
    }
  }
  const size_t n_backbone_calls = calls.size();
  const float* L4 = cur;  // layer4 output [N][h][h][2048]
  // the bottleneck conv over the layer4 channels; the folded PPM field FB enters as residual
  stage = 6;
  cc(&bb->bott, L4, N, h, h, 2048, feat, 512, 0, FB, 512, 1);

  // split-K scratch
  size_t part_floats = 0;
  std::vector<ConvPlan> plans;
  for (auto& c : calls) {
    ConvArgs a = make_args(c);
    if (b16 && !c.L->w_b) return fail(CWT_ESTATE, "bf16 conv weights missing (Ci % 64 != 0)");
    ConvPlan pl = b16 ? plan_conv_b16(a.M, a.Co, a.K) : conv_split ? plan_conv_x3s(a.M, a.Co, a.K)
                  : x6 ? plan_conv_x6(a.M, a.Co, a.K) : f32d ? plan_conv_f32d(a.M, a.Co, a.K)
                                                         : plan_conv(a.M, a.Co, a.K);
    plans.push_back(pl);
    if (pl.nsplit > 1) part_floats = std::max(part_floats, (size_t)pl.nsplit * a.M * a.Co);
  }
  const __bf16* zero = nullptr;
  if (dma && (rc = zero_line(ctx, &zero))) return rc;
  float *BNPART = nullptr, *BNSC = nullptr;
  size_t bn_part_floats = 0;
  if (tb) {
    bn_part_floats = bn_train_part_floats((long)N * Hs * Hs, 64);
    for (auto& c : calls) {
      ConvArgs a = make_args(c);
      bn_part_floats = std::max(bn_part_floats, bn_train_part_floats(a.M, a.Co));
    }
    if ((rc = ensure_ws(ctx, "bn.part", bn_part_floats * 4, &p))) return rc;
    BNPART = (float*)p;
    if ((rc = ensure_ws(ctx, "bn.bsc", 2 * 2048 * 4, &p))) return rc;
    BNSC = (float*)p;
  }
  // training-mode BN of a raw conv output y (layout / row stride), residual and ReLU after it
  auto bn_train = [&](const ConvLayer* L, void* y, int lay, int ld, long M, const void* res, int res_ld, int relu,
                      float drop_p, long rows_per_image) -> int {
    BnTrainArgs b;
    memset(&b, 0, sizeof(b));
    b.y = y;
    b.layout = lay;
    b.ld = ld;
    b.M = M;
    b.C = L->Co;
    b.res = res;
    b.res_ld = res_ld;
    b.relu = relu;
    b.bn = L->bn;
    b.scale = L->scale;
    b.shift = L->shift;
    b.eps = bb->eps;
    b.momentum = tb->momentum;
    b.drop_p = drop_p;
    b.seed = tb->seed;
    b.rows_per_image = rows_per_image;
    return launch_bn_train(b, BNPART, bn_part_floats, BNSC, st);
  };
  float* PART = nullptr;
  if (part_floats) {
    if ((rc = ensure_ws(ctx, "bb.PART", part_floats * 4, &p))) return rc;
    PART = (float*)p;
  }
  // the Winograd form: stride-1 3x3 layers whose transformed weights were built at load, on
  // images of a pixel stride equal to their channels
  auto c_wino = [&](const ConvCall& c) {
    return (c.L->wino_s || c.L->wino4_s) && c.L->k == 3 && c.L->stride == 1 && c.L->pad == c.L->dil &&
           c.x_ld == c.L->Ci;
  };
  auto run_call = [&](size_t i) -> int {
    ConvArgs a = make_args(calls[i]);
    // training-mode BN: raw conv (scale 1, shift 0); the bottleneck keeps its residual (the
    // raw PPM half of the same conv), every other residual / ReLU moves after the BN
    const bool keep_res = calls[i].stage == 6;
    if (tb) {
      a.scale = bb->ones;
      a.shift = bb->zeros;
      a.relu = 0;
      if (!keep_res) a.res = nullptr;
    }
    // A/B: CWT_WINO=0 every conv direct, 2 / 4 every Winograd-eligible conv in F(2x2) / F(4x4)
    static const int wino_env = getenv("CWT_WINO") && getenv("CWT_WINO")[0] ? atoi(getenv("CWT_WINO")) : -1;
    int wm = x6 && wino_env != 0 && c_wino(calls[i])
                 ? (wino_env == 2 || wino_env == 4 ? wino_env : wino_tile_default(a.Ci, a.Co, a.dil, a.Ho))
                 : 0;
    if (wm && !(wm == 4 ? calls[i].L->wino4_s : calls[i].L->wino_s)) wm = 0;  // form not built for this layer
    const bool wino = wm != 0;
    // the Winograd form's record names its batched GEMM's plan; its FLOPs stay the direct conv's
    // (algorithmic: the roofline prices the conv, not the form that computes it)
    const WinoGeom wg = wino_geom(a.N, a.Hi, a.Wi, a.dil, wm ? wm : 2);
    const ConvPlan pl = wino ? plan_conv_x6_batched((int)wg.T, a.Co, a.Ci, wg.P) : plans[i];
    const double flops = 2.0 * a.M * a.Co * a.K;
    // algorithmic bytes: every operand once; 4 B per element (fp32 or the bf16x3 S-layout),
    // 2 B for the bf16 stack's activations and weights (its fp32 bottleneck output: 4 B)
    const double eb = b16 ? 2.0 : 4.0, ob = calls[i].out_f32 ? 4.0 : eb;
    const double bytes = eb * ((double)a.N * a.Hi * a.Wi * a.Ci + (double)a.Co * a.K) +
                         ob * ((double)a.M * a.Co + (a.res ? (double)a.M * a.Co : 0.0));
    Prof p(ctx, st,
           std::string(b16 ? "conv_igemm_b16<" : conv_split ? "conv_igemm_x3s<" : wino ? (wm == 4 ? "conv_igemm_x6w4<" : "conv_igemm_x6w<")
                       : x6 ? "conv_igemm_x6<" : f32d ? "conv_igemm_f32d<" : "conv_igemm_f32<") +
               std::to_string(pl.bm) + "," +
               std::to_string(pl.bn) + "," +
               std::to_string(calls[i].stage) + ">" +
               (pl.nsplit > 1 ? "+splitk" + std::to_string(pl.nsplit) : std::string()) + " " +
               std::to_string(a.Ci) + "x" + std::to_string(a.Co) + "k" + std::to_string(a.kh) + "s" +
               std::to_string(a.stride) + "d" + std::to_string(a.dil) + "@" + std::to_string(a.Ho),
           flops, bytes, calls[i].stage == 6 ? 1 : 2);
    int r;
    if (wino) {
      const ConvCall& c = calls[i];
      r = run_wino_conv(ctx, c.x, a.N, a.Hi, a.Wi, a.Ci, a.Co, a.dil, wm, wm == 4 ? c.L->wino4_s : c.L->wino_s,
                        wm == 4 ? c.L->wino4_l : c.L->wino_l, a.scale, a.shift, a.res, c.res_ld, a.relu, c.y, c.y_ld,
                        c.y_off, c.stage, st);
    } else if (dma) {
      ConvSArgs sa;
      memset(&sa, 0, sizeof(sa));
      const ConvCall& c = calls[i];
      sa.xs = (const __bf16*)c.x;  // (f32d: the fp32 NHWC map, the same 128-B line geometry)
      sa.ws = b16 ? c.L->w_b : f32d ? (const __bf16*)c.L->w : c.L->w_s;  // x6: hi | mid (+ ws_lo)
      sa.ws_lo = x6 ? c.L->w_l : nullptr;
      sa.zero = zero;
      sa.scale = a.scale;
      sa.shift = a.shift;
      if (c.out_f32 || f32ops) {
        sa.y = c.y;
        sa.y_ld = c.y_ld;
        sa.y_off = c.y_off;
        sa.res = a.res;
        sa.res_ld = c.res_ld;
      } else {
        sa.ys = (__bf16*)c.y;
        sa.res_s = (const __bf16*)a.res;
      }
      sa.relu = a.relu;
      sa.N = a.N;
      sa.Hi = a.Hi;
      sa.Wi = a.Wi;
      sa.Ci = a.Ci;
      sa.Ho = a.Ho;
      sa.Wo = a.Wo;
      sa.Co = a.Co;
      sa.kh = a.kh;
      sa.kw = a.kw;
      sa.stride = a.stride;
      sa.pad = a.pad;
      sa.dil = a.dil;
      sa.M = a.M;
      sa.K = a.K;
      r = launch_conv_x3s(sa, pl, c.stage, PART, part_floats, st, prec);
    } else {
      r = launch_conv(a, pl, calls[i].stage, PART, part_floats, st);
    }
    p.end();
    if (r || !tb) return r;
    const ConvCall& c = calls[i];
    const bool f32 = c.out_f32 || !s_path;
    return bn_train(c.L, c.y, f32 ? ACT_F32 : layout, f32 ? c.y_ld : c.L->Co, a.M, keep_res ? nullptr : c.res,
                    f32 ? c.res_ld : c.L->Co, c.relu, c.stage == 6 ? tb->drop_p : 0.f, (long)a.Ho * a.Wo);
  };

  const long cells = (long)N * 50;
  const double ppm_flops = 2.0 * cells * 512 * 2048 + 2.0 * cells * 4608 * 512 +
                           2.0 * N * 12 * h * 3 * 512 * 3 * 6 + 2.0 * N * h * h * 512 * 36;
  double all_flops = 2.0 * N * Hs * Hs * 64 * 27 + ppm_flops, all_bytes = 0.0;
  for (auto& c : calls) {
    ConvArgs a = make_args(c);
    all_flops += 2.0 * a.M * a.Co * a.K;
    all_bytes += 4.0 * ((double)a.N * a.Hi * a.Wi * a.Ci + (double)a.Co * a.K + (double)a.M * a.Co);
  }
  Prof whole(ctx, st, "extract_features N=" + std::to_string(N) + " S=" + std::to_string(S), all_flops, all_bytes, 1);
  {
    Prof p(ctx, st, "stem_conv1 3x64k3s2", 2.0 * N * Hs * Hs * 64 * 27, 4.0 * ((double)N * 3 * S * S + (double)N * Hs * Hs * 64));
    if ((rc = launch_stem_conv1(img, N, S, bb->stem[0].w, tb ? bb->ones : bb->stem[0].scale,
                                tb ? bb->zeros : bb->stem[0].shift, A, Hs, st, layout, tb ? 0 : 1)))
      return rc;
    p.end();
    if (tb && (rc = bn_train(&bb->stem[0], A, layout, 64, (long)N * Hs * Hs, nullptr, 0, 1, 0.f, (long)Hs * Hs)))
      return rc;
  }
  for (size_t i = 0; i < n_stem_calls; ++i)
    if ((rc = run_call(i))) return rc;
  {
    Prof p(ctx, st, "maxpool3s2", 0.0, 4.0 * ((double)N * Hs * Hs * 128 + (double)N * H1 * H1 * 128));
    if ((rc = layout == ACT_BF16    ? launch_maxpool3s2_b16((const __bf16*)A, N, Hs, Hs, 128, (__bf16*)B, H1, H1, st)
              : layout == ACT_SPLIT ? launch_maxpool3s2_s((const __bf16*)A, N, Hs, Hs, 128, (__bf16*)B, H1, H1, st)
                                    : launch_maxpool3s2(A, N, Hs, Hs, 128, B, H1, H1, st)))
      return rc;
    p.end();
  }
  for (size_t i = n_stem_calls; i < n_backbone_calls; ++i) {
    if ((rc = run_call(i))) return rc;
    for (int li = 1; li < 4 && mid; ++li) {  // layer2 .. layer4 outputs, before the buffer is reused
      if (i != last_of_layer[li] || !mid[li - 1]) continue;
      const ConvCall& c = calls[i];
      const ConvArgs a = make_args(c);
      const long P = (long)a.M;
      if (layout == ACT_SPLIT)
        rc = launch_unsplit_act((const __bf16*)c.y, P, a.Co, mid[li - 1], a.Co, st);
      else if (layout == ACT_BF16)
        rc = launch_widen_bf16((const __bf16*)c.y, P * a.Co, mid[li - 1], st);
      else {
        const hipError_t e = hipMemcpyAsync(mid[li - 1], c.y, (size_t)P * a.Co * 4, hipMemcpyDeviceToDevice, st);
        rc = e == hipSuccess ? 0 : fail((int)e, "mid feature copy");
      }
      if (rc) return rc;
    }
  }
  {
    Prof p(ctx, st, "ppm_pool", 0.0, 4.0 * ((double)N * h * h * 2048 + (double)N * 50 * 2048));
    if ((rc = launch_ppm(L4, N, h, h, 2048, kBins, 4, COL, POOL, st, layout))) return rc;
    p.end();
  }
  int Mb[4];
  const float *Wp[4], *Wq[4], *Sc[4], *Sh[4];
  static const bool ppm_splitk = getenv("CWT_PPM_SPLITK") != nullptr;  // A/B: the split-K form
  const bool few_cells = cells <= kPpmGemmMaxRows && !ppm_splitk;
  for (int i = 0; i < 4; ++i) {
    Mb[i] = N * kBins[i] * kBins[i];
    Wp[i] = bb->ppm_wt[i];
    Wq[i] = tb ? bb->ppm_q_raw[i] : bb->ppm_q[i];
    Sc[i] = bb->ppm[i].scale;
    Sh[i] = bb->ppm[i].shift;
  }
  {  // PPM 1x1 conv + BN + ReLU over the pooled cells (pspnet.py:27-29)
    Prof p(ctx, st, "ppm_conv smallm 2048x512", 2.0 * cells * 512 * 2048, 4.0 * (4.0 * 2048 * 512 + cells * 2560.0));
    if ((rc = few_cells ? launch_ppm_gemm(POOL, 2048, Wp, Mb, 4, 512, 2048, tb ? nullptr : Sc, tb ? nullptr : Sh, PARTS,
                                          (size_t)sPartS, PPM, st)
                        : launch_smallm_gemm(POOL, 2048, Wp, Mb, 4, 512, 2048, kKcPpm, PARTS, (size_t)sPartS,
                                             tb ? nullptr : Sc, tb ? nullptr : Sh, PPM, st)))
      return rc;
    p.end();
  }
  if (tb) {  // the PPM BNs on the batch statistics of their pooled cells
    long row0 = 0;
    for (int i = 0; i < 4; ++i) {
      if ((rc = bn_train(&bb->ppm[i], PPM + row0 * 512, ACT_F32, 512, Mb[i], nullptr, 0, 1, 0.f,
                         (long)kBins[i] * kBins[i])))
        return rc;
      row0 += Mb[i];
    }
  }
  {  // per-tap products of the bottleneck's PPM channels with the cells
    Prof p(ctx, st, "ppm_fold_q smallm 512x4608", 2.0 * cells * 4608 * 512, 4.0 * (4.0 * 512 * 4608 + cells * 5120.0));
    if ((rc = few_cells ? launch_ppm_gemm(PPM, 512, Wq, Mb, 4, 4608, 512, nullptr, nullptr, PARTS, (size_t)sPartS, QB, st)
                        : launch_smallm_gemm(PPM, 512, Wq, Mb, 4, 4608, 512, kKcQ, PARTS, (size_t)sPartS, nullptr,
                                             nullptr, QB, st)))
      return rc;
    p.end();
  }
  {  // separable interpolation of the per-tap products: the PPM half of the bottleneck conv
    Prof p(ctx, st, "ppm_field", 2.0 * N * 12 * h * 3 * 512 * 3 * 6 + 2.0 * N * h * h * 512 * 36,
           4.0 * ((double)cells * 4608 + 2.0 * sR + sF));
    if ((rc = launch_ppm_field(QB, N, h, h, kBins, RB, FB, st))) return rc;
    p.end();
  }
  rc = run_call(n_backbone_calls);
  whole.end();
  if (!rc && tb)  // refold the bottleneck's new eval BN scale into the PPM-branch weights
    for (int i = 0; i < 4 && !rc; ++i)
      rc = launch_scale_cols(bb->ppm_q_raw[i], bb->ppm_q[i], 512L * 4608, 512, bb->bott.scale, st);
  return rc;
}

// device of a context (pretrain.hip)
int ctx_device(const cwt_ctx* ctx) { return ctx->device; }

}  // namespace cwt

using namespace cwt;

extern "C" {

#ifndef CWT_SRC_HASH
#define CWT_SRC_HASH "unknown"
#endif
// the content hash of the HIP sources and headers this library was built from (build.py
// source_hash); _lib.load_library refuses a library whose hash differs from the tree's
const char* cwt_version(void) { return "libcwt 0.2 (gfx950) src=" CWT_SRC_HASH; }

const char* cwt_last_error(void) { return g_err.c_str(); }

int cwt_ctx_create(int device, cwt_ctx** out) {
  if (!out) return fail(CWT_EARG, "out is NULL");
  int n = 0;
  CWT_HIP(hipGetDeviceCount(&n));
  if (device < 0 || device >= n) return fail(CWT_EARG, "no such device");
  CWT_HIP(hipSetDevice(device));
  cwt_ctx* c = new cwt_ctx();
  c->device = device;
  const char* g = getenv("CWT_ADAPT_GRAPH");
  c->use_graph = !(g && g[0] == '0');
  const char* cv = getenv("CWT_CONV");
  const std::string mode = cv ? std::string(cv) : std::string("x6");
  if (mode != "x6" && mode != "x3s" && mode != "f32") {
    delete c;
    return fail(CWT_EARG, "CWT_CONV must be x6 (default), x3s or f32");
  }
  c->conv_arith = mode == "x6" ? CWT_CONV_ARITH_BF16X6 : mode == "x3s" ? CWT_CONV_ARITH_BF16X3 : CWT_CONV_ARITH_F32;
  if (hipHostMalloc((void**)&c->status_host, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer((void**)&c->status_dev, c->status_host, 0) != hipSuccess) {
    if (c->status_host) (void)hipHostFree(c->status_host);
    delete c;
    return fail(CWT_ESTATE, "cwt_ctx_create: mapped status word");
  }
  for (int i = 0; i < 16; ++i) ((volatile unsigned*)c->status_host)[i] = 0u;
  *out = c;
  return 0;
}

int cwt_ctx_destroy(cwt_ctx* ctx) {
  if (!ctx) return 0;
  (void)hipSetDevice(ctx->device);
  (void)hipDeviceSynchronize();
  for (auto& kv : ctx->ws)
    if (kv.second.p) (void)hipFree(kv.second.p);
  if (ctx->status_host) (void)hipHostFree(ctx->status_host);
  if (ctx->fstamps) (void)hipFree(ctx->fstamps);
  if (ctx->aux) (void)hipStreamDestroy(ctx->aux);
  if (ctx->ev_fork) (void)hipEventDestroy(ctx->ev_fork);
  if (ctx->ev_join) (void)hipEventDestroy(ctx->ev_join);
  delete ctx;
  return 0;
}

int cwt_ctx_status(cwt_ctx* ctx, uint32_t* status, int clear) {
  if (!ctx || !status) return fail(CWT_EARG, "null argument");
  // one word per failure source (plain stores from the kernels, no PCIe atomics): word 0 the inner
  // loop, word 1 the post-loop tail; the caller sees their OR
  volatile unsigned* w = ctx->status_host;
  const unsigned w0 = w[0], w1 = w[1];
  *status = w0 | w1;
  // the tail aborted, or the inner loop did (a fused tail then never ran its barriers): the tail's
  // counters are re-zeroed before the next tail
  if (w0 || w1) ctx->tail_epoch = ~0u;
  if (clear) {
    w[0] = 0u;
    w[1] = 0u;
  }
  return 0;
}

int cwt_backbone_load(cwt_ctx* ctx, int layers, int n_tensors, const char* const* names,
                      const float* const* host_data, const int64_t* numel, float bn_eps, cwt_backbone** out) {
  if (!ctx || !names || !host_data || !numel || n_tensors <= 0 || !out) return fail(CWT_EARG, "null argument");
  CWT_HIP(hipSetDevice(ctx->device));
  HostParams hp;
  for (int i = 0; i < n_tensors; ++i) hp.m[names[i]] = {host_data[i], numel[i]};
  Backbone* bb = nullptr;
  int rc = load_backbone(layers, hp, bn_eps, &bb);
  if (rc) return rc;
  bb->device = ctx->device;
  *out = reinterpret_cast<cwt_backbone*>(bb);
  return 0;
}

int cwt_backbone_destroy(cwt_backbone* handle) {
  Backbone* bb = reinterpret_cast<Backbone*>(handle);
  if (!bb) return 0;
  (void)hipSetDevice(bb->device);
  (void)hipDeviceSynchronize();
  for (void* p : bb->allocs) (void)hipFree(p);
  delete bb;
  return 0;
}

int cwt_backbone_set_precision(cwt_backbone* handle, int precision) {
  Backbone* bb = reinterpret_cast<Backbone*>(handle);
  if (!bb) return fail(CWT_EARG, "backbone is NULL");
  if (precision != CWT_CONV_FP32 && precision != CWT_CONV_BF16)
    return fail(CWT_EARG, "precision must be CWT_CONV_FP32 (0) or CWT_CONV_BF16 (1)");
  bb->precision = precision;
  return 0;
}

int cwt_extract_features(cwt_ctx* ctx, const cwt_backbone* handle, const float* img, int N, int S, float* feat,
                         void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  const Backbone* bb = reinterpret_cast<const Backbone*>(handle);
  if (!bb) return fail(CWT_ESTATE, "backbone is NULL (cwt_backbone_load)");
  if (bb->device != ctx->device) return fail(CWT_EARG, "backbone and context are on different devices");
  CWT_CHECK(img && feat, "null buffer");
  CWT_CHECK(N >= 1 && S >= 9 && (S - 1) % 8 == 0, "need N >= 1 and (S-1) % 8 == 0 (pspnet.py:150)");
  CWT_HIP(hipSetDevice(ctx->device));
  return run_extract(ctx, bb, img, N, S, feat, (hipStream_t)stream);
}

int cwt_extract_features_mid(cwt_ctx* ctx, const cwt_backbone* handle, const float* img, int N, int S, float* feat,
                             float* l2, float* l3, float* l4, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  const Backbone* bb = reinterpret_cast<const Backbone*>(handle);
  if (!bb) return fail(CWT_ESTATE, "backbone is NULL (cwt_backbone_load)");
  if (bb->device != ctx->device) return fail(CWT_EARG, "backbone and context are on different devices");
  CWT_CHECK(img && feat, "null buffer");
  CWT_CHECK(N >= 1 && S >= 9 && (S - 1) % 8 == 0, "need N >= 1 and (S-1) % 8 == 0 (pspnet.py:150)");
  CWT_HIP(hipSetDevice(ctx->device));
  float* const mid[3] = {l2, l3, l4};
  return run_extract(ctx, bb, img, N, S, feat, (hipStream_t)stream, nullptr, mid);
}

int cwt_extract_features_train_bn(cwt_ctx* ctx, cwt_backbone* handle, const float* img, int N, int S, float* feat,
                                  float momentum, float dropout_p, uint64_t seed, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  Backbone* bb = reinterpret_cast<Backbone*>(handle);
  if (!bb) return fail(CWT_ESTATE, "backbone is NULL (cwt_backbone_load)");
  if (bb->device != ctx->device) return fail(CWT_EARG, "backbone and context are on different devices");
  CWT_CHECK(img && feat, "null buffer");
  CWT_CHECK(N >= 1 && S >= 9 && (S - 1) % 8 == 0, "need N >= 1 and (S-1) % 8 == 0 (pspnet.py:150)");
  CWT_CHECK(N >= 2, "Expected more than 1 value per channel when training (the PPM bin-1 BatchNorm2d needs N >= 2)");
  CWT_CHECK(momentum >= 0.f && momentum <= 1.f && dropout_p >= 0.f && dropout_p < 1.f, "bad momentum / dropout_p");
  CWT_HIP(hipSetDevice(ctx->device));
  TrainBn tb{momentum, dropout_p, (unsigned long long)seed};
  return run_extract(ctx, bb, img, N, S, feat, (hipStream_t)stream, &tb);
}

int cwt_backbone_read_bn(const cwt_backbone* handle, const char* name, float* out, int C) {
  const Backbone* bb = reinterpret_cast<const Backbone*>(handle);
  if (!bb) return fail(CWT_ESTATE, "backbone is NULL (cwt_backbone_load)");
  CWT_CHECK(name && out, "null argument");
  auto it = bb->bn_by_name.find(name);
  if (it == bb->bn_by_name.end()) return fail(CWT_EARG, std::string("no BatchNorm2d named ") + name);
  CWT_CHECK(it->second.second == C, "C does not match the BatchNorm2d's channel count");
  CWT_HIP(hipSetDevice(bb->device));
  CWT_HIP(hipDeviceSynchronize());
  CWT_HIP(hipMemcpy(out, it->second.first, sizeof(float) * 4 * C, hipMemcpyDeviceToHost));
  return 0;
}

int cwt_preprocess_image(cwt_ctx* ctx, const void* src, int src_dtype, int H, int W, int S, const float* mean,
                         const float* std_, const float* pad, int flip_h, int flip_v, float* dst, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(src && dst && mean && std_, "null argument");
  CWT_CHECK(src_dtype == CWT_U8 || src_dtype == CWT_F32, "src_dtype must be CWT_U8 or CWT_F32");
  CWT_CHECK(H >= 1 && W >= 1 && S >= 8, "bad sizes");
  CWT_HIP(hipSetDevice(ctx->device));
  return launch_episode_image(src, src_dtype == CWT_F32, H, W, S, mean, std_, pad, flip_h, flip_v, dst,
                              (hipStream_t)stream);
}

int cwt_preprocess_label(cwt_ctx* ctx, const uint8_t* src, int H, int W, int S, int class_chosen, int flip_h,
                         int flip_v, int64_t* dst, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(src && dst, "null argument");
  CWT_CHECK(H >= 1 && W >= 1 && S >= 8, "bad sizes");
  CWT_HIP(hipSetDevice(ctx->device));
  return launch_episode_label(src, H, W, S, class_chosen, flip_h, flip_v, (long long*)dst, (hipStream_t)stream);
}

size_t cwt_workspace_bytes(cwt_ctx* ctx) { return ctx ? ctx->ws_total : 0; }

int cwt_inner_adapt_batch(cwt_ctx* ctx, const float* f_s, const int64_t* s_label, int E, int n, int h, int w, int C,
                          int S, float lr, int iters, float* W_inout, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(f_s && s_label && W_inout, "null buffer");
  CWT_CHECK(C == 512, "C must be 512");
  CWT_CHECK(E >= 1 && E <= 64 && n >= 1 && h >= 2 && w >= 2 && iters >= 0, "bad sizes");
  CWT_CHECK(S - 1 == 8 * (h - 1) && S - 1 == 8 * (w - 1), "need S-1 == 8*(h-1) == 8*(w-1)");
  CWT_HIP(hipSetDevice(ctx->device));
  void *fws, *lbl, *sc, *acc, *wb, *dargs;
  size_t b_f, b_lbl, b_sc, b_acc, b_wb, b_args;
  adapt_ws_sizes(E, n, h, w, S, &b_f, &b_lbl, &b_sc, &b_acc, &b_wb, &b_args);
  int rc;
  if ((rc = ensure_ws(ctx, "adapt.f", b_f, &fws))) return rc;
  if ((rc = ensure_ws(ctx, "adapt.args", b_args, &dargs))) return rc;
  if ((rc = ensure_ws(ctx, "adapt.lbl", b_lbl, &lbl))) return rc;
  if ((rc = ensure_ws(ctx, "adapt.sc", b_sc, &sc))) return rc;
  if ((rc = ensure_ws(ctx, "adapt.acc", b_acc, &acc))) return rc;  // [E][3][ADAPT_RMAX][512]
  if ((rc = ensure_ws(ctx, "adapt.wbuf", b_wb, &wb))) return rc;
  // algorithmic work: per step 2 x (2*2*C*h*w*n) FLOPs; minimal bytes = f_s + labels once per step
  Prof p(ctx, (hipStream_t)stream,
         "inner_adapt x" + std::to_string(iters) + (E > 1 ? " E=" + std::to_string(E) : "") + " [" +
             adapt_kernel_name(E, n, h, w, iters, ctx->adapt_upw) + "]",
         (double)E * iters * 2.0 * (4.0 * C * h * w * n), (double)E * iters * ((double)n * h * w * C * 4 + (double)n * S * S),
         1);
  // the persistent kernel alone (no label prep / setup kernels): the launch rocprofv3 times
  const char* kname = adapt_kernel_name(E, n, h, w, iters, ctx->adapt_upw);
  const bool persist_k = strncmp(kname, "adapt_persist", 13) == 0;
  Prof pk(ctx, (hipStream_t)stream, std::string("inner_adapt_kernel [") + kname + "]",
          (double)E * iters * 2.0 * (4.0 * C * h * w * n), (double)E * iters * ((double)n * h * w * C * 4 + (double)n * S * S),
          1, persist_k);
  rc = launch_adapt(f_s, s_label, E, n, h, w, S, lr, iters, W_inout, (float*)fws, (uint8_t*)lbl, (AdaptScalars*)sc,
                    (float*)acc, (float*)wb, (AdaptDevArgs*)dargs, ctx->use_graph ? &ctx->adapt_graphs : nullptr,
                    ctx->adapt_upw, ctx->status_dev, ctx->adapt_spin_limit, (hipStream_t)stream, pk.ev0(), pk.ev1());
  p.end();
  return rc;
}

int cwt_inner_adapt(cwt_ctx* ctx, const float* f_s, const int64_t* s_label, int n, int h, int w, int C, int S,
                    float lr, int iters, float* W_inout, void* stream) {
  return cwt_inner_adapt_batch(ctx, f_s, s_label, 1, n, h, w, C, S, lr, iters, W_inout, stream);
}

int cwt_normalize(cwt_ctx* ctx, const float* f, int B, int P_per_b, int C, float* out, const float* W0,
                  float* logits0, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(f && out && C == 512 && B >= 1 && P_per_b >= 1, "bad arguments");
  CWT_CHECK((W0 == nullptr) == (logits0 == nullptr), "W0 and logits0 go together");
  CWT_HIP(hipSetDevice(ctx->device));
  return launch_normalize(f, B, P_per_b, out, W0, logits0, (hipStream_t)stream);
}

size_t cwt_attention_saved_floats(int B, int hw, int C, int H) { return attention_saved_floats(B, hw, C, H); }

int cwt_attention_fwd_train(cwt_ctx* ctx, const float* q, const float* f, int B, int hw, int C, int H,
                            const float* w_qkvs, const float* fc_w, const float* fc_b, const float* ln_w,
                            const float* ln_b, float* out, float* saved, float attn_dropout, float out_dropout,
                            uint64_t seed, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(q && f && w_qkvs && fc_w && fc_b && ln_w && ln_b && out, "null buffer");
  CWT_CHECK(B >= 1 && B <= 4 && hw >= 1 && C == 512, "need 1 <= B <= 4, C == 512");
  CWT_CHECK(attn_dropout >= 0.f && attn_dropout < 1.f && out_dropout >= 0.f && out_dropout < 1.f,
            "dropout probabilities must lie in [0, 1)");
  CWT_HIP(hipSetDevice(ctx->device));
  void* ws;
  int rc;
  if ((rc = ensure_ws(ctx, "attn.ws", attention_ws_floats(B, hw, C, H) * 4, &ws))) return rc;
  // reference-formulation FLOPs: k/v projections 2 x 2*hw*C*C*H + QK^T/AV 2 x 2*H*2*hw*C
  Prof p(ctx, (hipStream_t)stream, "attention_fwd",
         (double)B * (2.0 * 2.0 * hw * C * C * H + 2.0 * 2.0 * H * 2.0 * hw * C),
         4.0 * ((double)B * hw * C + 2.0 * H * C * C + 2.0 * C), 1);
  rc = attention_fwd(q, f, B, hw, C, H, w_qkvs, fc_w, fc_b, ln_w, ln_b, out, saved, (float*)ws, (hipStream_t)stream,
                     attn_dropout, out_dropout, (unsigned long long)seed);
  p.end();
  return rc;
}

int cwt_attention_fwd(cwt_ctx* ctx, const float* q, const float* f, int B, int hw, int C, int H,
                      const float* w_qkvs, const float* fc_w, const float* fc_b, const float* ln_w, const float* ln_b,
                      float* out, float* saved, void* stream) {
  return cwt_attention_fwd_train(ctx, q, f, B, hw, C, H, w_qkvs, fc_w, fc_b, ln_w, ln_b, out, saved, 0.f, 0.f, 0,
                                 stream);
}

int cwt_attention_bwd_train(cwt_ctx* ctx, const float* q, const float* f, int B, int hw, int C, int H,
                            const float* w_qkvs, const float* fc_w, const float* fc_b, const float* ln_w,
                            const float* ln_b, const float* saved, const float* d_out, float* g_w_qkvs, float* g_fc_w,
                            float* g_fc_b, float* g_ln_w, float* g_ln_b, float attn_dropout, float out_dropout,
                            uint64_t seed, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(q && f && w_qkvs && fc_w && fc_b && ln_w && ln_b && saved && d_out, "null buffer");
  CWT_CHECK(g_w_qkvs && g_fc_w && g_fc_b && g_ln_w && g_ln_b, "null gradient buffer");
  CWT_CHECK(B >= 1 && B <= 4 && hw >= 1 && C == 512, "need 1 <= B <= 4, C == 512");
  CWT_CHECK(attn_dropout >= 0.f && attn_dropout < 1.f && out_dropout >= 0.f && out_dropout < 1.f,
            "dropout probabilities must lie in [0, 1)");
  CWT_HIP(hipSetDevice(ctx->device));
  void* ws;
  int rc;
  if ((rc = ensure_ws(ctx, "attn.bws", attention_bwd_ws_floats(B, hw, C, H) * 4, &ws))) return rc;
  return attention_bwd(q, f, B, hw, C, H, w_qkvs, fc_w, fc_b, ln_w, ln_b, saved, d_out, g_w_qkvs, g_fc_w, g_fc_b,
                       g_ln_w, g_ln_b, (float*)ws, (hipStream_t)stream, attn_dropout, out_dropout,
                       (unsigned long long)seed);
}

int cwt_attention_bwd(cwt_ctx* ctx, const float* q, const float* f, int B, int hw, int C, int H,
                      const float* w_qkvs, const float* fc_w, const float* fc_b, const float* ln_w, const float* ln_b,
                      const float* saved, const float* d_out, float* g_w_qkvs, float* g_fc_w, float* g_fc_b,
                      float* g_ln_w, float* g_ln_b, void* stream) {
  return cwt_attention_bwd_train(ctx, q, f, B, hw, C, H, w_qkvs, fc_w, fc_b, ln_w, ln_b, saved, d_out, g_w_qkvs,
                                 g_fc_w, g_fc_b, g_ln_w, g_ln_b, 0.f, 0.f, 0, stream);
}

int cwt_attention_infer(cwt_ctx* ctx, const float* q, const float* f, int B, int hw, int C, int H,
                        const float* w_qkvs, const float* fc_w, const float* fc_b, const float* ln_w,
                        const float* ln_b, int64_t params_version, float* out, float* inv_norm, float* logits0,
                        void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(q && f && w_qkvs && fc_w && fc_b && ln_w && ln_b && out && inv_norm, "null buffer");
  CWT_CHECK(B >= 1 && B <= 4 && hw >= 1 && hw <= 512 * 32 && C == 512 && H == 4,
            "need 1 <= B <= 4, 1 <= hw <= 16384, C == 512, H == 4");
  CWT_HIP(hipSetDevice(ctx->device));
  const hipStream_t st = (hipStream_t)stream;
  void *fold, *ws;
  int rc;
  if ((rc = ensure_ws(ctx, "attn.fold", attention_fold_floats(C, H) * 4, &fold))) return rc;
  if ((rc = ensure_ws(ctx, "attn.iws", std::max(attention_infer_ws_floats(B, hw, C, H), (size_t)4 << 20) * 4, &ws)))
    return rc;
  Prof p(ctx, st, "attention_fwd", (double)B * (2.0 * 2.0 * hw * C * C * H + 2.0 * 2.0 * H * 2.0 * hw * C),
         4.0 * ((double)B * hw * C + 2.0 * H * C * C + 2.0 * C), 1);
  if (ctx->fold_w != w_qkvs || ctx->fold_fc != fc_w || ctx->fold_ver != params_version || ctx->fold_H != H) {
    if ((rc = attention_fold(w_qkvs, fc_w, C, H, (float*)fold, (float*)ws, (size_t)4 << 20, st))) return rc;
    ctx->fold_w = w_qkvs;
    ctx->fold_fc = fc_w;
    ctx->fold_ver = params_version;
    ctx->fold_H = H;
  }
  rc = attention_infer(q, f, B, hw, C, H, (const float*)fold, fc_b, ln_w, ln_b, out, inv_norm, logits0, (float*)ws, st);
  p.end();
  return rc;
}

int cwt_episode_tail(cwt_ctx* ctx, const float* q, const float* f, int B, int h, int w, int S, const int64_t* q_label,
                     const float* w_qkvs, const float* fc_w, const float* fc_b, const float* ln_w, const float* ln_b,
                     int64_t params_version, float* out, float* logits, float* logits0, float* iut, double* ce,
                     float* iut0, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(q && f && q_label && w_qkvs && fc_w && fc_b && ln_w && ln_b && out && logits && logits0 && iut && ce && iut0,
            "null buffer");
  const int hw = h * w;
  CWT_CHECK(B >= 1 && B <= 4 && h >= 1 && w >= 1 && hw <= 512 * 32 && S - 1 == 8 * (h - 1) && S - 1 == 8 * (w - 1),
            "need 1 <= B <= 4, h*w <= 16384, S - 1 == 8 (h - 1) == 8 (w - 1)");
  CWT_HIP(hipSetDevice(ctx->device));
  const hipStream_t st = (hipStream_t)stream;
  constexpr int C = 512, H = 4;
  int cu = 0;
  CWT_HIP(hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, ctx->device));
  // G co-resident 512-thread workgroups (~54 KB of LDS each): the whole chip (up to 256)
  // on a context that runs alone; 64 on one whose inner loop shares the chip with another
  // stream's extractor pass (cwt_ctx_set_adapt_units >= 2: EpisodePipeline's adapt context).
  // CWT_TAIL_G for A/B
  int G = std::min(ctx->adapt_upw >= 2 ? 64 : 256, cu);
  if (const char* gs = getenv("CWT_TAIL_G")) G = std::max(1, std::min(atoi(gs), cu));
  void *fold, *ws, *cnt;
  int rc;
  if ((rc = ensure_ws(ctx, "attn.fold", attention_fold_floats(C, H) * 4, &fold))) return rc;
  if ((rc = ensure_ws(ctx, "tail.ws", std::max(episode_tail_ws_floats(B, hw, G), (size_t)4 << 20) * 4, &ws))) return rc;
  if ((rc = ensure_ws(ctx, "tail.cnt", episode_tail_cnt_words() * 4, &cnt))) return rc;
  // phase record (the fold when the parameters changed + the launch) and the kernel alone
  Prof p(ctx, st, "post_loop_tail", (double)B * (2.0 * 2.0 * hw * C * C * H + 2.0 * 2.0 * H * 2.0 * hw * C),
         4.0 * ((double)B * hw * C + 2.0 * H * C * C + 2.0 * C), 1);
  Prof pk(ctx, st, "episode_tail_kernel", (double)B * (2.0 * 2.0 * hw * C * C * H + 2.0 * 2.0 * H * 2.0 * hw * C),
          4.0 * ((double)B * hw * C * 2 + 2.0 * H * C * C) + 9.0 * B * S * S, 1, true);
  if (ctx->fold_w != w_qkvs || ctx->fold_fc != fc_w || ctx->fold_ver != params_version || ctx->fold_H != H) {
    if ((rc = attention_fold(w_qkvs, fc_w, C, H, (float*)fold, (float*)ws, (size_t)4 << 20, st))) return rc;
    ctx->fold_w = w_qkvs;
    ctx->fold_fc = fc_w;
    ctx->fold_ver = params_version;
    ctx->fold_H = H;
  }
  if (ctx->tail_epoch > episode_tail_max_epoch(G) || ctx->tail_G != G) {  // fresh, wrapped, aborted or re-sized
    CWT_HIP(hipMemsetAsync(cnt, 0, episode_tail_cnt_words() * 4, st));
    ctx->tail_epoch = 0;
    ctx->tail_G = G;
  }
  void* stamps = nullptr;  // timing study (CWT_TAIL_STAMPS=1): per-workgroup phase stamps (cwt_debug_tail_stamps)
  if (getenv("CWT_TAIL_STAMPS") && getenv("CWT_TAIL_STAMPS")[0] == '1' &&
      (rc = ensure_ws(ctx, "tail.stamps", (size_t)G * 16 * 8, &stamps)))
    return rc;
  ctx->tail_stamp_G = stamps ? G : 0;
  if (pk.ev0()) CWT_HIP(hipEventRecord(pk.ev0(), st));
  rc = launch_episode_tail(q, f, B, hw, h, w, S, q_label, (const float*)fold, fc_b, ln_w, ln_b, out, logits, logits0,
                           iut, ce, iut0, (float*)ws, (unsigned*)cnt, ctx->tail_epoch++, G, ctx->adapt_spin_limit,
                           ctx->status_dev + 1, st, (unsigned long long*)stamps);  // the tail's status word
  if (pk.ev1()) CWT_HIP(hipEventRecord(pk.ev1(), st));
  p.end();
  return rc;
}

// cwt_inner_adapt_tail fuses the tail into the loop's launch where the loop runs as the two-unit
// register form (EpisodePipeline's adapt context) in its product instantiation
static bool fused_tail_applies(cwt_ctx* ctx, int n, int h, int w, int iters) {
  const char* kname = adapt_kernel_name(1, n, h, w, iters, ctx->adapt_upw);
  const char* dbg = getenv("CWT_ADAPT_DBG");
  const char* fz = getenv("CWT_FUSED_LOOP_TAIL");
  const char* tst = getenv("CWT_TAIL_STAMPS");
  return strcmp(kname, "adapt_persist_kernel<5") == 0 && !(dbg && atoi(dbg) != 0) && !(fz && fz[0] == '0') &&
         !(tst && tst[0] == '1');
}

int cwt_inner_adapt_tail(cwt_ctx* ctx, const float* f_s, const int64_t* s_label, int n, int h, int w, int C, int S,
                         float lr, int iters, float* W_inout, const float* f_q, const int64_t* q_label,
                         const float* w_qkvs, const float* fc_w, const float* fc_b, const float* ln_w,
                         const float* ln_b, int64_t params_version, float* out, float* logits, float* logits0,
                         float* iut, double* ce, float* iut0, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(f_s && s_label && W_inout && f_q && q_label && w_qkvs && fc_w && fc_b && ln_w && ln_b && out && logits &&
                logits0 && iut && ce && iut0,
            "null buffer");
  CWT_CHECK(C == 512, "C must be 512");
  CWT_CHECK(n >= 1 && h >= 2 && w >= 2 && iters >= 0 && h * w <= 512 * 32, "bad sizes");
  CWT_CHECK(S - 1 == 8 * (h - 1) && S - 1 == 8 * (w - 1), "need S-1 == 8*(h-1) == 8*(w-1)");
  CWT_HIP(hipSetDevice(ctx->device));
  // fused where the loop runs as the two-unit register form (EpisodePipeline's adapt context) in
  // its product instantiation; everything else (and CWT_FUSED_LOOP_TAIL=0) runs the two calls
  if (!fused_tail_applies(ctx, n, h, w, iters)) {
    int rc = cwt_inner_adapt(ctx, f_s, s_label, n, h, w, C, S, lr, iters, W_inout, stream);
    if (rc) return rc;
    return cwt_episode_tail(ctx, W_inout, f_q, 1, h, w, S, q_label, w_qkvs, fc_w, fc_b, ln_w, ln_b, params_version, out,
                            logits, logits0, iut, ce, iut0, stream);
  }
  const hipStream_t st = (hipStream_t)stream;
  constexpr int H = 4;
  const int hw = h * w;
  const int G = adapt_persist_workgroups(1, n, h, w, iters, ctx->adapt_upw);
  CWT_CHECK(G >= 1 && G <= 512, "fused tail: loop geometry");
  // the loop's workspaces (cwt_inner_adapt_batch)
  void *fws, *lbl, *sc, *acc, *wb, *dargs;
  size_t b_f, b_lbl, b_sc, b_acc, b_wb, b_args;
  adapt_ws_sizes(1, n, h, w, S, &b_f, &b_lbl, &b_sc, &b_acc, &b_wb, &b_args);
  int rc;
  if ((rc = ensure_ws(ctx, "adapt.f", b_f, &fws)) || (rc = ensure_ws(ctx, "adapt.args", b_args, &dargs)) ||
      (rc = ensure_ws(ctx, "adapt.lbl", b_lbl, &lbl)) || (rc = ensure_ws(ctx, "adapt.sc", b_sc, &sc)) ||
      (rc = ensure_ws(ctx, "adapt.acc", b_acc, &acc)) || (rc = ensure_ws(ctx, "adapt.wbuf", b_wb, &wb)))
    return rc;
  // the tail's (cwt_episode_tail), over the loop's G workgroups
  void *fold, *tws, *cnt, *wq;
  if ((rc = ensure_ws(ctx, "attn.fold", attention_fold_floats(C, H) * 4, &fold)) ||
      (rc = ensure_ws(ctx, "tail.ws", std::max(episode_tail_ws_floats(1, hw, G), (size_t)4 << 20) * 4, &tws)) ||
      (rc = ensure_ws(ctx, "tail.cnt", episode_tail_cnt_words() * 4, &cnt)) ||
      (rc = ensure_ws(ctx, "tail.wq", (size_t)G * 2 * C * 4, &wq)))
    return rc;
  if (ctx->fold_w != w_qkvs || ctx->fold_fc != fc_w || ctx->fold_ver != params_version || ctx->fold_H != H) {
    if ((rc = attention_fold(w_qkvs, fc_w, C, H, (float*)fold, (float*)tws, (size_t)4 << 20, st))) return rc;
    ctx->fold_w = w_qkvs;
    ctx->fold_fc = fc_w;
    ctx->fold_ver = params_version;
    ctx->fold_H = H;
  }
  if (ctx->tail_epoch > episode_tail_max_epoch(G) || ctx->tail_G != G) {  // fresh, wrapped, aborted or re-sized
    CWT_HIP(hipMemsetAsync(cnt, 0, episode_tail_cnt_words() * 4, st));
    ctx->tail_epoch = 0;
    ctx->tail_G = G;
  }
  // this launch's stamp slot: {start (min), loop end (max), tail end (max)}, pre-set {~0, 0, 0}; only
  // when the profile records it (otherwise no memsets on the adapt stream and no stamp atomics: the
  // kernel guards every use of a null slot)
  constexpr int kFSlots = 4096;
  int slot = -1;
  unsigned long long* fst = nullptr;
  if (ctx->prof_level >= 1) {
    if (!ctx->fstamps) CWT_HIP(hipMalloc(&ctx->fstamps, (size_t)kFSlots * 3 * sizeof(unsigned long long)));
    slot = ctx->fstamp_next;
    ctx->fstamp_next = (ctx->fstamp_next + 1) % kFSlots;
    fst = ctx->fstamps + 3 * slot;
    CWT_HIP(hipMemsetAsync(fst, 0xFF, sizeof(unsigned long long), st));
    CWT_HIP(hipMemsetAsync(fst + 1, 0, 2 * sizeof(unsigned long long), st));
  }
  TailArgs ta;
  if ((rc = fill_episode_tail_args(W_inout, f_q, 1, hw, h, w, S, q_label, (const float*)fold, fc_b, ln_w, ln_b, out,
                                   logits, logits0, iut, ce, iut0, (float*)tws, (unsigned*)cnt, ctx->tail_epoch++, G,
                                   ctx->adapt_spin_limit, ctx->status_dev + 1, nullptr, &ta)))
    return rc;
  const FusedTail ft{&ta, (float*)wq, fst};
  const std::string kn = "adapt_persist_tail_kernel<5";
  const double lfl = (double)iters * 2.0 * (4.0 * C * h * w * n), lby = (double)iters * ((double)n * h * w * C * 4 + (double)n * S * S);
  const double tfl = 2.0 * 2.0 * hw * C * C * H + 2.0 * 2.0 * H * 2.0 * hw * C;
  Prof p(ctx, st, "inner_adapt x" + std::to_string(iters) + " [" + kn + "]", lfl, lby, 1);
  // the launch's loop part and tail part (its stamps; the events only order the read-back)
  Prof pk(ctx, st, "inner_adapt_kernel [" + kn + "]", lfl, lby, 1, true);
  if (pk.idx >= 0) ctx->recs[pk.idx].fslot = slot;
  rc = launch_adapt(f_s, s_label, 1, n, h, w, S, lr, iters, W_inout, (float*)fws, (uint8_t*)lbl, (AdaptScalars*)sc,
                    (float*)acc, (float*)wb, (AdaptDevArgs*)dargs, nullptr, ctx->adapt_upw, ctx->status_dev,
                    ctx->adapt_spin_limit, st, pk.ev0(), pk.ev1(), &ft);
  p.end();
  if (rc) return rc;
  for (const char* tn : {"post_loop_tail", "episode_tail_kernel"}) {
    Prof pt(ctx, st, tn, tfl, 4.0 * ((double)hw * C * 2 + 2.0 * H * C * C) + 9.0 * S * S, 1);
    pt.end();
    if (pt.idx >= 0) {
      ctx->recs[pt.idx].fslot = slot;
      ctx->recs[pt.idx].fpart = 1;
    }
  }
  return 0;
}

int cwt_classify_scaled(cwt_ctx* ctx, const float* W, const float* f, const float* inv_norm, int B, int P, int C,
                        float* logits, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(W && f && inv_norm && logits && C == 512 && B >= 1 && P >= 1, "bad arguments");
  CWT_HIP(hipSetDevice(ctx->device));
  return launch_classify_scaled(W, f, inv_norm, B, P, logits, (hipStream_t)stream);
}

int cwt_classify(cwt_ctx* ctx, const float* W, const float* f, int B, int P, int C, float* logits, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(W && f && logits && C == 512 && B >= 1 && P >= 1, "bad arguments");
  CWT_HIP(hipSetDevice(ctx->device));
  return launch_classify(W, f, B, P, logits, (hipStream_t)stream);
}

int cwt_classify_bwd(cwt_ctx* ctx, const float* dlogits, const float* f, int B, int P, int C, float* dW,
                     void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(dlogits && f && dW && C == 512 && B >= 1 && P >= 1, "bad arguments");
  CWT_HIP(hipSetDevice(ctx->device));
  return launch_classify_bwd(dlogits, f, B, P, dW, (hipStream_t)stream);
}

int cwt_cos_classify(cwt_ctx* ctx, const float* x, int B, int P, int C, int n, float* weight, const float* g,
                     const float* bias, const float* scale, int mode, float* out, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(x && weight && scale && out && C == 512 && B >= 1 && P >= 1, "bad arguments");
  CWT_CHECK(n >= 1 && n <= 64, "n_classes must be in [1, 64]");
  CWT_CHECK(mode >= 0 && mode <= 3 && (!(mode & 1) || g), "mode: bit 0 WeightNorm (needs g), bit 1 weight_norm");
  CWT_HIP(hipSetDevice(ctx->device));
  void *weff, *vn;
  int rc;
  if ((rc = ensure_ws(ctx, "heads.weff", (size_t)n * C * 4, &weff)) || (rc = ensure_ws(ctx, "heads.vnorm", 64 * 4, &vn)))
    return rc;
  hipStream_t st = (hipStream_t)stream;
  if ((rc = launch_cos_weight(weight, g, n, C, mode, (float*)weff, (float*)vn, st))) return rc;
  return launch_cos_cls_fwd(x, P, B, n, (const float*)weff, bias, scale, out, st);
}

int cwt_cos_classify_bwd(cwt_ctx* ctx, const float* x, int B, int P, int C, int n, float* weight, const float* g,
                         const float* bias, const float* scale, int mode, const float* dscores, float* d_weight,
                         float* d_g, float* d_bias, float* d_scale, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(x && weight && scale && dscores && d_weight && C == 512 && B >= 1 && P >= 1, "bad arguments");
  CWT_CHECK(n >= 1 && n <= 64, "n_classes must be in [1, 64]");
  CWT_CHECK(mode >= 0 && mode <= 3 && (!(mode & 1) || (g && d_g)), "mode: bit 0 WeightNorm (needs g, d_g)");
  CWT_HIP(hipSetDevice(ctx->device));
  const int nb = cos_cls_bwd_blocks((long)B * P);
  void *weff, *vn, *part, *parts;
  int rc;
  if ((rc = ensure_ws(ctx, "heads.weff", (size_t)n * C * 4, &weff)) || (rc = ensure_ws(ctx, "heads.vnorm", 64 * 4, &vn)) ||
      (rc = ensure_ws(ctx, "heads.part", (size_t)nb * n * C * 4, &part)) ||
      (rc = ensure_ws(ctx, "heads.parts", (size_t)nb * n * 2 * 4, &parts)))
    return rc;
  hipStream_t st = (hipStream_t)stream;
  // the forward's weight (for weight_norm the stored weight is already normalised: idempotent)
  if ((rc = launch_cos_weight(weight, g, n, C, mode, (float*)weff, (float*)vn, st))) return rc;
  return launch_cos_cls_bwd(x, P, B, n, (const float*)weff, bias, scale, dscores, (float*)part, (float*)parts, mode,
                            weight, g, (const float*)vn, d_weight, d_g, d_bias, d_scale, st);
}

int cwt_corr(cwt_ctx* ctx, const float* q, const float* k, int B, int Pq, int Pk, int C, float* sim, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(q && k && sim && B >= 1 && Pq >= 1 && Pk >= 1 && C >= 4 && C % 4 == 0, "bad arguments (C % 4 == 0)");
  CWT_HIP(hipSetDevice(ctx->device));
  void *qn, *kn;
  int rc;
  if ((rc = ensure_ws(ctx, "corr.q", (size_t)B * Pq * C * 4, &qn)) || (rc = ensure_ws(ctx, "corr.k", (size_t)B * Pk * C * 4, &kn)))
    return rc;
  return launch_corr(q, k, B, Pq, Pk, C, (float*)qn, (float*)kn, sim, (hipStream_t)stream);
}

// ---- MatchNet (match.py:21-163, conv4d.py:11-62) ----
static int mm_ws(cwt_ctx* ctx, int B, int NA, int NB, int C, float** rowmax, float** colpart, float** colmax) {
  void *r, *p, *c;
  int rc;
  const long nrb = cdiv(NA, 8);  // row blocks of launch_mutual_matching (8 rows: vector forms; 16: scalar)
  if ((rc = ensure_ws(ctx, "match.rowmax", (size_t)B * C * NA * 4, &r)) ||
      (rc = ensure_ws(ctx, "match.colpart", (size_t)B * C * nrb * NB * 4, &p)) ||
      (rc = ensure_ws(ctx, "match.colmax", (size_t)B * C * NB * 4, &c)))
    return rc;
  *rowmax = (float*)r;
  *colpart = (float*)p;
  *colmax = (float*)c;
  return 0;
}

int cwt_mutual_matching(cwt_ctx* ctx, const float* x, int B, int NA, int NB, int C, float* y, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(x && y && B >= 1 && NA >= 1 && NB >= 1 && C >= 1 && C <= 64, "bad arguments");
  CWT_HIP(hipSetDevice(ctx->device));
  float *rm, *cp, *cm;
  int rc;
  if ((rc = mm_ws(ctx, B, NA, NB, C, &rm, &cp, &cm))) return rc;
  return launch_mutual_matching(x, B, NA, NB, C, y, rm, cp, cm, (hipStream_t)stream);
}

// the activations the corr_forward backward reads (cwt_match_corr_forward_train), carved from one
// caller buffer: x0 = MutualMatching(corr) channels-last [E][L], o[branch][layer] the ReLU outputs
// [E][10], [E][10], [E][1], y = o[0][2] + o[1][2] [E] (E = B NA NB), attn [B][NA][ld32(NB)]
struct MatchSaved {
  float* x0;
  float* o[2][3];
  float* y;
  float* attn;
};
static size_t match_saved_layout(float* base, int B, int L, long NA, int symmetric, int readout, MatchSaved* s) {
  const long E = (long)B * NA * NA, ldp = (NA + 31) & ~31L;
  size_t off = 0;
  auto take = [&](long n) {
    float* p = base ? base + off : nullptr;
    off += (size_t)n;
    return p;
  };
  MatchSaved d;
  d.x0 = take(E * L);
  for (int br = 0; br < 2; ++br)
    for (int l = 0; l < 3; ++l) d.o[br][l] = (br == 0 || symmetric) ? take(E * (l < 2 ? 10 : 1)) : nullptr;
  d.y = take(E);
  d.attn = readout ? take((long)B * NA * ldp) : nullptr;
  if (s) *s = d;
  return off;
}

// CWT_MM_FUSE=1: the 2-channel correlation's transposition folded into MutualMatching's passes
// and the symmetric branches' sum into the second MutualMatching (fewer passes over the 4-D map)
static bool mm_fuse() {
  static const bool on = getenv("CWT_MM_FUSE") && getenv("CWT_MM_FUSE")[0] == '1';
  return on;
}

static int match_corr_forward(cwt_ctx* ctx, const float* corr, int B, int L, int h, int w, const float* nc_params,
                              int symmetric, float temp, const float* v, int Cv, float* corr2d, float* weighted_v,
                              void* stream, bool cv4, float* saved = nullptr) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(corr && nc_params && corr2d && B >= 1 && (L == 1 || L == 2) && h >= 1 && w >= 1,
            "bad arguments (in_channel 1 or 2)");
  CWT_CHECK(!weighted_v || (v && Cv >= 1), "weighted_v needs v");
  CWT_HIP(hipSetDevice(ctx->device));
  hipStream_t st = (hipStream_t)stream;
  const long NA = (long)h * w, NB = NA, P = NA * NB;
  void *x0, *x1, *x2, *y1, *y2;
  int rc;
  if ((rc = ensure_ws(ctx, "match.x0", (size_t)B * P * L * 4, &x0)) ||
      (rc = ensure_ws(ctx, "match.x1", (size_t)B * P * 10 * 4, &x1)) ||
      (rc = ensure_ws(ctx, "match.x2", (size_t)B * P * 10 * 4, &x2)) ||
      (rc = ensure_ws(ctx, "match.y1", (size_t)B * P * 4, &y1)) ||
      (rc = ensure_ws(ctx, "match.y2", (size_t)B * P * 4, &y2)))
    return rc;
  MatchSaved S;
  if (saved) {
    CWT_CHECK(!cv4, "the training forward keeps CenterPivotConv4d ('red') activations only");
    match_saved_layout(saved, B, L, NA, symmetric, weighted_v != nullptr, &S);
    x0 = S.x0;
  }
  float *rm, *cp, *cm;
  if ((rc = mm_ws(ctx, B, (int)NA, (int)NB, L, &rm, &cp, &cm))) return rc;
  Prof p(ctx, st, "match_corr_forward", 2.0 * B * P * 2 * (18.0 * L * 10 + 18.0 * 100 + 18.0 * 10), 4.0 * B * P * (L + 1));
  // run_match_model: MutualMatching -> NeighConsensus -> MutualMatching (match.py:159-163)
  if (L == 1) {
    if ((rc = launch_mutual_matching(corr, B, (int)NA, (int)NB, 1, (float*)x0, rm, cp, cm, st))) return rc;
  } else {
    if (mm_fuse()) {
      if ((rc = launch_mutual_matching_planar2(corr, B, (int)NA, (int)NB, (float*)x0, rm, cp, cm, st))) return rc;
    } else {
      if ((rc = launch_to_channels_last(corr, B, L, P, (float*)x0, st))) return rc;
      if ((rc = launch_mutual_matching((const float*)x0, B, (int)NA, (int)NB, L, (float*)x0, rm, cp, cm, st)))
        return rc;
    }
  }
  const int ch[4] = {L, 10, 10, 1};
  if (cv4) {
    // Conv4d layers (conv4d.py:64-138): per layer weight [3][co][ci][3][3][3] (the reference's
    // pre-permuted filter), bias [co]; the symmetric branch is the same stack with each filter's
    // position pairs exchanged (cv4d_layer_kernel swap)
    const float* cw[3][2];
    const float* q = nc_params;
    for (int l = 0; l < 3; ++l) {
      cw[l][0] = q;
      q += 81 * ch[l] * ch[l + 1];
      cw[l][1] = q;
      q += ch[l + 1];
    }
    for (int br = 0; br < (symmetric ? 2 : 1); ++br) {
      const float* in = (const float*)x0;
      float* outs[3] = {(float*)x1, (float*)x2, br ? (float*)y2 : (float*)y1};
      for (int l = 0; l < 3; ++l) {
        if ((rc = launch_cv4d_layer(in, B, h, w, h, w, ch[l], ch[l + 1], cw[l][0], cw[l][1], br, outs[l], st)))
          return rc;
        in = outs[l];
      }
    }
  } else {
  // parameters per layer: conv1.weight [co][ci][3][3], conv1.bias [co], conv2.weight, conv2.bias
  const float* lw[3][4];
  {
    const float* q = nc_params;
    for (int l = 0; l < 3; ++l) {
      const int n = ch[l + 1] * ch[l] * 9;
      lw[l][0] = q; q += n;
      lw[l][1] = q; q += ch[l + 1];
      lw[l][2] = q; q += n;
      lw[l][3] = q; q += ch[l + 1];
    }
  }
  // branch 0: conv(x) (conv1 over the query positions a, conv2 over the support positions b);
  // branch 1 (symmetric mode): conv(x^T)^T = the same stack with the two roles swapped.  The two
  // branches are independent until their sum: branch 1 runs on the context's second stream
  // (its own intermediate buffers), so one branch's store-bound layers overlap the other's
  // MFMA-bound ones (CWT_MATCH_BRANCH_STREAMS=0: one after the other on the caller's stream)
  static const bool two_streams = !(getenv("CWT_MATCH_BRANCH_STREAMS") && getenv("CWT_MATCH_BRANCH_STREAMS")[0] == '0');
  const bool fork = symmetric && two_streams;
  void *x1b = x1, *x2b = x2;
  if (fork) {
    if (!saved && ((rc = ensure_ws(ctx, "match.x1b", (size_t)B * P * 10 * 4, &x1b)) ||
                   (rc = ensure_ws(ctx, "match.x2b", (size_t)B * P * 10 * 4, &x2b))))
      return rc;
    if (!ctx->aux) CWT_HIP(hipStreamCreateWithFlags(&ctx->aux, hipStreamNonBlocking));
    if (!ctx->ev_fork) CWT_HIP(hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming));
    if (!ctx->ev_join) CWT_HIP(hipEventCreateWithFlags(&ctx->ev_join, hipEventDisableTiming));
    CWT_HIP(hipEventRecord(ctx->ev_fork, st));
    CWT_HIP(hipStreamWaitEvent(ctx->aux, ctx->ev_fork, 0));
  }
  for (int br = 0; br < (symmetric ? 2 : 1); ++br) {
    const float* in = (const float*)x0;
    const hipStream_t bst = (fork && br == 1) ? ctx->aux : st;
    float* outs[3] = {br && fork ? (float*)x1b : (float*)x1, br && fork ? (float*)x2b : (float*)x2,
                      br ? (float*)y2 : (float*)y1};
    if (saved)
      for (int l = 0; l < 3; ++l) outs[l] = S.o[br][l];
    for (int l = 0; l < 3; ++l) {
      const float* Wa = br ? lw[l][2] : lw[l][0];
      const float* ba = br ? lw[l][3] : lw[l][1];
      const float* Wb = br ? lw[l][0] : lw[l][2];
      const float* bb = br ? lw[l][1] : lw[l][3];
      if ((rc = launch_cp4d_layer(in, B, h, w, h, w, ch[l], ch[l + 1], Wa, ba, Wb, bb, outs[l], bst))) return rc;
      in = outs[l];
    }
  }
  if (fork) {
    CWT_HIP(hipEventRecord(ctx->ev_join, ctx->aux));
    CWT_HIP(hipStreamWaitEvent(st, ctx->ev_join, 0));
  }
  }
  if (saved) {  // y = o[0][2] (+ o[1][2]) into its own slot: the ReLU outputs stay for the backward
    CWT_HIP(hipMemcpyAsync(S.y, S.o[0][2], (size_t)B * P * 4, hipMemcpyDeviceToDevice, st));
    if (symmetric && (rc = launch_add_inplace(S.y, (const float*)S.o[1][2], B * P, st))) return rc;
    y1 = S.y;
  } else if (symmetric && !mm_fuse() && (rc = launch_add_inplace((float*)y1, (const float*)y2, B * P, st))) {
    return rc;
  }
  if ((rc = mm_ws(ctx, B, (int)NA, (int)NB, 1, &rm, &cp, &cm))) return rc;
  if (!saved && symmetric && mm_fuse()) {  // MutualMatching of y1 + y2 (the sum folded into its two passes)
    if ((rc = launch_mutual_matching_sum((const float*)y1, (const float*)y2, B, (int)NA, (int)NB, corr2d, rm, cp, cm,
                                         st)))
      return rc;
  } else if ((rc = launch_mutual_matching((const float*)y1, B, (int)NA, (int)NB, 1, corr2d, rm, cp, cm, st))) {
    return rc;
  }
  if (weighted_v) {
    // attn = softmax(temp * corr2d, dim=-1); weighted_v = bmm(v, attn^T) (match.py:151-153),
    // here as tokens [B][NA][Cv] = attn . v
    const int ldp = (int)((NB + 31) & ~31L);  // zero-padded to whole 32-deep K tiles (gemm_f32d)
    void *pw, *vt;
    if ((rc = ensure_ws(ctx, "match.attn", (size_t)B * NA * ldp * 4, &pw)) ||
        (rc = ensure_ws(ctx, "match.vt", (size_t)B * Cv * ldp * 4, &vt)))
      return rc;
    if (saved) pw = S.attn;
    if ((rc = launch_match_softmax(corr2d, B, (int)NA, (int)NB, temp, ldp, (float*)pw, st))) return rc;
    if ((rc = launch_match_vt(v, B, (int)NB, Cv, ldp, (float*)vt, st))) return rc;
    if ((rc = readout_gemm(ctx, (const float*)pw, (const float*)vt, B, (int)NA, Cv, ldp, weighted_v, st))) return rc;
  }
  p.end();
  return 0;
}

int cwt_match_corr_forward(cwt_ctx* ctx, const float* corr, int B, int L, int h, int w, const float* nc_params,
                           int symmetric, float temp, const float* v, int Cv, float* corr2d, float* weighted_v,
                           void* stream) {
  return match_corr_forward(ctx, corr, B, L, h, w, nc_params, symmetric, temp, v, Cv, corr2d, weighted_v, stream, false);
}

int cwt_match_corr_forward_cv4(cwt_ctx* ctx, const float* corr, int B, int L, int h, int w, const float* nc_params,
                               int symmetric, float temp, const float* v, int Cv, float* corr2d, float* weighted_v,
                               void* stream) {
  return match_corr_forward(ctx, corr, B, L, h, w, nc_params, symmetric, temp, v, Cv, corr2d, weighted_v, stream, true);
}

// ---- MatchNet / MMN backward (match_bwd.hip) ----
static inline long ld32(long n) { return (n + 31) & ~31L; }

// C [M][N] = A [M][K] . W [N][K]^T (K % 4 == 0): the exact-fp32 conv body where its shape rules
// allow (gemm_f32d), else corr_gemm_kernel
static int gemm_nt(cwt_ctx* ctx, const float* A, const float* W, int M, int N, int K, float* C, hipStream_t st) {
  if (gemm_f32d_ok(M, N, K, A, W, C, nullptr)) return gemm_f32d(ctx, A, W, M, N, K, C, nullptr, nullptr, 0, st);
  if (K % 4) return fail(CWT_EARG, "gemm_nt: K % 4 != 0");
  return launch_gemm_abt(A, W, 1, M, N, K, C, st);
}

static int mm_bwd_ws(cwt_ctx* ctx, int B, int NA, int NB, int C, MmBwdWs* w) {
  const long nrb = cdiv(NA, 16), bc = (long)B * C;
  const char* nm[8] = {"mb.rowmax", "mb.rowarg", "mb.colpv", "mb.colpi", "mb.colmax", "mb.colarg", "mb.srow", "mb.scol"};
  const long sz[8] = {bc * NA, bc * NA, bc * nrb * NB, bc * nrb * NB, bc * NB, bc * NB, bc * NA, bc * NB};
  void* p[8];
  int rc;
  for (int i = 0; i < 8; ++i)
    if ((rc = ensure_ws(ctx, nm[i], (size_t)sz[i] * 4, &p[i]))) return rc;
  w->rowmax = (float*)p[0];
  w->rowarg = (int*)p[1];
  w->colpv = (float*)p[2];
  w->colpi = (int*)p[3];
  w->colmax = (float*)p[4];
  w->colarg = (int*)p[5];
  w->srow = (float*)p[6];
  w->scol = (float*)p[7];
  return 0;
}

int cwt_match_corr_saved_floats(int B, int L, int h, int w, int symmetric, int readout, int64_t* n) {
  if (!n || B < 1 || (L != 1 && L != 2) || h < 1 || w < 1) return fail(CWT_EARG, "bad arguments");
  *n = (int64_t)match_saved_layout(nullptr, B, L, (long)h * w, symmetric, readout, nullptr);
  return 0;
}

int cwt_match_corr_forward_train(cwt_ctx* ctx, const float* corr, int B, int L, int h, int w, const float* nc_params,
                                 int symmetric, float temp, const float* v, int Cv, float* corr2d, float* weighted_v,
                                 float* saved, void* stream) {
  if (!saved) return fail(CWT_EARG, "saved is NULL");
  return match_corr_forward(ctx, corr, B, L, h, w, nc_params, symmetric, temp, v, Cv, corr2d, weighted_v, stream, false,
                            saved);
}

int cwt_match_corr_backward(cwt_ctx* ctx, const float* corr, int B, int L, int h, int w, const float* nc_params,
                            int symmetric, float temp, const float* v, int Cv, const float* saved,
                            const float* d_corr2d, const float* d_weighted_v, float* d_corr, float* d_params,
                            float* d_v, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(corr && nc_params && saved && d_params && B >= 1 && (L == 1 || L == 2) && h >= 1 && w >= 1,
            "bad arguments (in_channel 1 or 2)");
  CWT_CHECK(!d_weighted_v || (v && Cv >= 4 && Cv % 4 == 0), "d_weighted_v needs v and Cv % 4 == 0");
  CWT_CHECK(!d_v || d_weighted_v, "d_v needs d_weighted_v");
  CWT_HIP(hipSetDevice(ctx->device));
  hipStream_t st = (hipStream_t)stream;
  const long NA = (long)h * w, NB = NA, P = NA * NB, E = (long)B * P, ldp = ld32(NB);
  MatchSaved S;
  match_saved_layout((float*)saved, B, L, NA, symmetric, d_weighted_v != nullptr, &S);
  const int ch[4] = {L, 10, 10, 1};
  const float* lw[3][4];
  float* dlw[3][4];
  long np = 0;
  for (int l = 0; l < 3; ++l) {
    const long n = (long)ch[l + 1] * ch[l] * 9;
    const long off[4] = {np, np + n, np + n + ch[l + 1], np + 2 * n + ch[l + 1]};
    for (int q = 0; q < 4; ++q) {
      lw[l][q] = nc_params + off[q];
      dlw[l][q] = d_params + off[q];
    }
    np += 2 * (n + ch[l + 1]);
  }
  const size_t part_floats = (size_t)cp4d_wgrad_part_floats(10, 10);
  void *g2d, *dy, *gA, *gm, *dx0, *part;
  int rc;
  if ((rc = ensure_ws(ctx, "mb.g2d", (size_t)E * 4, &g2d)) || (rc = ensure_ws(ctx, "mb.dy", (size_t)E * 4, &dy)) ||
      (rc = ensure_ws(ctx, "mb.gA", (size_t)E * 10 * 4, &gA)) || (rc = ensure_ws(ctx, "mb.gm", (size_t)E * 10 * 4, &gm)) ||
      (rc = ensure_ws(ctx, "mb.dx0", (size_t)E * L * 4, &dx0)) || (rc = ensure_ws(ctx, "mb.part", part_floats * 4, &part)))
    return rc;
  MmBwdWs mw;
  if ((rc = mm_bwd_ws(ctx, B, (int)NA, (int)NB, L, &mw))) return rc;
  Prof p(ctx, st, "match_corr_backward", 2.0 * 2.0 * B * P * 2 * (18.0 * L * 10 + 18.0 * 100 + 18.0 * 10),
         4.0 * B * P * (L + 44));
  CWT_HIP(hipMemsetAsync(d_params, 0, (size_t)np * 4, st));
  // the gradient at corr2d: the caller's, plus the softmax readout's (match.py:151-153)
  if (d_corr2d)
    CWT_HIP(hipMemcpyAsync(g2d, d_corr2d, (size_t)E * 4, hipMemcpyDeviceToDevice, st));
  else
    CWT_HIP(hipMemsetAsync(g2d, 0, (size_t)E * 4, st));
  if (d_weighted_v) {
    void* dA;
    if ((rc = ensure_ws(ctx, "mb.dA", (size_t)E * 4, &dA))) return rc;
    for (int b = 0; b < B; ++b)  // dA = d_wv . v^T
      if ((rc = gemm_nt(ctx, d_weighted_v + (long)b * NA * Cv, v + (long)b * NB * Cv, (int)NA, (int)NB, Cv,
                        (float*)dA + (long)b * NA * NB, st)))
        return rc;
    if ((rc = launch_match_softmax_bwd(S.attn, (int)ldp, (const float*)dA, (int)(B * NA), (int)NB, temp, 1,
                                       (float*)g2d, st)))
      return rc;
    if (d_v) {  // d_v[b] = attn[b]^T . d_wv[b]
      const long lda = ld32(NA);
      void *pt, *dwt;
      if ((rc = ensure_ws(ctx, "mb.PT", (size_t)B * ldp * lda * 4, &pt)) ||
          (rc = ensure_ws(ctx, "mb.dwvT", (size_t)B * Cv * lda * 4, &dwt)))
        return rc;
      if ((rc = launch_match_vt(S.attn, B, (int)NA, (int)ldp, (int)lda, (float*)pt, st)) ||
          (rc = launch_match_vt(d_weighted_v, B, (int)NA, Cv, (int)lda, (float*)dwt, st)))
        return rc;
      for (int b = 0; b < B; ++b)
        if ((rc = gemm_nt(ctx, (const float*)pt + (long)b * ldp * lda, (const float*)dwt + (long)b * Cv * lda, (int)NB, Cv,
                          (int)lda, d_v + (long)b * NB * Cv, st)))
          return rc;
    }
  }
  // the second MutualMatching (match.py:162)
  if ((rc = launch_mutual_matching_bwd(S.y, (const float*)g2d, B, (int)NA, (int)NB, 1, (float*)dy, mw, st))) return rc;
  // NeighConsensus: both branches see the same output gradient (y = branch 0 + branch 1); branch 1
  // applied conv2's filter over the a plane and conv1's over the b plane (match.py:75-80)
  for (int br = 0; br < (symmetric ? 2 : 1); ++br) {
    const float* gcur = (const float*)dy;
    for (int l = 2; l >= 0; --l) {
      const int cin = ch[l], cout = ch[l + 1];
      const float* out = S.o[br][l];
      const float* in = l ? S.o[br][l - 1] : S.x0;
      if ((rc = launch_relu_mask(gcur, out, E * cout, (float*)gm, st))) return rc;
      const float* Wa = br ? lw[l][2] : lw[l][0];
      const float* Wb = br ? lw[l][0] : lw[l][2];
      float* dWa = br ? dlw[l][2] : dlw[l][0];
      float* dWb = br ? dlw[l][0] : dlw[l][2];
      if ((rc = launch_cp4d_wgrad(in, (const float*)gm, B, h, w, h, w, cin, cout, (float*)part, part_floats, dWa, dWb,
                                  dlw[l][1], dlw[l][3], st)))
        return rc;
      if (l > 0) {
        if ((rc = launch_cp4d_dgrad((const float*)gm, B, h, w, h, w, cout, cin, Wa, Wb, (float*)gA, 0, st))) return rc;
        gcur = (const float*)gA;
      } else if (d_corr) {
        if ((rc = launch_cp4d_dgrad((const float*)gm, B, h, w, h, w, cout, cin, Wa, Wb, (float*)dx0, br, st))) return rc;
      }
    }
  }
  // the first MutualMatching (match.py:160), back to the caller's channel-first layout
  if (d_corr) {
    if (L == 1) {
      if ((rc = launch_mutual_matching_bwd(corr, (const float*)dx0, B, (int)NA, (int)NB, 1, d_corr, mw, st))) return rc;
    } else {
      void *xcl, *dxcl;
      if ((rc = ensure_ws(ctx, "mb.xcl", (size_t)E * L * 4, &xcl)) || (rc = ensure_ws(ctx, "mb.dxcl", (size_t)E * L * 4, &dxcl)))
        return rc;
      if ((rc = launch_to_channels_last(corr, B, L, P, (float*)xcl, st)) ||
          (rc = launch_mutual_matching_bwd((const float*)xcl, (const float*)dx0, B, (int)NA, (int)NB, L, (float*)dxcl, mw,
                                           st)) ||
          (rc = launch_to_channels_first((const float*)dxcl, B, L, P, d_corr, st)))
        return rc;
    }
  }
  p.end();
  return 0;
}

int cwt_corr_backward(cwt_ctx* ctx, const float* q, const float* k, int B, int Pq, int Pk, int C, const float* d_sim,
                      float* dq, float* dk, int accum_q, int accum_k, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(q && k && d_sim && B >= 1 && Pq >= 1 && Pk >= 1 && C >= 1, "bad arguments");
  CWT_HIP(hipSetDevice(ctx->device));
  hipStream_t st = (hipStream_t)stream;
  const float eps = 1e-12f;
  void *qn, *qr, *kn, *kr;
  int rc;
  if ((rc = ensure_ws(ctx, "cb.qn", (size_t)B * Pq * C * 4, &qn)) || (rc = ensure_ws(ctx, "cb.qr", (size_t)B * Pq * 4, &qr)) ||
      (rc = ensure_ws(ctx, "cb.kn", (size_t)B * Pk * C * 4, &kn)) || (rc = ensure_ws(ctx, "cb.kr", (size_t)B * Pk * 4, &kr)))
    return rc;
  Prof p(ctx, st, "corr_backward", 2.0 * 2.0 * B * (double)Pq * Pk * C, 4.0 * B * ((double)Pq * Pk + 2.0 * (Pq + Pk) * C));
  if ((rc = launch_token_norm(q, (long)B * Pq, C, eps, (float*)qn, (float*)qr, st)) ||
      (rc = launch_token_norm(k, (long)B * Pk, C, eps, (float*)kn, (float*)kr, st)))
    return rc;
  if (dq) {  // d qn = d_sim . kn
    const long ldk = ld32(Pk);
    void *dsp, *knt, *dqn;
    if ((rc = ensure_ws(ctx, "cb.dsp", (size_t)B * Pq * ldk * 4, &dsp)) ||
        (rc = ensure_ws(ctx, "cb.knT", (size_t)B * C * ldk * 4, &knt)) ||
        (rc = ensure_ws(ctx, "cb.dqn", (size_t)B * Pq * C * 4, &dqn)))
      return rc;
    if ((rc = launch_copy_pad(d_sim, (long)B * Pq, Pk, (int)ldk, (float*)dsp, st)) ||
        (rc = launch_match_vt((const float*)kn, B, Pk, C, (int)ldk, (float*)knt, st)))
      return rc;
    for (int b = 0; b < B; ++b)
      if ((rc = gemm_nt(ctx, (const float*)dsp + (long)b * Pq * ldk, (const float*)knt + (long)b * C * ldk, Pq, C, (int)ldk,
                        (float*)dqn + (long)b * Pq * C, st)))
        return rc;
    if ((rc = launch_token_norm_bwd((const float*)qn, (const float*)qr, (const float*)dqn, (long)B * Pq, C, C, eps, accum_q,
                                    dq, st)))
      return rc;
  }
  if (dk) {  // d kn = d_sim^T . qn
    const long ldq = ld32(Pq);
    void *dst, *qnt, *dkn;
    if ((rc = ensure_ws(ctx, "cb.dsT", (size_t)B * Pk * ldq * 4, &dst)) ||
        (rc = ensure_ws(ctx, "cb.qnT", (size_t)B * C * ldq * 4, &qnt)) ||
        (rc = ensure_ws(ctx, "cb.dkn", (size_t)B * Pk * C * 4, &dkn)))
      return rc;
    if ((rc = launch_match_vt(d_sim, B, Pq, Pk, (int)ldq, (float*)dst, st)) ||
        (rc = launch_match_vt((const float*)qn, B, Pq, C, (int)ldq, (float*)qnt, st)))
      return rc;
    for (int b = 0; b < B; ++b)
      if ((rc = gemm_nt(ctx, (const float*)dst + (long)b * Pk * ldq, (const float*)qnt + (long)b * C * ldq, Pk, C, (int)ldq,
                        (float*)dkn + (long)b * Pk * C, st)))
        return rc;
    if ((rc = launch_token_norm_bwd((const float*)kn, (const float*)kr, (const float*)dkn, (long)B * Pk, C, C, eps, accum_k,
                                    dk, st)))
      return rc;
  }
  p.end();
  return 0;
}

int cwt_sce_descriptor(cwt_ctx* ctx, const float* x, int B, int h, int w, int C, int k, int ldg, float* g,
                       void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(x && g && B >= 1 && h >= 1 && w >= 1 && C >= 1, "bad arguments");
  CWT_HIP(hipSetDevice(ctx->device));
  hipStream_t st = (hipStream_t)stream;
  Prof p(ctx, st, "sce_descriptor", 2.0 * B * h * w * (double)k * k * C, 4.0 * B * h * w * ((double)C + ldg));
  int rc;
  if ((rc = launch_sce_descriptor(x, B, h, w, C, k, ldg, g, st))) return rc;
  p.end();
  return 0;
}

int cwt_channel_sum(cwt_ctx* ctx, const float* x, int B, int L, int64_t P, float* y, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(x && y && B >= 1 && L >= 1 && P >= 1, "bad arguments");
  CWT_HIP(hipSetDevice(ctx->device));
  hipStream_t st = (hipStream_t)stream;
  Prof p(ctx, st, "channel_sum", (double)B * L * P, 4.0 * B * P * (L + 1));
  int rc;
  if ((rc = launch_channel_sum(x, B, L, (long)P, y, st))) return rc;
  p.end();
  return 0;
}

int cwt_match_masks(cwt_ctx* ctx, float* corr2d, int B, int NA, int NB, const uint8_t* ig_mask,
                    const int64_t* s_mask, float* inconsistent, void* stream) {
  return cwt_match_masks_train(ctx, corr2d, B, NA, NB, ig_mask, s_mask, inconsistent, 0.f, 0, stream);
}

int cwt_match_masks_train(cwt_ctx* ctx, float* corr2d, int B, int NA, int NB, const uint8_t* ig_mask,
                          const int64_t* s_mask, float* inconsistent, float drop_p, uint64_t seed, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(corr2d && B >= 1 && NA >= 1 && NB >= 1 && drop_p >= 0.f && drop_p < 1.f, "bad arguments");
  CWT_CHECK(!s_mask || inconsistent, "the cycle mask needs inconsistent");
  CWT_HIP(hipSetDevice(ctx->device));
  hipStream_t st = (hipStream_t)stream;
  void *q2k = nullptr, *pv = nullptr, *pi = nullptr;
  int rc;
  if (s_mask && ((rc = ensure_ws(ctx, "match.q2k", (size_t)B * NA * 4, &q2k)) ||
                 (rc = ensure_ws(ctx, "match.colv", (size_t)B * 16 * NB * 4, &pv)) ||
                 (rc = ensure_ws(ctx, "match.coli", (size_t)B * 16 * NB * 4, &pi))))
    return rc;
  Prof p(ctx, st, "match_masks", 0.0, 4.0 * B * NA * NB * (s_mask ? 4 : 2));
  if ((rc = launch_match_masks(corr2d, B, NA, NB, ig_mask, s_mask, inconsistent, (int*)q2k, (float*)pv, (int*)pi, st,
                               drop_p, (unsigned long long)seed)))
    return rc;
  p.end();
  return 0;
}

int cwt_match_readout(cwt_ctx* ctx, const float* corr2d, int B, int NA, int NB, float temp, const float* v, int Cv,
                      float* weighted_v, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(corr2d && v && weighted_v && B >= 1 && NA >= 1 && NB >= 1 && Cv >= 1, "bad arguments");
  CWT_HIP(hipSetDevice(ctx->device));
  hipStream_t st = (hipStream_t)stream;
  const int ldp = (int)((NB + 31) & ~31L);  // zero-padded to whole 32-deep K tiles (gemm_f32d)
  void *pw, *vt;
  int rc;
  if ((rc = ensure_ws(ctx, "match.attn", (size_t)B * NA * ldp * 4, &pw)) ||
      (rc = ensure_ws(ctx, "match.vt", (size_t)B * Cv * ldp * 4, &vt)))
    return rc;
  Prof p(ctx, st, "match_readout", 2.0 * B * NA * (double)NB * Cv, 4.0 * B * ((double)NA * NB * 2 + (double)NB * Cv));
  if ((rc = launch_match_softmax(corr2d, B, NA, NB, temp, ldp, (float*)pw, st))) return rc;
  if ((rc = launch_match_vt(v, B, NB, Cv, ldp, (float*)vt, st))) return rc;
  if ((rc = readout_gemm(ctx, (const float*)pw, (const float*)vt, B, NA, Cv, ldp, weighted_v, st))) return rc;
  p.end();
  return 0;
}

int cwt_match_readout_backward(cwt_ctx* ctx, const float* corr2d, int B, int NA, int NB, float temp, const float* v,
                               int Cv, const float* d_weighted_v, const uint8_t* ig_mask, float* d_corr2d, float* d_v,
                               void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(corr2d && d_corr2d && B >= 1 && NA >= 1 && NB >= 1, "bad arguments");
  CWT_CHECK(!d_weighted_v || (v && Cv >= 4 && Cv % 4 == 0), "d_weighted_v needs v and Cv % 4 == 0");
  CWT_CHECK(!d_v || d_weighted_v, "d_v needs d_weighted_v");
  CWT_HIP(hipSetDevice(ctx->device));
  hipStream_t st = (hipStream_t)stream;
  const int ldp = (int)((NB + 31) & ~31L);
  const long E = (long)B * NA * NB;
  void *pw, *dA;
  int rc;
  if ((rc = ensure_ws(ctx, "match.attn", (size_t)B * NA * ldp * 4, &pw)) ||
      (rc = ensure_ws(ctx, "mb.dA", (size_t)E * 4, &dA)))
    return rc;
  Prof p(ctx, st, "match_readout_backward", 2.0 * 2.0 * B * NA * (double)NB * Cv,
         4.0 * B * ((double)NA * NB * 4 + (double)(NA + NB) * Cv * 2));
  if (d_weighted_v) {
    // attn = softmax(temp corr2d) again (the forward's masked corr2d), dA = d_wv . v^T
    if ((rc = launch_match_softmax(corr2d, B, NA, NB, temp, ldp, (float*)pw, st))) return rc;
    for (int b = 0; b < B; ++b)
      if ((rc = gemm_nt(ctx, d_weighted_v + (long)b * NA * Cv, v + (long)b * NB * Cv, NA, NB, Cv,
                        (float*)dA + (long)b * NA * NB, st)))
        return rc;
    // d corr2d += temp P (dA - <P, dA>) (accumulating into the caller's gradient at corr2d)
    if ((rc = launch_match_softmax_bwd((const float*)pw, ldp, (const float*)dA, B * NA, NB, temp, 1, d_corr2d, st)))
      return rc;
  }
  if (ig_mask && (rc = launch_match_zero_ig_cols(d_corr2d, ig_mask, B, NA, NB, st))) return rc;
  if (d_v) {  // d_v[b] = attn[b]^T . d_wv[b]
    const long lda = ld32(NA);
    void *pt, *dwt;
    if ((rc = ensure_ws(ctx, "mb.PT", (size_t)B * ldp * lda * 4, &pt)) ||
        (rc = ensure_ws(ctx, "mb.dwvT", (size_t)B * Cv * lda * 4, &dwt)))
      return rc;
    if ((rc = launch_match_vt((const float*)pw, B, NA, ldp, (int)lda, (float*)pt, st)) ||
        (rc = launch_match_vt(d_weighted_v, B, NA, Cv, (int)lda, (float*)dwt, st)))
      return rc;
    for (int b = 0; b < B; ++b)
      if ((rc = gemm_nt(ctx, (const float*)pt + (long)b * ldp * lda, (const float*)dwt + (long)b * Cv * lda, NB, Cv,
                        (int)lda, d_v + (long)b * NB * Cv, st)))
        return rc;
  }
  p.end();
  return 0;
}

static int weight_average(cwt_ctx* ctx, const float* x, int N, int h, int w, int C, const float* w_tpg,
                          const float* b_theta, const float* b_phi, const float* b_g, const float* w_back,
                          const float* b_back, float* out, void* stream, float* tpg_keep, float* wavg_keep) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(x && w_tpg && b_theta && b_phi && b_g && w_back && b_back && out && N >= 1 && h >= 1 && w >= 1,
            "bad arguments");
  CWT_CHECK(C == 512 || C == 1024 || C == 2048, "WeightAverage: c_in 512, 1024 or 2048");
  CWT_HIP(hipSetDevice(ctx->device));
  hipStream_t st = (hipStream_t)stream;
  const int co = C / 2;
  const long P = (long)N * h * w;
  void *tpg, *wavg, *back;
  int rc;
  if ((rc = ensure_ws(ctx, "wa.tpg", (size_t)P * 3 * co * 4, &tpg)) ||
      (rc = ensure_ws(ctx, "wa.avg", (size_t)P * co * 4, &wavg)) ||
      (rc = ensure_ws(ctx, "wa.back", (size_t)P * C * 4, &back)))
    return rc;
  if (tpg_keep) tpg = tpg_keep;
  if (wavg_keep) wavg = wavg_keep;
  Prof p(ctx, st, "weight_average c" + std::to_string(C), 2.0 * P * C * co * 4, 4.0 * P * (2.0 * C + 5.0 * co));
  // theta | phi | g of every pixel: one GEMM against the three stacked 1x1 weights [3co][C]
  const bool wa_f32d = gemm_f32d_mode() != 0;
  if (wa_f32d && gemm_f32d_ok((int)P, 3 * co, C, x, w_tpg, tpg, nullptr)) {
    if ((rc = gemm_f32d(ctx, x, w_tpg, (int)P, 3 * co, C, (float*)tpg, nullptr, nullptr, 0, st))) return rc;
  } else if ((rc = launch_gemm_abt(x, w_tpg, 1, (int)P, 3 * co, C, (float*)tpg, st))) {
    return rc;
  }
  if ((rc = launch_wa_attn((const float*)tpg, N, h, w, co, b_theta, b_phi, b_g, (float*)wavg, st))) return rc;
  if (wa_f32d && gemm_f32d_ok((int)P, C, co, wavg, w_back, out, x)) {  // conv_back + bias + residual in one epilogue
    if ((rc = gemm_f32d(ctx, (const float*)wavg, w_back, (int)P, C, co, out, b_back, x, C, st))) return rc;
  } else {
    if ((rc = launch_gemm_abt((const float*)wavg, w_back, 1, (int)P, C, co, (float*)back, st))) return rc;
    if ((rc = launch_wa_residual(x, (const float*)back, b_back, P * C, C, out, st))) return rc;
  }
  p.end();
  return 0;
}

int cwt_weight_average(cwt_ctx* ctx, const float* x, int N, int h, int w, int C, const float* w_tpg,
                       const float* b_theta, const float* b_phi, const float* b_g, const float* w_back,
                       const float* b_back, float* out, void* stream) {
  return weight_average(ctx, x, N, h, w, C, w_tpg, b_theta, b_phi, b_g, w_back, b_back, out, stream, nullptr, nullptr);
}

int cwt_weight_average_train(cwt_ctx* ctx, const float* x, int N, int h, int w, int C, const float* w_tpg,
                             const float* b_theta, const float* b_phi, const float* b_g, const float* w_back,
                             const float* b_back, float* out, float* tpg, float* wavg, void* stream) {
  if (!tpg || !wavg) return fail(CWT_EARG, "tpg / wavg is NULL");
  return weight_average(ctx, x, N, h, w, C, w_tpg, b_theta, b_phi, b_g, w_back, b_back, out, stream, tpg, wavg);
}

int cwt_weight_average_backward(cwt_ctx* ctx, const float* x, int N, int h, int w, int C, const float* w_tpg,
                                const float* b_theta, const float* b_phi, const float* b_g, const float* w_back,
                                const float* tpg, const float* wavg, const float* d_out, float* d_x,
                                float* d_w_tpg, float* d_b_theta, float* d_b_phi, float* d_b_g, float* d_w_back,
                                float* d_b_back, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(x && w_tpg && b_theta && b_phi && b_g && w_back && tpg && wavg && d_out && d_w_tpg && d_b_theta &&
                d_b_phi && d_b_g && d_w_back && d_b_back && N >= 1 && h >= 1 && w >= 1,
            "bad arguments");
  CWT_CHECK(C == 512 || C == 1024 || C == 2048, "WeightAverage: c_in 512, 1024 or 2048");
  CWT_HIP(hipSetDevice(ctx->device));
  hipStream_t st = (hipStream_t)stream;
  const int co = C / 2;
  const long P = (long)N * h * w, ldP = ld32(P);
  void *wbt, *dwavg, *coef, *dtpg, *dot, *wvt, *dtt, *xt;
  int rc;
  if ((rc = ensure_ws(ctx, "wab.wbT", (size_t)co * C * 4, &wbt)) || (rc = ensure_ws(ctx, "wab.dwavg", (size_t)P * co * 4, &dwavg)) ||
      (rc = ensure_ws(ctx, "wab.coef", (size_t)P * 27 * 4, &coef)) ||
      (rc = ensure_ws(ctx, "wab.dtpg", (size_t)P * 3 * co * 4, &dtpg)) ||
      (rc = ensure_ws(ctx, "wab.doT", (size_t)C * ldP * 4, &dot)) || (rc = ensure_ws(ctx, "wab.wvT", (size_t)co * ldP * 4, &wvt)) ||
      (rc = ensure_ws(ctx, "wab.dtT", (size_t)3 * co * ldP * 4, &dtt)) || (rc = ensure_ws(ctx, "wab.xT", (size_t)C * ldP * 4, &xt)))
    return rc;
  Prof p(ctx, st, "weight_average_backward c" + std::to_string(C), 2.0 * P * C * co * 8, 4.0 * P * (4.0 * C + 8.0 * co));
  // d wavg = d_out . w_back  (conv_back, msm_func.py:99)
  if ((rc = launch_match_vt(w_back, 1, C, co, C, (float*)wbt, st)) ||
      (rc = gemm_nt(ctx, d_out, (const float*)wbt, (int)P, co, C, (float*)dwavg, st)))
    return rc;
  // softmax-weighted neighbourhood and the cosine similarities (msm_func.py:66-97)
  if ((rc = launch_wa_bwd(tpg, N, h, w, co, b_theta, b_phi, b_g, (const float*)dwavg, (float*)coef, (float*)dtpg, st)))
    return rc;
  // biases: column sums in a fixed order
  void* csw;
  const size_t csn = colsum_ws_floats(P, C);
  if ((rc = ensure_ws(ctx, "colsum", csn * 4, &csw))) return rc;
  if ((rc = launch_colsum((const float*)dtpg, P, co, 3L * co, 0, d_b_theta, (float*)csw, csn, st)) ||
      (rc = launch_colsum((const float*)dtpg + co, P, co, 3L * co, 0, d_b_phi, (float*)csw, csn, st)) ||
      (rc = launch_colsum((const float*)dtpg + 2 * co, P, co, 3L * co, 0, d_b_g, (float*)csw, csn, st)) ||
      (rc = launch_colsum(d_out, P, C, C, 0, d_b_back, (float*)csw, csn, st)))
    return rc;
  // d w_back = d_out^T . wavg, d w_tpg = d tpg^T . x (reductions over the pixels, zero-padded to 32)
  if ((rc = launch_match_vt(d_out, 1, (int)P, C, (int)ldP, (float*)dot, st)) ||
      (rc = launch_match_vt(wavg, 1, (int)P, co, (int)ldP, (float*)wvt, st)) ||
      (rc = gemm_nt(ctx, (const float*)dot, (const float*)wvt, C, co, (int)ldP, d_w_back, st)) ||
      (rc = launch_match_vt((const float*)dtpg, 1, (int)P, 3 * co, (int)ldP, (float*)dtt, st)) ||
      (rc = launch_match_vt(x, 1, (int)P, C, (int)ldP, (float*)xt, st)) ||
      (rc = gemm_nt(ctx, (const float*)dtt, (const float*)xt, 3 * co, C, (int)ldP, d_w_tpg, st)))
    return rc;
  if (d_x) {  // d x = d_out (the residual) + d tpg . w_tpg
    void* wtt;
    if ((rc = ensure_ws(ctx, "wab.wtT", (size_t)C * 3 * co * 4, &wtt))) return rc;
    if ((rc = launch_match_vt(w_tpg, 1, 3 * co, C, 3 * co, (float*)wtt, st))) return rc;
    if (gemm_f32d_ok((int)P, C, 3 * co, dtpg, wtt, d_x, d_out)) {
      if ((rc = gemm_f32d(ctx, (const float*)dtpg, (const float*)wtt, (int)P, C, 3 * co, d_x, nullptr, d_out, C, st))) return rc;
    } else if ((rc = gemm_nt(ctx, (const float*)dtpg, (const float*)wtt, (int)P, C, 3 * co, d_x, st)) ||
               (rc = launch_add_inplace(d_x, d_out, P * C, st))) {
      return rc;
    }
  }
  p.end();
  return 0;
}

int cwt_mmn_blend_backward(cwt_ctx* ctx, const float* d_fq, const float* d_att_mean, int B, int64_t n, float att_wt,
                           float* d_att, float* d_fq_in, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(d_att && B >= 1 && n >= 1, "bad arguments");
  CWT_HIP(hipSetDevice(ctx->device));
  return launch_mmn_blend_bwd(d_fq, d_att_mean, B, (long)n, att_wt, d_att, d_fq_in, (hipStream_t)stream);
}

int cwt_mmn_blend(cwt_ctx* ctx, const float* f_q, const float* att_fq, int B, int64_t n, float att_wt,
                  float* att_mean, float* fq_out, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(f_q && att_fq && att_mean && fq_out && B >= 1 && n >= 1, "bad arguments");
  CWT_HIP(hipSetDevice(ctx->device));
  return launch_mmn_blend(f_q, att_fq, B, (long)n, att_wt, att_mean, fq_out, (hipStream_t)stream);
}

int cwt_linear(cwt_ctx* ctx, const float* x, int64_t P, int K, const float* w, const float* bias, int N, int relu,
               int accumulate, float* out, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(x && w && out && P >= 1 && K >= 4 && K % 4 == 0 && N >= 1 && P <= (1L << 30), "bad arguments");
  CWT_HIP(hipSetDevice(ctx->device));
  hipStream_t st = (hipStream_t)stream;
  void* tmp;
  int rc;
  if ((rc = ensure_ws(ctx, "linear.tmp", (size_t)P * N * 4, &tmp))) return rc;
  Prof p(ctx, st, "linear " + std::to_string(K) + "x" + std::to_string(N), 2.0 * P * N * K,
         4.0 * ((double)P * K + (double)N * K + (double)P * N));
  if (!accumulate && gemm_f32d_ok((int)P, N, K, x, w, out, nullptr)) {  // (tmp + bias), relu: the epilogue's order
    if ((rc = gemm_f32d(ctx, x, w, (int)P, N, K, out, bias, nullptr, 0, st, relu))) return rc;
  } else {
    if (gemm_f32d_ok((int)P, N, K, x, w, tmp, nullptr)) {
      if ((rc = gemm_f32d(ctx, x, w, (int)P, N, K, (float*)tmp, nullptr, nullptr, 0, st))) return rc;
    } else if ((rc = launch_gemm_abt(x, w, 1, (int)P, N, K, (float*)tmp, st))) {
      return rc;
    }
    if ((rc = launch_linear_epilogue((const float*)tmp, bias, accumulate ? out : nullptr, (long)P, N, relu, out, st)))
      return rc;
  }
  p.end();
  return 0;
}

int cwt_sine_pos_add(cwt_ctx* ctx, const float* x, int B, int h, int w, int C, float temperature, int normalize,
                     float scale, float eps, float* out, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(x && out && B >= 1 && h >= 1 && w >= 1 && C >= 2 && C % 2 == 0 && temperature > 0.f, "bad arguments");
  CWT_HIP(hipSetDevice(ctx->device));
  return launch_sine_pos_add(x, B, h, w, C, temperature, normalize, scale, eps, out, (hipStream_t)stream);
}

int cwt_deform_attn(cwt_ctx* ctx, const float* value, const float* offsets, const float* logits, int B, int H, int W,
                    int n_heads, int n_points, int d_head, float* out, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(value && offsets && logits && out && B >= 1 && H >= 1 && W >= 1 && n_heads >= 1 && n_points >= 1 &&
                d_head >= 1,
            "bad arguments");
  CWT_HIP(hipSetDevice(ctx->device));
  hipStream_t st = (hipStream_t)stream;
  Prof p(ctx, st, "deform_attn", 2.0 * B * H * W * n_heads * n_points * d_head * 5,
         4.0 * (double)B * H * W * n_heads * (d_head * 2 + n_points * 3));
  int rc = launch_deform_attn(value, offsets, logits, B, H, W, n_heads, n_points, d_head, out, st);
  p.end();
  return rc;
}

int cwt_norm_blend(cwt_ctx* ctx, const float* a, const float* b, int64_t T, int C, float wt, float* out,
                   void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(a && b && out && T >= 1 && C >= 1, "bad arguments");
  CWT_HIP(hipSetDevice(ctx->device));
  return launch_norm_blend(a, b, (long)T, C, wt, out, (hipStream_t)stream);
}

// ---- DeTr head backward (train_trans.py:100): linear / 1x1 conv, deformable attention, blend ----
int cwt_linear_backward(cwt_ctx* ctx, const float* x, int64_t P, int K, const float* w, int N, const float* out,
                        const float* d_out, float* d_x, float* d_w, int ldw, float* d_b, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(x && w && d_out && P >= 1 && K >= 1 && N >= 1 && P <= (1L << 30) && (!d_w || ldw >= K), "bad arguments");
  CWT_HIP(hipSetDevice(ctx->device));
  hipStream_t st = (hipStream_t)stream;
  const long ldN = ld32(N), ldP = ld32(P);
  void *gm, *wt, *gt, *xt, *dw;
  int rc;
  if ((rc = ensure_ws(ctx, "lb.gm", (size_t)P * ldN * 4, &gm))) return rc;
  Prof p(ctx, st, "linear_backward " + std::to_string(K) + "x" + std::to_string(N), 4.0 * P * N * K,
         4.0 * ((double)P * K * 2 + (double)N * K * 2 + (double)P * N * 2));
  // the output gradient through the ReLU (out > 0) when out is given
  const float* g = d_out;
  if (out) {
    if ((rc = launch_relu_mask(d_out, out, P * N, (float*)gm, st))) return rc;
    g = (const float*)gm;
  }
  if (d_b) {
    void* csw;
    const size_t csn = colsum_ws_floats(P, N);
    if ((rc = ensure_ws(ctx, "colsum", csn * 4, &csw)) || (rc = launch_colsum(g, P, N, N, 0, d_b, (float*)csw, csn, st)))
      return rc;
  }
  if (d_x) {  // d x = g . w   (A = g [P][ldN], B^T = w^T [K][ldN])
    const float* gp = g;
    if (ldN != N) {
      void* gpad;
      if ((rc = ensure_ws(ctx, "lb.gpad", (size_t)P * ldN * 4, &gpad)) ||
          (rc = launch_copy_pad(g, P, N, (int)ldN, (float*)gpad, st)))
        return rc;
      gp = (const float*)gpad;
    }
    if ((rc = ensure_ws(ctx, "lb.wT", (size_t)K * ldN * 4, &wt)) ||
        (rc = launch_match_vt(w, 1, N, K, (int)ldN, (float*)wt, st)) ||
        (rc = gemm_nt(ctx, gp, (const float*)wt, (int)P, K, (int)ldN, d_x, st)))
      return rc;
  }
  if (d_w) {  // d w = g^T . x   (A = g^T [N][ldP], B^T = x^T [K][ldP])
    if ((rc = ensure_ws(ctx, "lb.gT", (size_t)N * ldP * 4, &gt)) || (rc = ensure_ws(ctx, "lb.xT", (size_t)K * ldP * 4, &xt)) ||
        (rc = launch_match_vt(g, 1, (int)P, N, (int)ldP, (float*)gt, st)) ||
        (rc = launch_match_vt(x, 1, (int)P, K, (int)ldP, (float*)xt, st)))
      return rc;
    float* dst = d_w;
    if (ldw != K) {
      if ((rc = ensure_ws(ctx, "lb.dw", (size_t)N * K * 4, &dw))) return rc;
      dst = (float*)dw;
    }
    if ((rc = gemm_nt(ctx, (const float*)gt, (const float*)xt, N, K, (int)ldP, dst, st))) return rc;
    if (ldw != K && (rc = launch_copy_2d(dst, N, K, K, d_w, ldw, st))) return rc;
  }
  p.end();
  return 0;
}

int cwt_deform_attn_backward(cwt_ctx* ctx, const float* value, const float* offsets, const float* logits, int B, int H,
                             int W, int n_heads, int n_points, int d_head, const float* d_out, float* d_value,
                             float* d_offsets, float* d_logits, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(value && offsets && logits && d_out && d_value && d_offsets && d_logits && B >= 1 && H >= 1 && W >= 1 &&
                n_heads >= 1 && n_points >= 1 && d_head >= 1,
            "bad arguments");
  CWT_HIP(hipSetDevice(ctx->device));
  hipStream_t st = (hipStream_t)stream;
  Prof p(ctx, st, "deform_attn_backward", 2.0 * B * H * W * n_heads * n_points * d_head * 12,
         4.0 * (double)B * H * W * n_heads * (d_head * 7 + n_points * 6));
  void* ws;
  int rc;
  if ((rc = ensure_ws(ctx, "detr.dv64", deform_attn_bwd_ws_bytes(B, H, W, n_heads, d_head), &ws))) return rc;
  rc = launch_deform_attn_bwd(value, offsets, logits, B, H, W, n_heads, n_points, d_head, d_out, d_value, d_offsets,
                              d_logits, ws, st);
  p.end();
  return rc;
}

int cwt_norm_blend_backward(cwt_ctx* ctx, const float* a, const float* b, int64_t T, int C, float wt, const float* d_out,
                            float* d_a, float* d_b, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(a && b && d_out && T >= 1 && C >= 1, "bad arguments");
  CWT_HIP(hipSetDevice(ctx->device));
  return launch_norm_blend_bwd(a, b, d_out, (long)T, C, wt, d_a, d_b, (hipStream_t)stream);
}

int cwt_seg_metrics(cwt_ctx* ctx, const float* logits, const int64_t* target, int B, int h, int w, int S,
                    float* iut_out, double* ce_out, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(logits && target && iut_out && B >= 1 && B <= 64 && h >= 1 && w >= 1 && S >= 1, "bad arguments");
  CWT_HIP(hipSetDevice(ctx->device));
  void* cnt;
  int rc;
  if ((rc = ensure_ws(ctx, "metrics.cnt", (size_t)B * 256 * (2 * 6 * 4 + 2 * 8) + 16, &cnt))) return rc;
  return launch_seg_metrics(logits, target, B, h, w, S, iut_out, ce_out, (unsigned*)cnt, (hipStream_t)stream);
}

int cwt_seg_metrics_pair(cwt_ctx* ctx, const float* logits, const float* logits0, const int64_t* target, int B,
                         int h, int w, int S, float* iut_out, double* ce_out, float* iut0_out, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(logits && logits0 && target && iut_out && iut0_out && B >= 1 && B <= 64 && h >= 1 && w >= 1 && S >= 1,
            "bad arguments");
  CWT_HIP(hipSetDevice(ctx->device));
  void* cnt;
  int rc;
  if ((rc = ensure_ws(ctx, "metrics.cnt", (size_t)B * 256 * (2 * 6 * 4 + 2 * 8) + 16, &cnt))) return rc;
  return launch_seg_metrics(logits, target, B, h, w, S, iut_out, ce_out, (unsigned*)cnt, (hipStream_t)stream,
                            logits0, iut0_out);
}

int cwt_seg_ce_fwd_bwd(cwt_ctx* ctx, const float* logits, const int64_t* target, int B, int h, int w, int S,
                       float* loss_out, float* dlogits, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(logits && target && loss_out && dlogits && B >= 1, "bad arguments");
  CWT_CHECK(S - 1 == 8 * (h - 1) && S - 1 == 8 * (w - 1), "need S-1 == 8*(h-1) == 8*(w-1)");
  CWT_HIP(hipSetDevice(ctx->device));
  void *lbl, *sc, *num;
  int rc;
  if ((rc = ensure_ws(ctx, "ce.lbl", (size_t)B * S * S, &lbl))) return rc;
  if ((rc = ensure_ws(ctx, "ce.sc", 8192, &sc))) return rc;
  if ((rc = ensure_ws(ctx, "ce.num", 64, &num))) return rc;
  return launch_seg_ce(logits, target, B, h, w, S, loss_out, dlogits, (uint8_t*)lbl, (AdaptScalars*)sc,
                       (double*)num, (hipStream_t)stream);
}

int cwt_debug_conv(cwt_ctx* ctx, const float* x, int N, int Hi, int Wi, int Ci, int x_ld, const float* w_packed,
                   const float* scale, const float* shift, int Co, int k, int stride, int pad, int dil,
                   const float* res, int res_ld, int relu, float* y, int y_ld, int y_off, int bm, int bn,
                   int nsplit, int precision, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(x && w_packed && scale && shift && y, "null buffer");
  CWT_CHECK(Ci % 32 == 0 && Co % 64 == 0 && x_ld >= Ci && y_ld >= y_off + Co, "need Ci%32==0, Co%64==0");
  CWT_HIP(hipSetDevice(ctx->device));
  ConvLayer L;
  L.Ci = Ci;
  L.Co = Co;
  L.k = k;
  L.stride = stride;
  L.pad = pad;
  L.dil = dil;
  L.w = (float*)w_packed;
  int rc;
  if (k > 1) {  // caller layout [Co][k][k][Ci] -> packed_k order
    void* wp;
    if ((rc = ensure_ws(ctx, "dbg.wpack", (size_t)Co * k * k * Ci * 4, &wp))) return rc;
    if ((rc = launch_repack_cblock(w_packed, (float*)wp, Co, k * k, Ci, (hipStream_t)stream))) return rc;
    L.w = (float*)wp;
    w_packed = L.w;
  }
  L.scale = (float*)scale;
  L.shift = (float*)shift;
  ConvCall c{0, &L, x, N, Hi, Wi, x_ld, y, y_ld, y_off, res, res_ld, relu, true};
  ConvArgs a = make_args(c);
  CWT_CHECK(precision == 0, "cwt_debug_conv runs the exact-fp32 conv only (bf16x3 plans: cwt_debug_conv_s)");
  ConvPlan p = plan_conv(a.M, a.Co, a.K);
  if (bm > 0) {
    CWT_CHECK((bm == 128 && (bn == 128 || bn == 64)) || (bm == 64 && bn == 64), "tile must be 128x128, 128x64 or 64x64");
    CWT_CHECK(Co % bn == 0, "Co % bn");
    p.bm = bm;
    p.bn = bn;
  }
  if (nsplit > 0) {
    const int kt = a.K / 32;
    p.kt_per_split = cdiv(kt, nsplit);
    p.nsplit = cdiv(kt, p.kt_per_split);
  }
  void* part = nullptr;
  size_t pf = (size_t)p.nsplit * a.M * a.Co;
  if (p.nsplit > 1 && (rc = ensure_ws(ctx, "dbg.PART", pf * 4, &part))) return rc;
  return launch_conv(a, p, 0, (float*)part, pf, (hipStream_t)stream);
}

}  // extern "C"

namespace cwt {
// HW_REG_HW_ID (wave, SIMD, CU, SH, SE fields) and HW_REG_XCC_ID of each workgroup's first wave
__global__ void census_kernel(unsigned* out) {
  unsigned hw, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = hw;
    out[2 * blockIdx.x + 1] = xcc;
  }
}
}  // namespace cwt

extern "C" {

int cwt_debug_census(cwt_ctx* ctx, int nblocks, unsigned* out, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(out && nblocks > 0, "bad arguments");
  CWT_HIP(hipSetDevice(ctx->device));
  hipLaunchKernelGGL(census_kernel, dim3(nblocks), dim3(64), 0, (hipStream_t)stream, out);
  CWT_LAUNCH_CHECK();
  return 0;
}

int cwt_debug_split_act(cwt_ctx* ctx, const float* x, int64_t P, int C, int ld, void* out, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(x && out && P >= 0 && C % 32 == 0 && ld >= C && ld % 4 == 0, "bad arguments");
  CWT_HIP(hipSetDevice(ctx->device));
  return launch_split_act(x, P, C, ld, (__bf16*)out, (hipStream_t)stream);
}

int cwt_debug_unsplit_act(cwt_ctx* ctx, const void* s, int64_t P, int C, float* out, int ld, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(s && out && P >= 0 && C % 32 == 0 && ld >= C && ld % 4 == 0, "bad arguments");
  CWT_HIP(hipSetDevice(ctx->device));
  return launch_unsplit_act((const __bf16*)s, P, C, out, ld, (hipStream_t)stream);
}

int cwt_debug_pack_wsplit(cwt_ctx* ctx, const float* w, int Co, int k, int Ci, void* out, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(w && out && Co > 0 && Ci % 32 == 0 && (k == 1 || k == 3), "bad arguments");
  CWT_HIP(hipSetDevice(ctx->device));
  void* wp;
  int rc;
  const long K = (long)k * k * Ci;
  if ((rc = ensure_ws(ctx, "dbg.wpack", (size_t)Co * K * 4, &wp))) return rc;
  if ((rc = launch_repack_cblock(w, (float*)wp, Co, k * k, Ci, (hipStream_t)stream))) return rc;
  return launch_split_act((const float*)wp, Co, (int)K, (int)K, (__bf16*)out, (hipStream_t)stream);
}

}  // extern "C"

static int debug_conv_s(cwt_ctx* ctx, int prec, const void* xs, int N, int Hi, int Wi, int Ci, const void* ws,
                        const float* scale, const float* shift, int Co, int k, int stride, int pad, int dil,
                        const float* res, int res_ld, const void* res_s, int relu, float* y, int y_ld, int y_off,
                        void* ys, int bm, int bn, int nsplit, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(xs && ws && scale && shift && (y || ys), "null buffer");
  const int kb = prec == 1 ? 64 : 32;
  CWT_CHECK(Ci % kb == 0 && Co % 64 == 0, prec == 1 ? "need Ci%64==0, Co%64==0" : "need Ci%32==0, Co%64==0");
  CWT_CHECK(!y || (y_ld >= y_off + Co && y_ld % 4 == 0 && y_off % 4 == 0), "bad y stride");
  CWT_HIP(hipSetDevice(ctx->device));
  ConvSArgs a;
  memset(&a, 0, sizeof(a));
  int rc;
  if ((rc = zero_line(ctx, &a.zero))) return rc;
  a.xs = (const __bf16*)xs;
  a.ws = (const __bf16*)ws;
  a.scale = scale;
  a.shift = shift;
  a.res = res;
  a.res_ld = res_ld;
  a.res_s = (const __bf16*)res_s;
  a.relu = relu;
  a.y = y;
  a.y_ld = y_ld;
  a.y_off = y_off;
  a.ys = (__bf16*)ys;
  a.N = N;
  a.Hi = Hi;
  a.Wi = Wi;
  a.Ci = Ci;
  a.Co = Co;
  a.kh = a.kw = k;
  a.stride = stride;
  a.pad = pad;
  a.dil = dil;
  a.Ho = (Hi + 2 * pad - dil * (k - 1) - 1) / stride + 1;
  a.Wo = (Wi + 2 * pad - dil * (k - 1) - 1) / stride + 1;
  a.M = N * a.Ho * a.Wo;
  a.K = k * k * Ci;
  ConvPlan p = prec == 1   ? plan_conv_b16(a.M, a.Co, a.K)
               : prec == 0 ? plan_conv_f32d(a.M, a.Co, a.K)
               : prec == 6 ? plan_conv_x6(a.M, a.Co, a.K)
                           : plan_conv_x3s(a.M, a.Co, a.K);
  if (bm > 0) {
    const int var = bm / 1000;  // bm = 1000 * variant + rows (cwt_debug.h)
    bm %= 1000;
    CWT_CHECK((bm == 256 && (bn == 256 || bn == 128)) || (bm == 128 && (bn == 256 || bn == 128 || bn == 64)) ||
                  (bm == 64 && (bn == 128 || bn == 64)),
              "tile must be one of 256x256, 256x128, 128x256, 128x128, 128x64, 64x128, 64x64");
    const bool x6_var = prec == 6 && ((var == 3 && (bm >= 128 && bn >= 128)) || (var == 5 && bm == 128 && bn == 128) ||
                                      ((var == 3 || var == 5) && bm == 64 && bn == 128) ||
                                      ((var == 3 || var == 5) && bm == 128 && bn == 64) || (var == 3 && bm == 64 && bn == 64) ||
                                      ((var == 12 || (var >= 14 && var <= 18)) && bm == 128 && bn == 128) ||
                                      (var == 13 && bm == 256 && bn == 256));
    CWT_CHECK((var >= 0 && var <= 2) || (var == 4 && bm == 128 && bn == 128) || (var >= 8 && var <= 11) || x6_var,
              "variant must be 0, 1, 2, 4 (128x128 only), 8 .. 11 (timing study), or for x6 3 (tiles >= 128x128) "
              "and 5 (128x128)");
    if (var >= 8 && var <= 11 && !x6_var) {  // the timing-study kernels have fixed tiles: the grid must be theirs
      bm = bn = var < 10 ? 64 : 128;
    }
    CWT_CHECK(Co % bn == 0, "Co % bn");
    p.bm = bm;
    p.bn = bn;
    p.var = var;
  }
  if (nsplit > 0) {
    const int kt = a.K / kb;
    p.kt_per_split = cdiv(kt, nsplit);
    p.nsplit = cdiv(kt, p.kt_per_split);
  }
  if (prec == 6) {  // the fp32 packed weights -> the x6 kernel's hi | mid line and lo plane
    void *w3s, *w3l;
    if ((rc = ensure_ws(ctx, "dbg.w3s", (size_t)Co * a.K * 4, &w3s)) ||
        (rc = ensure_ws(ctx, "dbg.w3l", (size_t)Co * a.K * 2, &w3l)))
      return rc;
    // CWT_DBG_W3_CACHE=1 (timing tools that call the same conv repeatedly): split the weights only when
    // the source buffer or its shape changes, so the timed calls are the conv alone
    static const bool w3_cache = getenv("CWT_DBG_W3_CACHE") && getenv("CWT_DBG_W3_CACHE")[0] == '1';
    static const void* w3_src = nullptr;
    static long w3_n = 0;
    static void* w3_dst = nullptr;
    if (!(w3_cache && w3_src == ws && w3_n == (long)Co * a.K && w3_dst == w3s)) {
      if ((rc = launch_split_w3((const float*)ws, Co, a.K, (__bf16*)w3s, (__bf16*)w3l, (hipStream_t)stream))) return rc;
      w3_src = ws;
      w3_n = (long)Co * a.K;
      w3_dst = w3s;
    }
    a.ws = (const __bf16*)w3s;
    a.ws_lo = (const __bf16*)w3l;
  }
  void* part = nullptr;
  const size_t pf = (size_t)p.nsplit * a.M * a.Co;
  if (p.nsplit > 1 && (rc = ensure_ws(ctx, "dbg.PART", pf * 4, &part))) return rc;
  return launch_conv_x3s(a, p, 0, (float*)part, pf, (hipStream_t)stream, prec);
}

extern "C" {

int cwt_debug_conv_s(cwt_ctx* ctx, const void* xs, int N, int Hi, int Wi, int Ci, const void* ws, const float* scale,
                     const float* shift, int Co, int k, int stride, int pad, int dil, const float* res, int res_ld,
                     const void* res_s, int relu, float* y, int y_ld, int y_off, void* ys, int bm, int bn, int nsplit,
                     void* stream) {
  return debug_conv_s(ctx, 3, xs, N, Hi, Wi, Ci, ws, scale, shift, Co, k, stride, pad, dil, res, res_ld, res_s, relu, y,
                      y_ld, y_off, ys, bm, bn, nsplit, stream);
}

int cwt_debug_conv_f32d(cwt_ctx* ctx, const float* x, int N, int Hi, int Wi, int Ci, const float* w_packed,
                        const float* scale, const float* shift, int Co, int k, int stride, int pad, int dil,
                        const float* res, int res_ld, int relu, float* y, int y_ld, int y_off, int bm, int bn,
                        int nsplit, void* stream) {
  return debug_conv_s(ctx, 0, x, N, Hi, Wi, Ci, w_packed, scale, shift, Co, k, stride, pad, dil, res, res_ld, nullptr,
                      relu, y, y_ld, y_off, nullptr, bm, bn, nsplit, stream);
}

int cwt_debug_conv_x6(cwt_ctx* ctx, const float* x, int N, int Hi, int Wi, int Ci, const float* w_packed,
                      const float* scale, const float* shift, int Co, int k, int stride, int pad, int dil,
                      const float* res, int res_ld, int relu, float* y, int y_ld, int y_off, int bm, int bn,
                      int nsplit, void* stream) {
  return debug_conv_s(ctx, 6, x, N, Hi, Wi, Ci, w_packed, scale, shift, Co, k, stride, pad, dil, res, res_ld, nullptr,
                      relu, y, y_ld, y_off, nullptr, bm, bn, nsplit, stream);
}

int cwt_debug_conv_x6w(cwt_ctx* ctx, const float* x, int N, int Hi, int Wi, int Ci, const float* w_packed,
                       const float* scale, const float* shift, int Co, int k, int stride, int pad, int dil,
                       const float* res, int res_ld, int relu, float* y, int y_ld, int y_off, int bm, int bn,
                       int nsplit, void* stream) {
  const int m = nsplit == 4 ? 4 : 2;  // nsplit selects the output tile: 4 = F(4x4,3x3), else F(2x2,3x3)
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(x && w_packed && scale && shift && y, "null buffer");
  CWT_CHECK(nsplit == 0 || nsplit == 1 || nsplit == 2 || nsplit == 4, "nsplit (the Winograd tile) must be 0, 2 or 4");
  CWT_CHECK(k == 3 && stride == 1 && pad == dil && dil >= 1, "winograd form: 3x3, stride 1, padding = dilation");
  CWT_CHECK(Ci % 32 == 0 && Co % 64 == 0 && N >= 1 && Hi >= 1 && Wi >= 1, "need Ci % 32 == 0, Co % 64 == 0");
  CWT_CHECK(y_ld >= y_off + Co && y_ld % 4 == 0 && y_off % 4 == 0 && (!res || res_ld % 4 == 0), "bad strides");
  CWT_CHECK(bm == 0 || ((bm % 1000 == 256 || bm % 1000 == 128 || bm % 1000 == 64) && (bn == 256 || bn == 128 || bn == 64)),
            "bad tile");
  CWT_HIP(hipSetDevice(ctx->device));
  const hipStream_t st = (hipStream_t)stream;
  const int P = (m + 2) * (m + 2);
  const size_t n = (size_t)P * Co * Ci;
  void *U, *us, *ul;
  int rc;
  if ((rc = ensure_ws(ctx, "dbg.wU", n * 4, &U)) || (rc = ensure_ws(ctx, "dbg.wUs", n * 4, &us)) ||
      (rc = ensure_ws(ctx, "dbg.wUl", n * 2, &ul)))
    return rc;
  // CWT_DBG_W3_CACHE=1: transform and split the weights only when their source or shape changes
  static const bool w3_cache = getenv("CWT_DBG_W3_CACHE") && getenv("CWT_DBG_W3_CACHE")[0] == '1';
  static const void* u_src = nullptr;
  static long u_n = 0;
  static void* u_dst = nullptr;
  if (!(w3_cache && u_src == w_packed && u_n == (long)n * m && u_dst == us)) {
    if ((rc = launch_wino_weights(w_packed, Co, Ci, (float*)U, st, m)) ||
        (rc = launch_split_w3((const float*)U, (long)P * Co, Ci, (__bf16*)us, (__bf16*)ul, st)))
      return rc;
    u_src = w_packed;
    u_n = (long)n * m;
    u_dst = us;
  }
  return run_wino_conv(ctx, x, N, Hi, Wi, Ci, Co, dil, m, (const __bf16*)us, (const __bf16*)ul, scale, shift, res,
                       res_ld, relu, y, y_ld, y_off, 0, st, bm, bn);
}

int cwt_debug_conv_b16(cwt_ctx* ctx, const void* xs, int N, int Hi, int Wi, int Ci, const void* ws, const float* scale,
                       const float* shift, int Co, int k, int stride, int pad, int dil, const float* res, int res_ld,
                       const void* res_s, int relu, float* y, int y_ld, int y_off, void* ys, int bm, int bn,
                       int nsplit, void* stream) {
  return debug_conv_s(ctx, 1, xs, N, Hi, Wi, Ci, ws, scale, shift, Co, k, stride, pad, dil, res, res_ld, res_s, relu, y,
                      y_ld, y_off, ys, bm, bn, nsplit, stream);
}

// one CenterPivotConv4d layer (+ ReLU) on [B][NA][NB][cin] -> [B][NA][NB][cout] (launch_cp4d_layer);
// variant 0 the automatic kernel choice, 1 never the rolling-window form, 2 only it
int cwt_debug_cp4d_layer(cwt_ctx* ctx, const float* x, int B, int hA, int wA, int hB, int wB, int cin, int cout,
                         const float* Wa, const float* ba, const float* Wb, const float* bb, float* y, int variant,
                         void* stream) {
  if (!ctx || !x || !Wa || !ba || !Wb || !bb || !y) return fail(CWT_EARG, "null argument");
  if (B < 1 || hA < 1 || wA < 1 || hB < 1 || wB < 1) return fail(CWT_EARG, "bad shape");
  return launch_cp4d_layer_variant(x, B, hA, wA, hB, wB, cin, cout, Wa, ba, Wb, bb, y, variant, (hipStream_t)stream);
}

int cwt_debug_occupy(cwt_ctx* ctx, int nwg, int us, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(nwg >= 1 && nwg <= 256 && us >= 1 && us <= 100000, "occupy: 1 <= nwg <= 256, 1 <= us <= 100000");
  CWT_HIP(hipSetDevice(ctx->device));
  return launch_occupy(nwg, us, (hipStream_t)stream);
}

int cwt_debug_tail_stamps(cwt_ctx* ctx, unsigned long long* host_out, int64_t max_count, int64_t* count) {
  if (!ctx || !count) return fail(CWT_EARG, "null argument");
  CWT_HIP(hipSetDevice(ctx->device));
  auto it = ctx->ws.find("tail.stamps");
  *count = (it == ctx->ws.end() || !ctx->tail_stamp_G) ? 0 : (int64_t)ctx->tail_stamp_G * 16;
  if (host_out && *count > 0 && max_count > 0) {
    CWT_HIP(hipDeviceSynchronize());
    CWT_HIP(hipMemcpy(host_out, it->second.p, (size_t)std::min<int64_t>(max_count, *count) * 8, hipMemcpyDeviceToHost));
  }
  return 0;
}

int cwt_debug_adapt_stamps(cwt_ctx* ctx, unsigned long long* host_out, int64_t max_count, int64_t* count) {
  if (!ctx || !count) return fail(CWT_EARG, "null argument");
  CWT_HIP(hipSetDevice(ctx->device));
  *count = g_adapt_stamps ? g_adapt_stamps_n : 0;
  if (host_out && g_adapt_stamps && max_count > 0) {
    CWT_HIP(hipDeviceSynchronize());
    CWT_HIP(hipMemcpy(host_out, g_adapt_stamps, (size_t)std::min<int64_t>(max_count, g_adapt_stamps_n) * 8,
                      hipMemcpyDeviceToHost));
  }
  return 0;
}

int cwt_iou_preds(cwt_ctx* ctx, const int64_t* preds, const int64_t* target, int64_t n, int num_classes,
                  int ignore_index, float* iut_out, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(preds && target && iut_out && n >= 0 && num_classes >= 1 && num_classes <= 16, "bad arguments");
  CWT_HIP(hipSetDevice(ctx->device));
  void* cnt;
  int rc;
  if ((rc = ensure_ws(ctx, "iou.cnt", 3 * 16 * 4, &cnt))) return rc;
  return launch_iou_preds(preds, target, n, num_classes, ignore_index, iut_out, (unsigned*)cnt, (hipStream_t)stream);
}

int cwt_ctx_set_conv_arith(cwt_ctx* ctx, int arith) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(arith == CWT_CONV_ARITH_BF16X3 || arith == CWT_CONV_ARITH_F32 || arith == CWT_CONV_ARITH_BF16X6,
            "arith must be CWT_CONV_ARITH_BF16X3 (0), CWT_CONV_ARITH_F32 (1) or CWT_CONV_ARITH_BF16X6 (2)");
  ctx->conv_arith = arith;
  return 0;
}

int cwt_debug_adapt_spin_limit(cwt_ctx* ctx, int64_t limit) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(limit >= 0, "limit must be >= 0");
  ctx->adapt_spin_limit = (long)limit;
  return 0;
}

int cwt_ctx_set_adapt_units(cwt_ctx* ctx, int units_per_workgroup) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(units_per_workgroup >= 0 && units_per_workgroup <= 3, "units per workgroup must be 0 (automatic), 1, 2 or 3");
  ctx->adapt_upw = units_per_workgroup;
  return 0;
}

int cwt_profile_enable(cwt_ctx* ctx, int on) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  ctx->prof_level = on;
  if (on) {
    ctx->recs.clear();
    ctx->ev_used = 0;
  }
  return 0;
}

int cwt_profile_count(cwt_ctx* ctx) { return ctx ? (int)ctx->recs.size() : 0; }

int cwt_profile_record(cwt_ctx* ctx, int i, char* name, int name_len, double* flops, double* bytes, float* ms) {
  if (!ctx || i < 0 || i >= (int)ctx->recs.size()) return fail(CWT_EARG, "no such profile record");
  auto& r = ctx->recs[i];
  if (name && name_len > 0) {
    strncpy(name, r.name.c_str(), name_len - 1);
    name[name_len - 1] = 0;
  }
  if (flops) *flops = r.flops;
  if (bytes) *bytes = r.bytes;
  if (ms) {
    CWT_HIP(hipEventSynchronize(r.e1));
    if (r.fslot >= 0) {  // a fused loop + tail launch: its part from the kernel's realtime stamps (100 MHz)
      unsigned long long v[3];
      CWT_HIP(hipMemcpy(v, ctx->fstamps + 3 * r.fslot, sizeof(v), hipMemcpyDeviceToHost));
      const unsigned long long t0 = r.fpart ? v[1] : v[0], t1 = r.fpart ? v[2] : v[1];
      *ms = t1 > t0 ? (float)((double)(t1 - t0) * 1e-5) : 0.f;
    } else {
      CWT_HIP(hipEventElapsedTime(ms, r.e0, r.e1));
    }
  }
  return 0;
}

int cwt_adapt_workgroups(cwt_ctx* ctx, int E, int n, int h, int w, int iters, int* G) {
  if (!ctx || !G || E < 1 || n < 1 || h < 2 || w < 2) return fail(CWT_EARG, "bad arguments");
  CWT_HIP(hipSetDevice(ctx->device));
  *G = adapt_persist_workgroups(E, n, h, w, iters, ctx->adapt_upw);
  return 0;
}

int cwt_adapt_fuses_tail(cwt_ctx* ctx, int n, int h, int w, int iters, int* fused) {
  if (!ctx || !fused || n < 1 || h < 2 || w < 2 || iters < 0) return fail(CWT_EARG, "bad arguments");
  CWT_HIP(hipSetDevice(ctx->device));
  *fused = fused_tail_applies(ctx, n, h, w, iters) ? 1 : 0;
  return 0;
}

int cwt_cu_count(cwt_ctx* ctx, int* count) {
  if (!ctx || !count) return fail(CWT_EARG, "null argument");
  hipDeviceProp_t prop;
  CWT_HIP(hipGetDeviceProperties(&prop, ctx->device));
  *count = prop.multiProcessorCount;
  return 0;
}

int cwt_stream_create_masked(cwt_ctx* ctx, const uint32_t* mask, int mask_words, void** stream) {
  if (!ctx || !mask || !stream || mask_words < 1) return fail(CWT_EARG, "bad arguments");
  CWT_HIP(hipSetDevice(ctx->device));
  hipStream_t s;
  CWT_HIP(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask_words, mask));
  *stream = (void*)s;
  return 0;
}

int cwt_stream_destroy(void* stream) {
  if (!stream) return fail(CWT_EARG, "stream is NULL");
  CWT_HIP(hipStreamDestroy((hipStream_t)stream));
  return 0;
}

int cwt_sgd_step(cwt_ctx* ctx, float* param, const float* grad, float* momentum_buf, int64_t n, float lr,
                 float momentum, float weight_decay, int nesterov, int first_step, void* stream) {
  if (!ctx) return fail(CWT_EARG, "ctx is NULL");
  CWT_CHECK(param && grad && n >= 0, "bad arguments");
  CWT_CHECK(momentum == 0.f || momentum_buf, "momentum needs a buffer");
  CWT_HIP(hipSetDevice(ctx->device));
  return launch_sgd(param, grad, momentum_buf, n, lr, momentum, weight_decay, nesterov, first_step,
                    (hipStream_t)stream);
}

}  // extern "C"

// The post-loop episode tail in ONE launch (test.py:190-224 after the inner loop):
//   pred_q0 = W . f_q,  f_hat = F.normalize(f_q),  W' = CWT(W, f_hat, f_hat)  (transformer.py:54-83),
//   pred_q = W' . f_hat,  upsample + argmax + intersection / union / target + CE of pred_q and
//   pred_q0 against q_label (util.py:237-308, test.py:214-224).
// The module-by-module form is 8 dependent launches (rowdot, token pass, combine, rowdot,
// LayerNorm, classifier, metrics, metrics final: cwt_attention_infer + cwt_classify_scaled +
// cwt_seg_metrics_pair), each of them a small kernel near the ~4-us floor of a dependent launch.
// Here one grid of G co-resident 512-thread workgroups runs the same phases back to back,
// separated by in-kernel grid barriers (the persistent inner loop's counter barrier: replicated
// arrival counters, agent-scope atomic arrivals after every storing wave's vmcnt(0), sc1 polls):
//   P0  r[v][h][k] = M_h[k] . q_v / sqrt(C)              (a wave per row of the folded M)
//   P1  token chunks: 1/||f_p||, W . f_p (pred_q0), chunk softmax partials (the token pass)
//   P2  g = softmax-weighted token means                  (chunk combine)
//   P3  y[v][j] = P[j] . g_v + fc_b[j] + q_v[j]           (a wave per row of the folded P)
//   P4  LayerNorm (every workgroup, its own copy) -> W'; pred_q = (W' . f_p) / ||f_p|| for the
//       workgroup's own token chunks
//   P5  upsample + argmax + counts + CE of pred_q and pred_q0 per pixel, per-workgroup partials;
//       the last workgroup to arrive (agent-scope ticket) sums them in workgroup order.
// Every value one workgroup hands to another is stored write-through (sc1) and loaded with sc1
// loads (MI355X_MICROARCH.md, hand-off table, first row): no L2 write-back or invalidate.  The
// arithmetic of every phase is the module kernels' (the same per-lane partitions and reduction
// trees), except the chunk combine (8 waves take every 8th chunk instead of 4 every 4th), the
// token pass's per-wave sums (added pairwise into two LDS slots: the phases' LDS is ~54 KB, so a
// tail workgroup can share a CU with an extractor conv's workgroup in the episode pipeline) and
// the order of the CE's double partial sums.  P5 gives each workgroup one contiguous pixel range
// and stages the low-res rows it reads in LDS.
// Counters are monotonic over launches: launch e's barrier k waits for G (e NBAR + k) arrivals,
// its ticket's last arriver sees e G + G - 1 (the host bumps e per launch and re-zeroes the
// counters before the 32-bit range would wrap, or after a launch aborted).
#include <cstring>

#include "tail_body.h"

namespace cwt {

template <bool ST>
__global__ __launch_bounds__(TL_T) void episode_tail_kernel(TailArgs a) {
  __shared__ __attribute__((aligned(16))) char smem_raw[sizeof(TailTok)];
  __shared__ int abort_flag, last_flag;
  episode_tail_body<ST>(a, blockIdx.x, smem_raw, abort_flag, last_flag);
}

size_t episode_tail_ws_floats(int B, int hw, int G) {
  const long nchunk = cdiv(hw, TL_TPB);
  return (size_t)(B * TL_NR * TL_C                  // r
                  + B * nchunk * TL_NR * (TL_C + 2)  // part_g, part_ml
                  + B * TL_NR * TL_C                 // g
                  + 2L * B * TL_C                    // y
                  + (long)B * hw                     // inv
                  + 2L * B * G * 6                   // counts
                  + 2L * B * G * 2 + 8);             // ce_part (doubles, 8-B aligned)
}
size_t episode_tail_cnt_words() { return (TL_REP + 2) * TL_STRIDE; }

// One launch of the tail.  fold: the folded CWT weights (attention_fold); cnt: the context's
// counters (episode_tail_cnt_words, zeroed when created); epoch: this launch's number on them.
int fill_episode_tail_args(const float* q, const float* f, int B, int hw, int h, int w, int S, const int64_t* target,
                           const float* fold, const float* fc_b, const float* ln_w, const float* ln_b, float* out,
                           float* logits, float* logits0, float* iut, double* ce, float* iut0, float* ws,
                           unsigned* cnt, unsigned epoch, int G, long spin_limit, unsigned* status,
                           unsigned long long* stamps, TailArgs* out_args) {
  if (B < 1 || B > TL_MAXB || hw < 1 || hw > TL_MAXCHUNK * TL_TPB || h * w != hw || G < 1 || G > TL_T)
    return fail(CWT_EARG, "episode_tail: need 1 <= B <= 4, hw = h*w <= 16384, 1 <= G <= 512");
  TailArgs& a = *out_args;
  std::memset(&a, 0, sizeof(a));
  const int nchunk = cdiv(hw, TL_TPB);
  a.q = q;
  a.f = f;
  a.M = fold;
  a.P = fold + (size_t)TL_H * TL_C * TL_C;
  a.fc_b = fc_b;
  a.ln_w = ln_w;
  a.ln_b = ln_b;
  a.target = target;
  a.B = B;
  a.hw = hw;
  a.h = h;
  a.w = w;
  a.S = S;
  a.G = G;
  a.nchunk = nchunk;
  a.sy = align_corners_scale(h, S);
  a.sx = align_corners_scale(w, S);
  float* p = ws;
  a.r = p;
  p += (size_t)B * TL_NR * TL_C;
  a.part_g = p;
  p += (size_t)B * nchunk * TL_NR * TL_C;
  a.part_ml = p;
  p += (size_t)B * nchunk * TL_NR * 2;
  a.g = p;
  p += (size_t)B * TL_NR * TL_C;
  a.y = p;
  p += (size_t)2 * B * TL_C;
  a.inv = p;
  p += (size_t)B * hw;
  a.counts = (unsigned*)p;
  p += (size_t)2 * B * G * 6;
  a.ce_part = (double*)(((uintptr_t)p + 7) & ~(uintptr_t)7);
  a.out = out;
  a.logits = logits;
  a.logits0 = logits0;
  a.iut = iut;
  a.ce = ce;
  a.iut0 = iut0;
  a.cnt = cnt;
  a.bar_base = epoch * (unsigned)G * TL_NBAR;
  a.tick_base = epoch * (unsigned)G;
  a.spin_limit = spin_limit > 0 ? spin_limit : 4000000;
  a.status = status;
  a.stamps = stamps;
  return 0;
}

int launch_episode_tail(const float* q, const float* f, int B, int hw, int h, int w, int S, const int64_t* target,
                        const float* fold, const float* fc_b, const float* ln_w, const float* ln_b, float* out,
                        float* logits, float* logits0, float* iut, double* ce, float* iut0, float* ws,
                        unsigned* cnt, unsigned epoch, int G, long spin_limit, unsigned* status, hipStream_t st,
                        unsigned long long* stamps) {
  TailArgs a;
  const int rc = fill_episode_tail_args(q, f, B, hw, h, w, S, target, fold, fc_b, ln_w, ln_b, out, logits, logits0, iut,
                                        ce, iut0, ws, cnt, epoch, G, spin_limit, status, stamps, &a);
  if (rc) return rc;
  if (stamps)
    hipLaunchKernelGGL((episode_tail_kernel<true>), dim3(G), dim3(TL_T), 0, st, a);
  else
    hipLaunchKernelGGL((episode_tail_kernel<false>), dim3(G), dim3(TL_T), 0, st, a);
  CWT_LAUNCH_CHECK();
  return 0;
}

// The largest launch number the counters take before they must be re-zeroed (32-bit range).
unsigned episode_tail_max_epoch(int G) { return (unsigned)(0x7fffffffu / ((unsigned)G * TL_NBAR)) - 1u; }

}  // namespace cwt

// Stage-1 pretraining of the PSPNet (reference src/pretrain.py:104-121 with compute_loss
// :182-219 and the SGD param groups :60-72): one call = model.train(); logits = model(images);
// label-smoothed CE; zero_grad; backward over every parameter; SGD(momentum, weight decay,
// nesterov) with lr for layer0-4 and lr * scale_lr for ppm / bottleneck / classifier.
//
// Layout: every trainable tensor lives in ONE flat fp32 buffer P (gradients G and momentum
// buffers MOM alike): layer0-4 first (SGD group 1), then ppm / bottleneck / classifier
// (group 2), so the optimizer step is two launches.  Conv weights are kept in the packed
// [Co][K] order of the implicit-GEMM conv (conv.hip, packed_k) and their gradients are produced
// in that order; stem conv1 as [ci*9 + tap][co] (launch_stem_conv1); the rest as in PyTorch.
// cwt_pretrain_get converts to PyTorch layouts by name.  Activations are fp32 NHWC; the forward
// keeps each conv's raw output (for its BN backward) and each BN's output (ReLU mask, next conv's
// input for the weight gradient).  The PPM branch is folded into the bottleneck conv as in the
// episode path (its field as the conv's residual), with the field's adjoint for its gradients.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/cwt.h"
#include "../../include/cwt_debug.h"
#include "common.h"
#include "kernels.h"
#include "pretrain.h"

namespace cwt {

int ctx_device(const cwt_ctx* ctx);

static const int kPtBlocks50[4] = {3, 4, 6, 3};
static const int kPtBlocks101[4] = {3, 4, 23, 3};
static const int kPtBins[4] = {1, 2, 3, 6};
static inline int pt_down2(int x) { return (x - 1) / 2 + 1; }

enum PtKind { PT_CONV = 0, PT_STEM1 = 1, PT_PLAIN = 2 };

struct PtParam {
  std::string name;
  long off = 0, numel = 0;
  int kind = PT_PLAIN, Co = 0, Ci = 0, k = 1;
};

struct PtBn {
  int C = 0;
  long g_off = 0, b_off = 0;  // gamma / beta in P
  float* run = nullptr;       // [2][C] running mean, running var
  float* stats = nullptr;     // [2][C] mean, 1/sqrt(var + eps) of the last forward
  std::string prefix;
};

struct PtConv {
  int Ci = 0, Co = 0, k = 1, stride = 1, pad = 0, dil = 1;
  long w_off = 0;
  float* wt = nullptr;  // transposed, tap-flipped weights (input gradient), rebuilt each backward
  PtBn bn;
  // activations of the last forward
  float* y = nullptr;  // raw conv output [M][Co]
  float* a = nullptr;  // BN (+res) (+ReLU) output [M][Co] (row stride a_ld)
  int a_ld = 0;
  int Hi = 0, Ho = 0;
};

struct PtBlock {
  PtConv c1, c2, c3, down;
  bool has_down = false;
  const float* x = nullptr;  // block input (row stride x_ld)
  int x_ld = 0;
};

}  // namespace cwt

struct cwt_pretrain {
  int device = 0, layers = 50, nc = 16;
  float eps = 1e-5f;
  std::vector<cwt::PtParam> params;
  std::map<std::string, int> by_name;
  std::map<std::string, cwt::PtBn*> bn_by_name;
  long n_bb = 0, n_all = 0;
  float *P = nullptr, *G = nullptr, *MOM = nullptr;
  bool first_step = true;
  cwt::PtConv stem[3];
  std::vector<cwt::PtBlock> blocks[4];
  cwt::PtConv ppm[4];
  cwt::PtConv bott;
  long cls_off = 0;
  float *ones = nullptr, *zeros = nullptr;
  std::vector<void*> allocs;
  std::map<std::string, std::pair<void*, size_t>> ws;
  // last forward's geometry and tensors
  int N = 0, S = 0, Hs = 0, H1 = 0, h = 0;
  float *CAT = nullptr, *POOL = nullptr, *Fpre = nullptr, *F = nullptr, *LOGITS = nullptr, *MP = nullptr;
  uint8_t* MPIDX = nullptr;
  const float* img = nullptr;
  float drop_p = 0.f;
  unsigned long long seed = 0;
  // test hook (cwt_debug_pretrain_capture): copies of the backward's transient gradients at the
  // block boundaries, for the teacher-forced per-block parity test
  bool capture = false;
  std::map<std::string, std::pair<const float*, long>> cap;  // name -> (device copy, floats)
};

namespace cwt {

static int pt_alloc(cwt_pretrain* pt, size_t bytes, void** out) {
  void* p = nullptr;
  CWT_HIP(hipMalloc(&p, std::max<size_t>(bytes, 256)));
  pt->allocs.push_back(p);
  *out = p;
  return 0;
}

// named workspace, grown on demand (a step never frees it: the next call reuses it)
static int pt_ws(cwt_pretrain* pt, const std::string& name, size_t bytes, float** out) {
  auto& b = pt->ws[name];
  if (b.second < bytes) {
    if (b.first) {
      CWT_HIP(hipDeviceSynchronize());
      CWT_HIP(hipFree(b.first));
    }
    size_t nb = (bytes + 4095) & ~(size_t)4095;
    CWT_HIP(hipMalloc(&b.first, nb));
    b.second = nb;
  }
  *out = (float*)b.first;
  return 0;
}

// ---------------------------------------------------------------- parameter registry
struct PtBuilder {
  cwt_pretrain* pt;
  std::vector<std::pair<int, long>> order;  // (param index, group)
  long off = 0;
  int add(const std::string& name, long numel, int kind, int Co = 0, int Ci = 0, int k = 1) {
    PtParam p;
    p.name = name;
    p.off = off;
    p.numel = numel;
    p.kind = kind;
    p.Co = Co;
    p.Ci = Ci;
    p.k = k;
    off += (numel + 3) & ~3L;  // 16-B aligned tensors
    pt->by_name[name] = (int)pt->params.size();
    pt->params.push_back(p);
    return (int)pt->params.size() - 1;
  }
  void conv(PtConv& L, const std::string& wname, const std::string& bnp, int Ci, int Co, int k, int stride, int pad,
            int dil, bool stem1 = false) {
    L.Ci = Ci;
    L.Co = Co;
    L.k = k;
    L.stride = stride;
    L.pad = pad;
    L.dil = dil;
    L.w_off = pt->params[add(wname, (long)Co * Ci * k * k, stem1 ? PT_STEM1 : PT_CONV, Co, Ci, k)].off;
    bn(L.bn, bnp, Co);
  }
  void bn(PtBn& b, const std::string& bnp, int C) {
    b.C = C;
    b.prefix = bnp;
    b.g_off = pt->params[add(bnp + ".weight", C, PT_PLAIN)].off;
    b.b_off = pt->params[add(bnp + ".bias", C, PT_PLAIN)].off;
  }
};

static int pt_build(cwt_pretrain* pt) {
  PtBuilder B{pt};
  B.conv(pt->stem[0], "layer0.0.weight", "layer0.1", 3, 64, 3, 2, 1, 1, true);
  B.conv(pt->stem[1], "layer0.3.weight", "layer0.4", 64, 64, 3, 1, 1, 1);
  B.conv(pt->stem[2], "layer0.6.weight", "layer0.7", 64, 128, 3, 1, 1, 1);
  const int* nb = pt->layers == 50 ? kPtBlocks50 : kPtBlocks101;
  const int planes_of[4] = {64, 128, 256, 512};
  int inplanes = 128;
  for (int li = 0; li < 4; ++li) {
    const int planes = planes_of[li];
    for (int bi = 0; bi < nb[li]; ++bi) {
      PtBlock blk;
      int s2 = 1, d2 = 1, sd = 1;  // dilation surgery (pspnet.py:103-112)
      if (li == 1 && bi == 0) s2 = sd = 2;
      if (li == 2) d2 = 2;
      if (li == 3) d2 = 4;
      const std::string p = "layer" + std::to_string(li + 1) + "." + std::to_string(bi);
      B.conv(blk.c1, p + ".conv1.weight", p + ".bn1", inplanes, planes, 1, 1, 0, 1);
      B.conv(blk.c2, p + ".conv2.weight", p + ".bn2", planes, planes, 3, s2, d2, d2);
      B.conv(blk.c3, p + ".conv3.weight", p + ".bn3", planes, planes * 4, 1, 1, 0, 1);
      if (bi == 0) {
        blk.has_down = true;
        B.conv(blk.down, p + ".downsample.0.weight", p + ".downsample.1", inplanes, planes * 4, 1, sd, 0, 1);
      }
      inplanes = planes * 4;
      pt->blocks[li].push_back(blk);
    }
  }
  pt->n_bb = B.off;
  for (int i = 0; i < 4; ++i) {
    const std::string p = "ppm.features." + std::to_string(i);
    // the PPM 1x1 conv keeps PyTorch's [512][2048] layout (few-row GEMMs, not the conv kernel)
    pt->ppm[i].Ci = 2048;
    pt->ppm[i].Co = 512;
    pt->ppm[i].w_off = pt->params[B.add(p + ".1.weight", 512L * 2048, PT_PLAIN)].off;
    B.bn(pt->ppm[i].bn, p + ".2", 512);
  }
  B.conv(pt->bott, "bottleneck.0.weight", "bottleneck.1", 4096, 512, 3, 1, 1, 1);
  pt->cls_off = pt->params[B.add("classifier.weight", (long)pt->nc * 512, PT_PLAIN)].off;
  pt->n_all = B.off;
  return 0;
}

// every BN of the model (for running statistics and stats buffers)
template <typename F>
static void pt_for_each_conv(cwt_pretrain* pt, F f) {
  for (auto& c : pt->stem) f(c);
  for (int li = 0; li < 4; ++li)
    for (auto& b : pt->blocks[li]) {
      f(b.c1);
      f(b.c2);
      f(b.c3);
      if (b.has_down) f(b.down);
    }
  for (auto& c : pt->ppm) f(c);
  f(pt->bott);
}

// host -> device packed layouts
static void pt_pack(const PtParam& p, const float* src, std::vector<float>& dst) {
  dst.assign((size_t)p.numel, 0.f);
  if (p.kind == PT_PLAIN) {
    std::memcpy(dst.data(), src, (size_t)p.numel * 4);
    return;
  }
  const int taps = p.k * p.k;
  const long K = (long)taps * p.Ci;
  for (int co = 0; co < p.Co; ++co)
    for (int ci = 0; ci < p.Ci; ++ci)
      for (int tap = 0; tap < taps; ++tap) {
        const float v = src[((long)co * p.Ci + ci) * taps + tap];
        if (p.kind == PT_STEM1)
          dst[(size_t)(ci * 9 + tap) * p.Co + co] = v;
        else
          dst[(size_t)co * K + packed_k(ci, tap, taps)] = v;
      }
}

static void pt_unpack(const PtParam& p, const float* src, float* dst) {
  if (p.kind == PT_PLAIN) {
    std::memcpy(dst, src, (size_t)p.numel * 4);
    return;
  }
  const int taps = p.k * p.k;
  const long K = (long)taps * p.Ci;
  for (int co = 0; co < p.Co; ++co)
    for (int ci = 0; ci < p.Ci; ++ci)
      for (int tap = 0; tap < taps; ++tap)
        dst[((long)co * p.Ci + ci) * taps + tap] =
            p.kind == PT_STEM1 ? src[(size_t)(ci * 9 + tap) * p.Co + co] : src[(size_t)co * K + packed_k(ci, tap, taps)];
}

// ---------------------------------------------------------------- layer helpers
static const float* const kReluFromY = reinterpret_cast<const float*>(1);  // bn_bwd: mask from y

struct PtStep {
  cwt_pretrain* pt;
  hipStream_t st;
  float *part = nullptr, *slab = nullptr, *sums = nullptr;
  size_t part_floats = 0, slab_floats = 0, split_floats = 0;
  float* split = nullptr;  // conv split-K partials

  int conv_fwd(const PtConv& L, const float* x, int N, int Hi, int x_ld, float* y, int y_ld, int stage,
               const float* w = nullptr, int Ci = -1, int Co = -1, int stride = -1, int pad = -1,
               const float* res = nullptr, int res_ld = 0) {
    ConvArgs a;
    std::memset(&a, 0, sizeof(a));
    a.x = x;
    a.w = w ? w : pt->P + L.w_off;
    a.scale = pt->ones;
    a.shift = pt->zeros;
    a.res = res;
    a.res_ld = res_ld;
    a.y = y;
    a.N = N;
    a.Hi = a.Wi = Hi;
    a.Ci = Ci >= 0 ? Ci : L.Ci;
    a.Co = Co >= 0 ? Co : L.Co;
    a.x_ld = x_ld;
    a.kh = a.kw = L.k;
    a.stride = stride >= 0 ? stride : L.stride;
    a.pad = pad >= 0 ? pad : L.pad;
    a.dil = L.dil;
    a.Ho = a.Wo = (Hi + 2 * a.pad - a.dil * (L.k - 1) - 1) / a.stride + 1;
    a.M = N * a.Ho * a.Wo;
    a.K = L.k * L.k * a.Ci;
    a.y_ld = y_ld;
    a.relu = 0;
    const ConvPlan pl = plan_conv(a.M, a.Co, a.K);
    if (pl.nsplit > 1 && (size_t)pl.nsplit * a.M * a.Co > split_floats) {
      int rc = pt_ws(pt, "split", (size_t)pl.nsplit * a.M * a.Co * 4, &split);
      if (rc) return rc;
      split_floats = (size_t)pl.nsplit * a.M * a.Co;
    }
    return launch_conv(a, pl, stage, split, split_floats, st);
  }

  int bn_fwd(PtConv& L, const float* y, int ld, long M, int train, float momentum) {
    return launch_ptbn_fwd(y, ld, M, L.bn.C, L.bn.run, pt->eps, momentum, train, L.bn.stats, part, part_floats, st);
  }

  int bn_apply(const PtConv& L, long M, float* out, int out_ld, int relu, const PtConv* resL = nullptr,
               const float* res = nullptr, int res_ld = 0, long rows_per_image = 1, float drop = 0.f,
               float* out_pre = nullptr) {
    PtBnApply a;
    std::memset(&a, 0, sizeof(a));
    a.y = L.y;
    a.y_ld = L.Co;
    a.M = M;
    a.C = L.Co;
    a.gamma = pt->P + L.bn.g_off;
    a.beta = pt->P + L.bn.b_off;
    a.stats = L.bn.stats;
    if (resL) {
      a.res = resL->y;
      a.res_ld = resL->Co;
      a.res_gamma = pt->P + resL->bn.g_off;
      a.res_beta = pt->P + resL->bn.b_off;
      a.res_stats = resL->bn.stats;
    } else if (res) {
      a.res = res;
      a.res_ld = res_ld;
    }
    a.relu = relu;
    a.drop_p = drop;
    a.seed = pt->seed;
    a.rows_per_image = rows_per_image;
    a.out = out;
    a.out_pre = out_pre;
    a.out_ld = out_ld;
    return launch_ptbn_apply(a, st);
  }

  // gradient at a BN's raw conv output; dgamma / dbeta into G
  // act == RELU_FROM_Y: the BN has no residual, its ReLU mask is recomputed from y (no act read)
  int bn_bwd(const PtConv& L, long M, const float* dout, int dout_ld, const float* act, int act_ld, float* dy,
             float* g_out = nullptr, int g_ld = 0, long rows_per_image = 1, float drop = 0.f) {
    PtBnBwd b;
    std::memset(&b, 0, sizeof(b));
    b.dout = dout;
    b.dout_ld = dout_ld;
    b.relu_from_y = act == kReluFromY;
    b.act = b.relu_from_y ? nullptr : act;
    b.act_ld = act_ld;
    b.beta = pt->P + L.bn.b_off;
    b.drop_p = drop;
    b.seed = pt->seed;
    b.rows_per_image = rows_per_image;
    b.y = L.y;
    b.y_ld = L.Co;
    b.gamma = pt->P + L.bn.g_off;
    b.stats = L.bn.stats;
    b.M = M;
    b.C = L.Co;
    b.dy = dy;
    b.dy_ld = L.Co;
    b.g_out = g_out;
    b.g_ld = g_ld;
    return launch_ptbn_bwd(b, pt->G + L.bn.g_off, pt->G + L.bn.b_off, part, part_floats, sums, st);
  }

  // Ci >= 0: only the first Ci input channels (a K prefix of the packed order), into out [Co][k k Ci]
  int wgrad(const PtConv& L, const float* dy, const float* x, int x_ld, int N, int Hi, int Ci = -1,
            float* out = nullptr) {
    WgradArgs w;
    std::memset(&w, 0, sizeof(w));
    w.dy = dy;
    w.dy_ld = L.Co;
    w.x = x;
    w.x_ld = x_ld;
    w.N = N;
    w.Hi = w.Wi = Hi;
    w.Ho = w.Wo = (Hi + 2 * L.pad - L.dil * (L.k - 1) - 1) / L.stride + 1;
    w.M = (long)N * w.Ho * w.Wo;
    w.Co = L.Co;
    w.K = L.k * L.k * (Ci >= 0 ? Ci : L.Ci);
    w.kh = w.kw = L.k;
    w.stride = L.stride;
    w.pad = L.pad;
    w.dil = L.dil;
    return launch_conv_wgrad(w, out ? out : pt->G + L.w_off, slab, slab_floats, st);
  }

  // dx (row stride dx_ld) = input gradient of conv L from dy [N][Ho][Ho][Co] (+ res); Ci >= 0:
  // only the first Ci input channels
  int dgrad(PtConv& L, const float* dy, int N, int Hi, float* dx, int dx_ld, const float* res, int res_ld, int stage,
            int Ci = -1) {
    int rc;
    const int taps = L.k * L.k;
    if ((rc = launch_wt_transpose(pt->P + L.w_off, L.wt, L.Co, L.Ci, taps, st))) return rc;
    const int Ho = (Hi + 2 * L.pad - L.dil * (L.k - 1) - 1) / L.stride + 1;
    const float* src = dy;
    if (L.stride == 2) {
      float* z;
      if ((rc = pt_ws(pt, "zins", (size_t)N * Hi * Hi * L.Co * 4, &z))) return rc;
      if ((rc = launch_zero_insert(dy, N, Ho, Ho, L.Co, z, Hi, Hi, st))) return rc;
      src = z;
    }
    return conv_fwd(L, src, N, Hi, L.Co, dx, dx_ld, stage, L.wt, L.Co, Ci >= 0 ? Ci : L.Ci, 1,
                    L.dil * (L.k - 1) - L.pad, res, res_ld);
  }

  int gemm(const float* A, long sai, long sak, const float* Bm, long sbk, long sbj, float* C, long ldc, int M, int N,
           long K) {
    PtGemm g;
    std::memset(&g, 0, sizeof(g));
    g.A = A;
    g.sai = sai;
    g.sak = sak;
    g.B = Bm;
    g.sbk = sbk;
    g.sbj = sbj;
    g.C = C;
    g.ldc = ldc;
    g.M = M;
    g.N = N;
    g.K = K;
    return launch_pt_gemm(g, slab, slab_floats, st);
  }
};

static int pt_ensure_acts(cwt_pretrain* pt, int N, int S) {
  if (pt->N == N && pt->S == S && pt->CAT) return 0;
  const int Hs = pt_down2(S), H1 = pt_down2(Hs), h = pt_down2(H1);
  pt->Hs = Hs;
  pt->H1 = H1;
  pt->h = h;
  int rc;
  auto act = [&](PtConv& L, const std::string& nm, long M, bool need_a) -> int {
    int r;
    if ((r = pt_ws(pt, nm + ".y", (size_t)M * L.Co * 4, &L.y))) return r;
    if (need_a) {
      if ((r = pt_ws(pt, nm + ".a", (size_t)M * L.Co * 4, &L.a))) return r;
      L.a_ld = L.Co;
    }
    return 0;
  };
  const long Ms = (long)N * Hs * Hs, M1 = (long)N * H1 * H1, Mh = (long)N * h * h;
  for (int i = 0; i < 3; ++i)
    if ((rc = act(pt->stem[i], "stem" + std::to_string(i), Ms, true))) return rc;
  if ((rc = pt_ws(pt, "mp", (size_t)M1 * 128 * 4, &pt->MP))) return rc;
  float* idx;
  if ((rc = pt_ws(pt, "mpidx", (size_t)M1 * 128, &idx))) return rc;
  pt->MPIDX = (uint8_t*)idx;
  if ((rc = pt_ws(pt, "cat", (size_t)Mh * 2048 * 4, &pt->CAT))) return rc;
  int H = H1;
  for (int li = 0; li < 4; ++li)
    for (int bi = 0; bi < (int)pt->blocks[li].size(); ++bi) {
      PtBlock& b = pt->blocks[li][bi];
      const std::string p = "l" + std::to_string(li) + "." + std::to_string(bi);
      const int Ho = b.c2.stride == 2 ? pt_down2(H) : H;
      b.c1.Hi = H;
      b.c1.Ho = H;
      b.c2.Hi = H;
      b.c2.Ho = Ho;
      b.c3.Hi = b.c3.Ho = Ho;
      b.down.Hi = H;
      b.down.Ho = Ho;
      const long Mi = (long)N * H * H, Mo = (long)N * Ho * Ho;
      if ((rc = act(b.c1, p + ".c1", Mi, true)) || (rc = act(b.c2, p + ".c2", Mo, true))) return rc;
      const bool last = li == 3 && bi == (int)pt->blocks[3].size() - 1;
      if (last) {
        if ((rc = act(b.c3, p + ".c3", Mo, false))) return rc;
        b.c3.a = pt->CAT;  // layer4's output: the PPM's and the bottleneck conv's input
        b.c3.a_ld = 2048;
      } else if ((rc = act(b.c3, p + ".c3", Mo, true))) {
        return rc;
      }
      if (b.has_down && (rc = act(b.down, p + ".down", Mo, false))) return rc;
      H = Ho;
    }
  int ncells = 0;
  for (int b : kPtBins) ncells += b * b;
  if ((rc = pt_ws(pt, "pool", (size_t)N * ncells * 2048 * 4, &pt->POOL))) return rc;
  for (int i = 0; i < 4; ++i)
    if ((rc = act(pt->ppm[i], "ppm" + std::to_string(i), (long)N * kPtBins[i] * kPtBins[i], true))) return rc;
  if ((rc = act(pt->bott, "bott", Mh, false))) return rc;
  if ((rc = pt_ws(pt, "fpre", (size_t)Mh * 512 * 4, &pt->Fpre)) || (rc = pt_ws(pt, "f", (size_t)Mh * 512 * 4, &pt->F)) ||
      (rc = pt_ws(pt, "logits", (size_t)Mh * pt->nc * 4, &pt->LOGITS)))
    return rc;
  pt->N = N;
  pt->S = S;
  return 0;
}

static int pt_workspaces(cwt_pretrain* pt, PtStep& s) {
  const int N = pt->N;
  const long Ms = (long)N * pt->Hs * pt->Hs;
  int rc;
  const long M1 = (long)N * pt->H1 * pt->H1, Mh = (long)N * pt->h * pt->h;
  s.part_floats = std::max({ptbn_part_floats(Ms, 128), ptbn_part_floats(M1, 256), ptbn_part_floats(Mh, 2048)});
  if ((rc = pt_ws(pt, "bnpart", s.part_floats * 4, &s.part))) return rc;
  if ((rc = pt_ws(pt, "bnsums", 2 * 4096 * 4, &s.sums))) return rc;
  // weight-gradient slabs: up to 32 M floats (128 MB)
  s.slab_floats = (size_t)32 << 20;
  if ((rc = pt_ws(pt, "slab", s.slab_floats * 4, &s.slab))) return rc;
  auto sp = pt->ws.find("split");
  if (sp != pt->ws.end()) {
    s.split = (float*)sp->second.first;
    s.split_floats = sp->second.second / 4;
  }
  return 0;
}

// The forward of pretrain.py:208 (model(images)) in train (batch statistics, running statistics
// moved, Dropout2d) or eval mode (running statistics).  Leaves every activation the backward needs.
static int pt_forward(cwt_pretrain* pt, PtStep& s, const float* img, int train, float bn_mom) {
  const int N = pt->N, S = pt->S, Hs = pt->Hs, H1 = pt->H1, h = pt->h;
  const long Ms = (long)N * Hs * Hs, M1 = (long)N * H1 * H1, Mh = (long)N * h * h;
  hipStream_t st = s.st;
  int rc;
  PtConv* sm = pt->stem;
  // layer0 (resnet.py:110-118)
  if ((rc = launch_stem_conv1(img, N, S, pt->P + sm[0].w_off, pt->ones, pt->zeros, sm[0].y, Hs, st, ACT_F32, 0)))
    return rc;
  if ((rc = s.bn_fwd(sm[0], sm[0].y, 64, Ms, train, bn_mom)) || (rc = s.bn_apply(sm[0], Ms, sm[0].a, 64, 1)))
    return rc;
  for (int i = 1; i < 3; ++i) {
    if ((rc = s.conv_fwd(sm[i], sm[i - 1].a, N, Hs, sm[i].Ci, sm[i].y, sm[i].Co, 0)) ||
        (rc = s.bn_fwd(sm[i], sm[i].y, sm[i].Co, Ms, train, bn_mom)) ||
        (rc = s.bn_apply(sm[i], Ms, sm[i].a, sm[i].Co, 1)))
      return rc;
  }
  if ((rc = launch_maxpool_idx(sm[2].a, N, Hs, 128, pt->MP, pt->MPIDX, H1, st))) return rc;
  const float* x = pt->MP;
  int x_ld = 128, H = H1;
  for (int li = 0; li < 4; ++li)
    for (auto& b : pt->blocks[li]) {
      b.x = x;
      b.x_ld = x_ld;
      const long Mi = (long)N * H * H, Mo = (long)N * b.c2.Ho * b.c2.Ho;
      if ((rc = s.conv_fwd(b.c1, x, N, H, x_ld, b.c1.y, b.c1.Co, li + 1)) ||
          (rc = s.bn_fwd(b.c1, b.c1.y, b.c1.Co, Mi, train, bn_mom)) || (rc = s.bn_apply(b.c1, Mi, b.c1.a, b.c1.Co, 1)) ||
          (rc = s.conv_fwd(b.c2, b.c1.a, N, H, b.c1.Co, b.c2.y, b.c2.Co, li + 1)) ||
          (rc = s.bn_fwd(b.c2, b.c2.y, b.c2.Co, Mo, train, bn_mom)) || (rc = s.bn_apply(b.c2, Mo, b.c2.a, b.c2.Co, 1)) ||
          (rc = s.conv_fwd(b.c3, b.c2.a, N, b.c2.Ho, b.c2.Co, b.c3.y, b.c3.Co, li + 1)) ||
          (rc = s.bn_fwd(b.c3, b.c3.y, b.c3.Co, Mo, train, bn_mom)))
        return rc;
      if (b.has_down) {
        if ((rc = s.conv_fwd(b.down, x, N, H, x_ld, b.down.y, b.down.Co, li + 1)) ||
            (rc = s.bn_fwd(b.down, b.down.y, b.down.Co, Mo, train, bn_mom)) ||
            (rc = s.bn_apply(b.c3, Mo, b.c3.a, b.c3.a_ld, 1, &b.down)))
          return rc;
      } else if ((rc = s.bn_apply(b.c3, Mo, b.c3.a, b.c3.a_ld, 1, nullptr, x, x_ld))) {
        return rc;
      }
      x = b.c3.a;
      x_ld = b.c3.a_ld;
      H = b.c2.Ho;
    }
  // PPM (pspnet.py:19-38): adaptive pools of layer4 (CAT, 2048 channels).
  // The branch outputs P_b stay on their b x b grids and enter the bottleneck conv folded
  // (backbone.hip, "PPM branch of the bottleneck conv, folded"): Q_b = P_b . W_b[tap] over the
  // bottleneck weights' PPM columns (GEMM form Wq), the field F = sum over taps and cells of the
  // interpolation weights times Q is the residual of the conv over the 2048 layer4 channels.
  PtConv& Bt = pt->bott;
  int ncells = 0;
  for (int b : kPtBins) ncells += b * b;
  float *col, *Wq, *Q, *R, *Fld, *Wl;
  if ((rc = pt_ws(pt, "ppmcol", ((size_t)N * h * 16 * 2048 + (size_t)N * 16 * 16 * 2048) * 4, &col)) ||
      (rc = pt_ws(pt, "wq", (size_t)4 * 512 * 4608 * 4, &Wq)) ||
      (rc = pt_ws(pt, "q", (size_t)N * ncells * 4608 * 4, &Q)) ||
      (rc = pt_ws(pt, "r", (size_t)N * 12 * h * 3 * 512 * 4, &R)) || (rc = pt_ws(pt, "field", (size_t)Mh * 512 * 4, &Fld)) ||
      (rc = pt_ws(pt, "wl", (size_t)512 * 2048 * 9 * 4, &Wl)) ||
      (rc = launch_ppm(pt->CAT, N, h, h, 2048, kPtBins, 4, col, pt->POOL, st, ACT_F32)) ||
      (rc = launch_ppm_wq(pt->P + Bt.w_off, 4096 * 9, Wq, 0, st)))
    return rc;
  long base = 0;
  for (int i = 0; i < 4; ++i) {
    const int b = kPtBins[i];
    const long Mb = (long)N * b * b;
    PtConv& L = pt->ppm[i];
    const float* pool = pt->POOL + base * N * 2048;
    if ((rc = s.gemm(pool, 2048, 1, pt->P + L.w_off, 1, 2048, L.y, 512, (int)Mb, 512, 2048)) ||
        (rc = s.bn_fwd(L, L.y, 512, Mb, train, bn_mom)) || (rc = s.bn_apply(L, Mb, L.a, 512, 1)) ||
        (rc = s.gemm(L.a, 512, 1, Wq + (size_t)i * 512 * 4608, 4608, 1, Q + base * N * 4608, 4608, (int)Mb, 4608, 512)))
      return rc;
    base += b * b;
  }
  // bottleneck conv3x3 4096 -> 512 + BN + ReLU + Dropout2d (pspnet.py:124-129): the layer4
  // columns of the packed weights are a K prefix (packed_k's 32-channel blocks), copied dense
  if ((rc = launch_ppm_field(Q, N, h, h, kPtBins, R, Fld, st))) return rc;
  CWT_HIP(hipMemcpy2DAsync(Wl, (size_t)2048 * 9 * 4, pt->P + Bt.w_off, (size_t)4096 * 9 * 4, (size_t)2048 * 9 * 4, 512,
                           hipMemcpyDeviceToDevice, st));
  if ((rc = s.conv_fwd(Bt, pt->CAT, N, h, 2048, Bt.y, 512, 6, Wl, 2048, 512, -1, -1, Fld, 512)) ||
      (rc = s.bn_fwd(Bt, Bt.y, 512, Mh, train, bn_mom)) ||
      (rc = s.bn_apply(Bt, Mh, pt->F, 512, 1, nullptr, nullptr, 0, (long)h * h, train ? pt->drop_p : 0.f, pt->Fpre)))
    return rc;
  // classifier conv1x1 512 -> nc (pspnet.py:131-132), logits [M][nc]
  return s.gemm(pt->F, 512, 1, pt->P + pt->cls_off, 1, 512, pt->LOGITS, pt->nc, (int)Mh, pt->nc, 512);
}

static int pt_backward(cwt_pretrain* pt, PtStep& s, const float* dlogits) {
  const int N = pt->N, Hs = pt->Hs, H1 = pt->H1, h = pt->h;
  const long Ms = (long)N * Hs * Hs, Mh = (long)N * h * h;
  const float drop = pt->drop_p;
  int rc;
  // test hook: keep a dense copy of a transient gradient (rows x cols, row stride ld)
  auto capture = [&](const std::string& nm, const float* src, long rows, int cols, int ld) -> int {
    if (!pt->capture) return 0;
    float* dst;
    int r;
    if ((r = pt_ws(pt, "cap." + nm, (size_t)rows * cols * 4, &dst))) return r;
    CWT_HIP(hipMemcpy2DAsync(dst, (size_t)cols * 4, src, (size_t)ld * 4, (size_t)cols * 4, rows, hipMemcpyDeviceToDevice,
                             s.st));
    pt->cap[nm] = {dst, rows * cols};
    return 0;
  };
  if ((rc = capture("dlogits", dlogits, Mh, pt->nc, pt->nc))) return rc;
  // scratch gradients: the widest activation is the layer4 map (Mh x 2048) or layer1 / stem
  size_t mx = (size_t)Mh * 2048;
  mx = std::max(mx, (size_t)Ms * 128);
  mx = std::max(mx, (size_t)N * H1 * H1 * 256);
  float *gA, *gB, *gY, *gT, *gR, *dcat;
  if ((rc = pt_ws(pt, "gA", mx * 4, &gA)) || (rc = pt_ws(pt, "gB", mx * 4, &gB)) || (rc = pt_ws(pt, "gY", mx * 4, &gY)) ||
      (rc = pt_ws(pt, "gT", mx * 4, &gT)) || (rc = pt_ws(pt, "gR", mx * 4, &gR)) ||
      (rc = pt_ws(pt, "dcat", (size_t)Mh * 2048 * 4, &dcat)))
    return rc;
  // classifier: dF = dlogits . Wc, dWc = dlogits^T . F
  if ((rc = s.gemm(dlogits, pt->nc, 1, pt->P + pt->cls_off, 512, 1, gA, 512, (int)Mh, 512, pt->nc)) ||
      (rc = s.gemm(dlogits, 1, pt->nc, pt->F, 512, 1, pt->G + pt->cls_off, 512, pt->nc, 512, Mh)))
    return rc;
  // bottleneck: Dropout2d + ReLU + BN backward; the layer4 columns' weight gradient (dense, copied
  // into the packed rows) and input gradient; the PPM columns through the field's adjoint
  PtConv& Bt = pt->bott;
  int ncells = 0;
  for (int b : kPtBins) ncells += b * b;
  float *gWl, *gWq, *dQ, *R, *Wq;  // Wq: the forward's GEMM-form weights
  if ((rc = pt_ws(pt, "wq", (size_t)4 * 512 * 4608 * 4, &Wq)) || (rc = pt_ws(pt, "gwl", (size_t)512 * 2048 * 9 * 4, &gWl)) || (rc = pt_ws(pt, "gwq", (size_t)4 * 512 * 4608 * 4, &gWq)) ||
      (rc = pt_ws(pt, "dq", (size_t)N * ncells * 4608 * 4, &dQ)) || (rc = pt_ws(pt, "r", (size_t)N * 12 * h * 3 * 512 * 4, &R)))
    return rc;
  if ((rc = s.bn_bwd(Bt, Mh, gA, 512, kReluFromY, 512, gY, nullptr, 0, (long)h * h, drop)) ||
      (rc = s.wgrad(Bt, gY, pt->CAT, 2048, N, h, 2048, gWl)) ||
      (rc = s.dgrad(Bt, gY, N, h, dcat, 2048, nullptr, 0, 6, 2048)) ||
      (rc = launch_ppm_field_bwd(gY, N, h, h, kPtBins, R, dQ, s.st)))
    return rc;
  CWT_HIP(hipMemcpy2DAsync(pt->G + Bt.w_off, (size_t)4096 * 9 * 4, gWl, (size_t)2048 * 9 * 4, (size_t)2048 * 9 * 4, 512,
                           hipMemcpyDeviceToDevice, s.st));
  // PPM branch: dP_b = dQ_b . W_b^T and dW_b = P_b^T . dQ_b, then ReLU + BN backward -> 1x1 conv
  // gradients -> pool adjoint
  float* dpool;
  if ((rc = pt_ws(pt, "dpool", (size_t)N * ncells * 2048 * 4, &dpool))) return rc;
  long base = 0;
  for (int i = 0; i < 4; ++i) {
    const int b = kPtBins[i];
    const long Mb = (long)N * b * b;
    PtConv& L = pt->ppm[i];
    const float* pool = pt->POOL + base * N * 2048;
    const float* dQb = dQ + base * N * 4608;
    if ((rc = s.gemm(dQb, 4608, 1, Wq + (size_t)i * 512 * 4608, 1, 4608, gT, 512, (int)Mb, 512, 4608)) ||
        (rc = s.gemm(L.a, 1, 512, dQb, 4608, 1, gWq + (size_t)i * 512 * 4608, 4608, 512, 4608, Mb)) ||
        (rc = s.bn_bwd(L, Mb, gT, 512, kReluFromY, 512, gY)) ||
        (rc = s.gemm(gY, 1, 512, pool, 2048, 1, pt->G + L.w_off, 2048, 512, 2048, Mb)) ||
        (rc = s.gemm(gY, 512, 1, pt->P + L.w_off, 2048, 1, dpool + base * N * 2048, 2048, (int)Mb, 2048, 512)))
      return rc;
    base += b * b;
  }
  if ((rc = launch_ppm_wq(pt->G + Bt.w_off, 4096 * 9, gWq, 1, s.st)) ||
      (rc = launch_avgpool_bwd(dpool, N, h, 2048, kPtBins, dcat, 2048, s.st)) ||
      (rc = capture("dcat", dcat, Mh, 2048, 2048)))
    return rc;
  // ResNet blocks in reverse (resnet.py:74-96)
  const float* dout = dcat;
  int dout_ld = 2048;
  float* bufs[2] = {gA, gB};
  int nb = 0;
  for (int li = 3; li >= 0; --li)
    for (int bi = (int)pt->blocks[li].size() - 1; bi >= 0; --bi) {
      PtBlock& b = pt->blocks[li][bi];
      const int H = b.c1.Hi, Ho = b.c2.Ho;
      const long Mi = (long)N * H * H, Mo = (long)N * Ho * Ho;
      float* dx = bufs[nb];
      nb ^= 1;
      // conv3: g = dout * relu'(out); the identity residual's gradient is g itself
      if ((rc = s.bn_bwd(b.c3, Mo, dout, dout_ld, b.c3.a, b.c3.a_ld, gY, b.has_down ? nullptr : gR, b.c3.Co)) ||
          (rc = s.wgrad(b.c3, gY, b.c2.a, b.c2.Co, N, Ho)) ||
          (rc = s.dgrad(b.c3, gY, N, Ho, gT, b.c2.Co, nullptr, 0, li + 1)))
        return rc;
      if (b.has_down) {  // downsample branch: its BN sees the same g
        float* gD;
        if ((rc = pt_ws(pt, "gD", (size_t)Mo * b.down.Co * 4, &gD)) ||
            (rc = s.bn_bwd(b.down, Mo, dout, dout_ld, b.c3.a, b.c3.a_ld, gD)) ||
            (rc = s.wgrad(b.down, gD, b.x, b.x_ld, N, H)) ||
            (rc = s.dgrad(b.down, gD, N, H, gR, b.down.Ci, nullptr, 0, li + 1)))
          return rc;
      }
      // conv2 (stride / dilation), conv1; the input gradient of conv1 adds the residual branch's
      if ((rc = s.bn_bwd(b.c2, Mo, gT, b.c2.Co, kReluFromY, b.c2.Co, gY)) || (rc = s.wgrad(b.c2, gY, b.c1.a, b.c1.Co, N, H)) ||
          (rc = s.dgrad(b.c2, gY, N, H, gT, b.c1.Co, nullptr, 0, li + 1)) ||
          (rc = s.bn_bwd(b.c1, Mi, gT, b.c1.Co, kReluFromY, b.c1.Co, gY)) || (rc = s.wgrad(b.c1, gY, b.x, b.x_ld, N, H)) ||
          (rc = s.dgrad(b.c1, gY, N, H, dx, b.c1.Ci, gR, b.c1.Ci, li + 1)) ||
          (rc = capture("dx:l" + std::to_string(li + 1) + "." + std::to_string(bi), dx, Mi, b.c1.Ci, b.c1.Ci)))
        return rc;
      dout = dx;
      dout_ld = b.c1.Ci;
    }
  // layer0: max-pool adjoint, then the three conv + BN + ReLU in reverse
  PtConv* sm = pt->stem;
  float* dmp = bufs[nb];
  if ((rc = launch_maxpool_bwd(dout, pt->MPIDX, N, Hs, 128, H1, dmp, s.st))) return rc;
  const float* d = dmp;
  for (int i = 2; i >= 1; --i) {
    float* nx = (d == gA) ? gB : gA;
    if ((rc = s.bn_bwd(sm[i], Ms, d, sm[i].Co, kReluFromY, sm[i].Co, gY)) ||
        (rc = s.wgrad(sm[i], gY, sm[i - 1].a, sm[i].Ci, N, Hs)) ||
        (rc = s.dgrad(sm[i], gY, N, Hs, nx, sm[i].Ci, nullptr, 0, 0)))
      return rc;
    d = nx;
  }
  if ((rc = s.bn_bwd(sm[0], Ms, d, 64, kReluFromY, 64, gY))) return rc;
  return launch_stem1_wgrad(pt->img, N, pt->S, gY, Hs, pt->G + sm[0].w_off, s.slab, s.slab_floats, s.st);
}

}  // namespace cwt

using namespace cwt;

extern "C" {

int cwt_pretrain_create(cwt_ctx* ctx, int layers, int num_classes, int n_tensors, const char* const* names,
                        const float* const* host_data, const int64_t* numel, float bn_eps, cwt_pretrain** out) {
  if (!ctx || !names || !host_data || !numel || !out || n_tensors <= 0) return fail(CWT_EARG, "null argument");
  if (layers != 50 && layers != 101) return fail(CWT_EARG, "layers must be 50 or 101");
  if (num_classes != 2 && num_classes != 16 && num_classes != 61)
    return fail(CWT_EARG, "num_classes_tr must be 2, 16 (PASCAL) or 61 (COCO)");
  CWT_HIP(hipSetDevice(ctx_device(ctx)));
  cwt_pretrain* pt = new cwt_pretrain();
  pt->device = ctx_device(ctx);
  pt->layers = layers;
  pt->nc = num_classes;
  pt->eps = bn_eps;
  auto bail = [&](int rc) {
    for (void* p : pt->allocs) (void)hipFree(p);
    for (auto& w : pt->ws)
      if (w.second.first) (void)hipFree(w.second.first);
    delete pt;
    return rc;
  };
  pt_build(pt);
  std::map<std::string, std::pair<const float*, int64_t>> hp;
  for (int i = 0; i < n_tensors; ++i) hp[names[i]] = {host_data[i], numel[i]};
  void* p;
  int rc;
  if ((rc = pt_alloc(pt, (size_t)pt->n_all * 4, &p))) return bail(rc);
  pt->P = (float*)p;
  if ((rc = pt_alloc(pt, (size_t)pt->n_all * 4, &p))) return bail(rc);
  pt->G = (float*)p;
  if ((rc = pt_alloc(pt, (size_t)pt->n_all * 4, &p))) return bail(rc);
  pt->MOM = (float*)p;
  CWT_HIP(hipMemset(pt->P, 0, (size_t)pt->n_all * 4));
  CWT_HIP(hipMemset(pt->G, 0, (size_t)pt->n_all * 4));
  CWT_HIP(hipMemset(pt->MOM, 0, (size_t)pt->n_all * 4));
  std::vector<float> buf;
  for (const auto& prm : pt->params) {
    auto it = hp.find(prm.name);
    if (it == hp.end() || !it->second.first) return bail(fail(CWT_EARG, "missing tensor '" + prm.name + "'"));
    if (it->second.second != prm.numel)
      return bail(fail(CWT_EARG, "tensor '" + prm.name + "' has " + std::to_string(it->second.second) +
                                     " elements, expected " + std::to_string(prm.numel)));
    pt_pack(prm, it->second.first, buf);
    CWT_HIP(hipMemcpy(pt->P + prm.off, buf.data(), (size_t)prm.numel * 4, hipMemcpyHostToDevice));
  }
  // running statistics, per-forward statistics, input-gradient weights
  int err = 0;
  pt_for_each_conv(pt, [&](PtConv& L) {
    if (err) return;
    PtBn& b = L.bn;
    auto rm = hp.find(b.prefix + ".running_mean"), rv = hp.find(b.prefix + ".running_var");
    if (rm == hp.end() || rv == hp.end() || rm->second.second != b.C || rv->second.second != b.C) {
      err = fail(CWT_EARG, "missing running statistics of '" + b.prefix + "'");
      return;
    }
    void* q;
    if ((err = pt_alloc(pt, (size_t)2 * b.C * 4, &q))) return;
    b.run = (float*)q;
    if ((err = pt_alloc(pt, (size_t)2 * b.C * 4, &q))) return;
    b.stats = (float*)q;
    if (hipMemcpy(b.run, rm->second.first, (size_t)b.C * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(b.run + b.C, rv->second.first, (size_t)b.C * 4, hipMemcpyHostToDevice) != hipSuccess) {
      err = fail(CWT_ESTATE, "hipMemcpy of running statistics failed");
      return;
    }
    pt->bn_by_name[b.prefix] = &b;
    if (L.k > 0 && L.w_off >= 0 && &L != &pt->stem[0]) {
      bool is_ppm = false;
      for (auto& c : pt->ppm) is_ppm |= (&c == &L);
      if (!is_ppm && (err = pt_alloc(pt, (size_t)L.Co * L.Ci * L.k * L.k * 4, &q))) return;
      if (!is_ppm) L.wt = (float*)q;
    }
  });
  if (err) return bail(err);
  std::vector<float> ones(4096, 1.f);
  if ((rc = pt_alloc(pt, 4096 * 4, &p))) return bail(rc);
  pt->ones = (float*)p;
  if ((rc = pt_alloc(pt, 4096 * 4, &p))) return bail(rc);
  pt->zeros = (float*)p;
  CWT_HIP(hipMemcpy(pt->ones, ones.data(), 4096 * 4, hipMemcpyHostToDevice));
  CWT_HIP(hipMemset(pt->zeros, 0, 4096 * 4));
  *out = pt;
  return 0;
}

int cwt_pretrain_destroy(cwt_pretrain* pt) {
  if (!pt) return 0;
  (void)hipSetDevice(pt->device);
  (void)hipDeviceSynchronize();
  for (void* p : pt->allocs) (void)hipFree(p);
  for (auto& w : pt->ws)
    if (w.second.first) (void)hipFree(w.second.first);
  delete pt;
  return 0;
}

int cwt_pretrain_step(cwt_ctx* ctx, cwt_pretrain* pt, const float* images, const int64_t* labels, int N, int S,
                      const cwt_pretrain_hparams* hp, float* loss_out, void* stream) {
  if (!ctx || !pt || !images || !labels || !hp || !loss_out) return fail(CWT_EARG, "null argument");
  CWT_CHECK(N >= 2 && S >= 17 && (S - 1) % 8 == 0, "need N >= 2 (training BN) and (S-1) % 8 == 0 (pspnet.py:150)");
  CWT_HIP(hipSetDevice(pt->device));
  hipStream_t st = (hipStream_t)stream;
  int rc;
  if ((rc = pt_ensure_acts(pt, N, S))) return rc;
  PtStep s{pt, st};
  if ((rc = pt_workspaces(pt, s))) return rc;
  pt->img = images;
  pt->drop_p = hp->drop_p;
  pt->seed = hp->seed;
  if ((rc = pt_forward(pt, s, images, 1, hp->bn_momentum))) return rc;
  // loss and its gradient at the low-res logits
  const int h = pt->h;
  float* dlog;
  float* cews;
  if ((rc = pt_ws(pt, "dlogits", (size_t)N * h * h * pt->nc * 4, &dlog)) ||
      (rc = pt_ws(pt, "cews", seg_ce_ws_bytes(N, S, h, pt->nc), &cews)))
    return rc;
  PtLoss L;
  std::memset(&L, 0, sizeof(L));
  L.logits = pt->LOGITS;
  L.target = labels;
  L.dlogits = dlog;
  L.N = N;
  L.S = S;
  L.h = L.w = h;
  L.nc = pt->nc;
  L.ignore = hp->ignore_index;
  const float e = hp->smoothing ? 0.1f : 0.f;  // pretrain.py:197-199
  L.on = 1.f - e;
  L.off = e / (float)(pt->nc - 1);
  if ((rc = launch_seg_ce_smooth(L, cews, seg_ce_ws_bytes(N, S, h, pt->nc), loss_out, st))) return rc;
  if ((rc = pt_backward(pt, s, dlog))) return rc;
  // optimizer.step(): two SGD groups (pretrain.py:66-72)
  if ((rc = launch_sgd(pt->P, pt->G, pt->MOM, pt->n_bb, hp->lr, hp->momentum, hp->weight_decay, hp->nesterov,
                       pt->first_step ? 1 : 0, st)) ||
      (rc = launch_sgd(pt->P + pt->n_bb, pt->G + pt->n_bb, pt->MOM + pt->n_bb, pt->n_all - pt->n_bb, hp->lr_head,
                       hp->momentum, hp->weight_decay, hp->nesterov, pt->first_step ? 1 : 0, st)))
    return rc;
  pt->first_step = false;
  return 0;
}

int cwt_pretrain_forward(cwt_ctx* ctx, cwt_pretrain* pt, const float* images, int N, int S, int train, float* logits,
                         void* stream) {
  if (!ctx || !pt || !images || !logits) return fail(CWT_EARG, "null argument");
  CWT_CHECK(N >= 1 && S >= 17 && (S - 1) % 8 == 0, "need (S-1) % 8 == 0 (pspnet.py:150)");
  CWT_CHECK(!train || N >= 2, "training-mode BN needs N >= 2");
  CWT_HIP(hipSetDevice(pt->device));
  hipStream_t st = (hipStream_t)stream;
  int rc;
  if ((rc = pt_ensure_acts(pt, N, S))) return rc;
  PtStep s{pt, st};
  if ((rc = pt_workspaces(pt, s))) return rc;
  pt->img = images;
  pt->drop_p = 0.f;
  // train = 1: batch statistics without moving the running statistics (momentum 0)
  if ((rc = pt_forward(pt, s, images, train ? 1 : 0, 0.f))) return rc;
  const long n = (long)N * pt->h * pt->h * pt->nc;
  CWT_HIP(hipMemcpyAsync(logits, pt->LOGITS, (size_t)n * 4, hipMemcpyDeviceToDevice, st));
  return 0;
}

int cwt_pretrain_evaluate(cwt_ctx* ctx, cwt_pretrain* pt, const float* images, const int64_t* labels, int N, int S,
                          int train, float* loss_out, float* iu_out, void* stream) {
  if (!ctx || !pt || !images || !labels || !loss_out || !iu_out) return fail(CWT_EARG, "null argument");
  CWT_CHECK(N >= 1 && S >= 17 && (S - 1) % 8 == 0, "need (S-1) % 8 == 0 (pspnet.py:150)");
  CWT_CHECK(!train || N >= 2, "training-mode BN needs N >= 2");
  CWT_HIP(hipSetDevice(pt->device));
  hipStream_t st = (hipStream_t)stream;
  int rc;
  if ((rc = pt_ensure_acts(pt, N, S))) return rc;
  PtStep s{pt, st};
  if ((rc = pt_workspaces(pt, s))) return rc;
  pt->img = images;
  pt->drop_p = 0.f;
  if ((rc = pt_forward(pt, s, images, train ? 1 : 0, 0.f))) return rc;
  float* ws;
  const size_t wsb = seg_eval_ws_bytes(N, S, pt->h, pt->nc);
  if ((rc = pt_ws(pt, "evalws", wsb, &ws))) return rc;
  PtLoss L;
  std::memset(&L, 0, sizeof(L));
  L.logits = pt->LOGITS;
  L.target = labels;
  L.N = N;
  L.S = S;
  L.h = L.w = pt->h;
  L.nc = pt->nc;
  L.ignore = 255;
  return launch_seg_eval(L, ws, wsb, loss_out, iu_out, st);
}

int cwt_pretrain_get(cwt_pretrain* pt, const char* name, int what, float* host_out, int64_t numel) {
  if (!pt || !name || !host_out) return fail(CWT_EARG, "null argument");
  CWT_HIP(hipSetDevice(pt->device));
  CWT_HIP(hipDeviceSynchronize());
  const std::string nm(name);
  if (what == CWT_PT_RUNNING) {  // "<bn prefix>.running_mean" / ".running_var"
    for (const char* suf : {".running_mean", ".running_var"}) {
      const size_t L = std::strlen(suf);
      if (nm.size() > L && nm.compare(nm.size() - L, L, suf) == 0) {
        auto it = pt->bn_by_name.find(nm.substr(0, nm.size() - L));
        if (it == pt->bn_by_name.end()) break;
        const PtBn& b = *it->second;
        if (numel != b.C) return fail(CWT_EARG, "numel mismatch for '" + nm + "'");
        CWT_HIP(hipMemcpy(host_out, b.run + (suf[9] == 'm' ? 0 : b.C), (size_t)b.C * 4, hipMemcpyDeviceToHost));
        return 0;
      }
    }
    return fail(CWT_EARG, "no running statistic '" + nm + "'");
  }
  auto it = pt->by_name.find(nm);
  if (it == pt->by_name.end()) return fail(CWT_EARG, "no parameter '" + nm + "'");
  const PtParam& p = pt->params[it->second];
  if (numel != p.numel) return fail(CWT_EARG, "numel mismatch for '" + nm + "'");
  const float* src = what == CWT_PT_GRAD ? pt->G : what == CWT_PT_MOMENTUM ? pt->MOM : pt->P;
  std::vector<float> tmp((size_t)p.numel);
  CWT_HIP(hipMemcpy(tmp.data(), src + p.off, (size_t)p.numel * 4, hipMemcpyDeviceToHost));
  pt_unpack(p, tmp.data(), host_out);
  return 0;
}

int cwt_pretrain_set(cwt_pretrain* pt, const char* name, int what, const float* host_in, int64_t numel) {
  if (!pt || !name || !host_in) return fail(CWT_EARG, "null argument");
  CWT_HIP(hipSetDevice(pt->device));
  CWT_HIP(hipDeviceSynchronize());
  const std::string nm(name);
  if (what == CWT_PT_RUNNING) {
    for (const char* suf : {".running_mean", ".running_var"}) {
      const size_t L = std::strlen(suf);
      if (nm.size() > L && nm.compare(nm.size() - L, L, suf) == 0) {
        auto it = pt->bn_by_name.find(nm.substr(0, nm.size() - L));
        if (it == pt->bn_by_name.end()) break;
        const PtBn& b = *it->second;
        if (numel != b.C) return fail(CWT_EARG, "numel mismatch for '" + nm + "'");
        CWT_HIP(hipMemcpy(b.run + (suf[9] == 'm' ? 0 : b.C), host_in, (size_t)b.C * 4, hipMemcpyHostToDevice));
        return 0;
      }
    }
    return fail(CWT_EARG, "no running statistic '" + nm + "'");
  }
  if (what != CWT_PT_PARAM && what != CWT_PT_MOMENTUM) return fail(CWT_EARG, "what: parameter, momentum or running");
  auto it = pt->by_name.find(nm);
  if (it == pt->by_name.end()) return fail(CWT_EARG, "no parameter '" + nm + "'");
  const PtParam& p = pt->params[it->second];
  if (numel != p.numel) return fail(CWT_EARG, "numel mismatch for '" + nm + "'");
  std::vector<float> buf;
  pt_pack(p, host_in, buf);
  CWT_HIP(hipMemcpy((what == CWT_PT_MOMENTUM ? pt->MOM : pt->P) + p.off, buf.data(), (size_t)p.numel * 4,
                    hipMemcpyHostToDevice));
  if (what == CWT_PT_MOMENTUM) pt->first_step = false;  // a resumed optimizer has its momentum buffers
  return 0;
}

int cwt_pretrain_num_params(const cwt_pretrain* pt, int64_t* total, int64_t* backbone) {
  if (!pt) return fail(CWT_EARG, "null argument");
  long t = 0, b = 0;
  for (const auto& p : pt->params) {
    t += p.numel;
    if (p.off < pt->n_bb) b += p.numel;
  }
  if (total) *total = t;
  if (backbone) *backbone = b;
  return 0;
}

}  // extern "C"

// ---------------------------------------------------------------- teacher-forced test hooks
extern "C" {

int cwt_debug_pretrain_capture(cwt_pretrain* pt, int on) {
  if (!pt) return fail(CWT_EARG, "null argument");
  pt->capture = on != 0;
  if (!on) pt->cap.clear();
  return 0;
}

// Forward tensors of the last step / forward ("in:l<layer>.<block>": a ResNet block's input,
// [M][C]; "cat": layer4's output [M][2048]; "mp": the stem's max-pool output [M][128]) and the
// captured backward gradients ("dlogits", "dcat", "dx:l<layer>.<block>": a block's input gradient).
int cwt_debug_pretrain_tensor(cwt_pretrain* pt, const char* name, float* host_out, int64_t numel) {
  if (!pt || !name || !host_out) return fail(CWT_EARG, "null argument");
  CWT_HIP(hipSetDevice(pt->device));
  CWT_HIP(hipDeviceSynchronize());
  const std::string nm(name);
  const float* src = nullptr;
  long rows = 0;
  int cols = 0, ld = 0;
  if (nm == "cat") {
    src = pt->CAT, rows = (long)pt->N * pt->h * pt->h, cols = ld = 2048;
  } else if (nm == "mp") {
    src = pt->MP, rows = (long)pt->N * pt->H1 * pt->H1, cols = ld = 128;
  } else if (nm == "logits") {
    src = pt->LOGITS, rows = (long)pt->N * pt->h * pt->h, cols = ld = pt->nc;
  } else if (nm == "fpre") {  // the bottleneck's BN + ReLU output before Dropout2d
    src = pt->Fpre, rows = (long)pt->N * pt->h * pt->h, cols = ld = 512;
  } else if (nm.rfind("a:stem", 0) == 0) {
    const int i = std::atoi(nm.c_str() + 6);
    if (i < 0 || i > 2) return fail(CWT_EARG, "no activation '" + nm + "'");
    src = pt->stem[i].a, rows = (long)pt->N * pt->Hs * pt->Hs, cols = ld = pt->stem[i].Co;
  } else if (nm.rfind("a:ppm", 0) == 0) {
    const int i = std::atoi(nm.c_str() + 5);
    if (i < 0 || i > 3) return fail(CWT_EARG, "no activation '" + nm + "'");
    src = pt->ppm[i].a, rows = (long)pt->N * kPtBins[i] * kPtBins[i], cols = ld = 512;
  } else if (nm.rfind("a:l", 0) == 0) {  // "a:l<layer>.<block>.c<1|2|3>": BN (+ residual) + ReLU output
    const int li = std::atoi(nm.c_str() + 3) - 1;
    const size_t d1 = nm.find('.'), d2 = nm.rfind(".c");
    const int bi = d1 == std::string::npos ? -1 : std::atoi(nm.c_str() + d1 + 1);
    const int ci = d2 == std::string::npos ? 0 : std::atoi(nm.c_str() + d2 + 2);
    if (li < 0 || li > 3 || bi < 0 || bi >= (int)pt->blocks[li].size() || ci < 1 || ci > 3)
      return fail(CWT_EARG, "no activation '" + nm + "'");
    const PtBlock& b = pt->blocks[li][bi];
    const PtConv& L = ci == 1 ? b.c1 : ci == 2 ? b.c2 : b.c3;
    src = L.a, rows = (long)pt->N * L.Ho * L.Ho, cols = L.Co, ld = L.a_ld;
  } else if (nm.rfind("in:l", 0) == 0) {
    const int li = std::atoi(nm.c_str() + 4) - 1;
    const size_t dot = nm.find('.');
    const int bi = dot == std::string::npos ? -1 : std::atoi(nm.c_str() + dot + 1);
    if (li < 0 || li > 3 || bi < 0 || bi >= (int)pt->blocks[li].size() || !pt->blocks[li][bi].x)
      return fail(CWT_EARG, "no block input '" + nm + "'");
    const PtBlock& b = pt->blocks[li][bi];
    src = b.x, rows = (long)pt->N * b.c1.Hi * b.c1.Hi, cols = b.c1.Ci, ld = b.x_ld;
  } else {
    auto it = pt->cap.find(nm);
    if (it == pt->cap.end()) return fail(CWT_EARG, "nothing captured as '" + nm + "' (cwt_debug_pretrain_capture)");
    if (numel != it->second.second) return fail(CWT_EARG, "numel mismatch for '" + nm + "'");
    CWT_HIP(hipMemcpy(host_out, it->second.first, (size_t)numel * 4, hipMemcpyDeviceToHost));
    return 0;
  }
  if (numel != rows * cols) return fail(CWT_EARG, "numel mismatch for '" + nm + "'");
  CWT_HIP(hipMemcpy2D(host_out, (size_t)cols * 4, src, (size_t)ld * 4, (size_t)cols * 4, rows, hipMemcpyDeviceToHost));
  return 0;
}

}  // extern "C"

// ---------------------------------------------------------------- single-op test hooks
namespace cwt {
// test-hook workspace, one per device (the hook runs on the calling thread's current device;
// calls are serialised like every call on a context)
static float* dbg_ws(int device, size_t bytes) {
  static std::map<int, std::pair<void*, size_t>> ws;
  auto& b = ws[device];
  if (b.second < bytes) {
    if (b.first) {
      (void)hipDeviceSynchronize();
      (void)hipFree(b.first);
    }
    b = {nullptr, 0};
    if (hipMalloc(&b.first, bytes) != hipSuccess) return nullptr;
    b.second = bytes;
  }
  return (float*)b.first;
}
}  // namespace cwt

extern "C" int cwt_debug_pretrain_op(cwt_ctx* ctx, int op, void* const* b, const int64_t* ia, const float* fa,
                                     void* stream) {
  if (!ctx || !b || !ia) return fail(CWT_EARG, "null argument");
  CWT_HIP(hipSetDevice(ctx_device(ctx)));
  hipStream_t st = (hipStream_t)stream;
  const size_t wsf = (size_t)64 << 20;
  float* ws = dbg_ws(ctx_device(ctx), wsf * 4);
  if (!ws) return fail(CWT_ESTATE, "debug workspace allocation failed");
  if (op == 0 || op == 1) {  // 0: weight gradient, 1: input gradient of a conv (ia: N Hi Ci Co k stride pad dil)
    const int N = (int)ia[0], Hi = (int)ia[1], Ci = (int)ia[2], Co = (int)ia[3], k = (int)ia[4], s = (int)ia[5],
              pad = (int)ia[6], dil = (int)ia[7];
    const int Ho = (Hi + 2 * pad - dil * (k - 1) - 1) / s + 1;
    if (op == 0) {
      WgradArgs w;
      std::memset(&w, 0, sizeof(w));
      w.dy = (const float*)b[0];
      w.dy_ld = Co;
      w.x = (const float*)b[1];
      w.x_ld = Ci;
      w.N = N;
      w.Hi = w.Wi = Hi;
      w.Ho = w.Wo = Ho;
      w.M = (long)N * Ho * Ho;
      w.Co = Co;
      w.K = k * k * Ci;
      w.kh = w.kw = k;
      w.stride = s;
      w.pad = pad;
      w.dil = dil;
      return launch_conv_wgrad(w, (float*)b[2], ws, wsf, st);
    }
    // input gradient: transposed weights, zero-interleave (stride 2), stride-1 conv
    float* wt = ws;
    float* z = ws + (size_t)Co * Ci * k * k;
    float* ones = z + (size_t)N * Hi * Hi * Co;
    float* zeros = ones + 4096;
    float* part = zeros + 4096;
    std::vector<float> o(4096, 1.f);
    CWT_HIP(hipMemcpyAsync(ones, o.data(), 4096 * 4, hipMemcpyHostToDevice, st));
    CWT_HIP(hipMemsetAsync(zeros, 0, 4096 * 4, st));
    int rc;
    if ((rc = launch_wt_transpose((const float*)b[1], wt, Co, Ci, k * k, st))) return rc;
    const float* src = (const float*)b[0];
    if (s == 2) {
      if ((rc = launch_zero_insert(src, N, Ho, Ho, Co, z, Hi, Hi, st))) return rc;
      src = z;
    }
    ConvArgs a;
    std::memset(&a, 0, sizeof(a));
    a.x = src;
    a.w = wt;
    a.scale = ones;
    a.shift = zeros;
    a.y = (float*)b[2];
    a.N = N;
    a.Hi = a.Wi = Hi;
    a.Ci = Co;
    a.Co = Ci;
    a.x_ld = Co;
    a.kh = a.kw = k;
    a.stride = 1;
    a.pad = dil * (k - 1) - pad;
    a.dil = dil;
    a.Ho = a.Wo = Hi;
    a.M = N * Hi * Hi;
    a.K = k * k * Co;
    a.y_ld = Ci;
    const ConvPlan pl = plan_conv(a.M, a.Co, a.K);
    const size_t left = wsf - (size_t)(part - ws);
    return launch_conv(a, pl, 0, part, left, st);
  }
  if (op == 5) {  // folded PPM field and its adjoint: b = P dF F dP W dW; ia = N h
    // P [cells][512] bin-major (bins 1 2 3 6, cell = bin start * N + n b b + i b + j), W / dW the
    // packed bottleneck weights [512][4096 * 9] (dW: only the PPM columns written), F / dF [N][h][h][512]
    const int N = (int)ia[0], h = (int)ia[1];
    int ncells = 0;
    for (int bb : kPtBins) ncells += bb * bb;
    float* Wq = ws;
    float* gWq = Wq + (size_t)4 * 512 * 4608;
    float* Q = gWq + (size_t)4 * 512 * 4608;
    float* dQ = Q + (size_t)N * ncells * 4608;
    float* R = dQ + (size_t)N * ncells * 4608;
    float* slab = R + (size_t)N * 12 * h * 1536;
    const size_t used = (size_t)(slab - ws);
    if (used + ((size_t)8 << 20) > wsf) return fail(CWT_EARG, "debug PPM field: too large");
    auto gemm = [&](const float* A, long sai, long sak, const float* Bm, long sbk, long sbj, float* C, long ldc, int M,
                    int Nn, long K) {
      PtGemm g;
      std::memset(&g, 0, sizeof(g));
      g.A = A;
      g.sai = sai;
      g.sak = sak;
      g.B = Bm;
      g.sbk = sbk;
      g.sbj = sbj;
      g.C = C;
      g.ldc = ldc;
      g.M = M;
      g.N = Nn;
      g.K = K;
      return launch_pt_gemm(g, slab, wsf - used, st);
    };
    const float* P = (const float*)b[0];
    float* dP = (float*)b[3];
    int rc;
    if ((rc = launch_ppm_wq((float*)b[4], 4096 * 9, Wq, 0, st))) return rc;
    long base = 0;
    for (int i = 0; i < 4; ++i) {
      const int Mb = N * kPtBins[i] * kPtBins[i];
      if ((rc = gemm(P + base * N * 512, 512, 1, Wq + (size_t)i * 512 * 4608, 4608, 1, Q + base * N * 4608, 4608, Mb,
                     4608, 512)))
        return rc;
      base += kPtBins[i] * kPtBins[i];
    }
    if ((rc = launch_ppm_field(Q, N, h, h, kPtBins, R, (float*)b[2], st)) ||
        (rc = launch_ppm_field_bwd((const float*)b[1], N, h, h, kPtBins, R, dQ, st)))
      return rc;
    base = 0;
    for (int i = 0; i < 4; ++i) {
      const int Mb = N * kPtBins[i] * kPtBins[i];
      const float* dQb = dQ + base * N * 4608;
      if ((rc = gemm(dQb, 4608, 1, Wq + (size_t)i * 512 * 4608, 1, 4608, dP + base * N * 512, 512, Mb, 512, 4608)) ||
          (rc = gemm(P + base * N * 512, 1, 512, dQb, 4608, 1, gWq + (size_t)i * 512 * 4608, 4608, 512, 4608, Mb)))
        return rc;
      base += kPtBins[i] * kPtBins[i];
    }
    return launch_ppm_wq((float*)b[5], 4096 * 9, gWq, 1, st);
  }
  if (op == 2) {  // label-smoothed CE: b = logits, target, dlogits, loss; ia = N S h nc; fa = on off
    PtLoss L;
    std::memset(&L, 0, sizeof(L));
    L.logits = (const float*)b[0];
    L.target = (const int64_t*)b[1];
    L.dlogits = (float*)b[2];
    L.N = (int)ia[0];
    L.S = (int)ia[1];
    L.h = L.w = (int)ia[2];
    L.nc = (int)ia[3];
    L.ignore = 255;
    L.on = fa[0];
    L.off = fa[1];
    return launch_seg_ce_smooth(L, ws, wsf * 4, (float*)b[3], st);
  }
  if (op == 3) {  // BN train fwd + ReLU, then backward: b = y gamma beta out dout dy dgamma dbeta; ia = M C
    const long M = (long)ia[0];
    const int Cc = (int)ia[1];
    float* run = ws;
    float* stats = run + 2 * Cc;
    float* sums = stats + 2 * Cc;
    float* part = sums + 2 * Cc;
    CWT_HIP(hipMemsetAsync(run, 0, (size_t)2 * Cc * 4, st));
    int rc;
    if ((rc = launch_ptbn_fwd((const float*)b[0], Cc, M, Cc, run, fa ? fa[0] : 1e-5f, 0.1f, 1, stats, part,
                              wsf - 6 * Cc, st)))
      return rc;
    PtBnApply ap;
    std::memset(&ap, 0, sizeof(ap));
    ap.y = (const float*)b[0];
    ap.y_ld = Cc;
    ap.M = M;
    ap.C = Cc;
    ap.gamma = (const float*)b[1];
    ap.beta = (const float*)b[2];
    ap.stats = stats;
    ap.relu = 1;
    ap.rows_per_image = 1;
    ap.out = (float*)b[3];
    ap.out_ld = Cc;
    if ((rc = launch_ptbn_apply(ap, st))) return rc;
    PtBnBwd bw;
    std::memset(&bw, 0, sizeof(bw));
    bw.dout = (const float*)b[4];
    bw.dout_ld = Cc;
    bw.act = (const float*)b[3];
    bw.act_ld = Cc;
    bw.rows_per_image = 1;
    bw.y = (const float*)b[0];
    bw.y_ld = Cc;
    bw.gamma = (const float*)b[1];
    bw.stats = stats;
    bw.M = M;
    bw.C = Cc;
    bw.dy = (float*)b[5];
    bw.dy_ld = Cc;
    return launch_ptbn_bwd(bw, (float*)b[6], (float*)b[7], part, wsf - 6 * Cc, sums, st);
  }
  if (op == 4) {  // max pool 3x3 s2 p1 forward + adjoint: b = in out dout din; ia = N H C
    const int N = (int)ia[0], H = (int)ia[1], Cc = (int)ia[2];
    const int Ho = (H - 1) / 2 + 1;
    int rc;
    if ((rc = launch_maxpool_idx((const float*)b[0], N, H, Cc, (float*)b[1], (uint8_t*)ws, Ho, st))) return rc;
    return launch_maxpool_bwd((const float*)b[2], (const uint8_t*)ws, N, H, Cc, Ho, (float*)b[3], st);
  }
  return fail(CWT_EARG, "unknown op");
}

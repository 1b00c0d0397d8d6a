/*
 * cwt.h — C ABI of libcwt.so, the MI355X-native CWT episode engine.
 *
 * The reference (TeamOfProfGuo/Few_Shot_Seg_CWT) has no FFI layer: its "boundary" is
 * the PyTorch nn.Module API the episode drivers call.  Each entry
 * point below replaces one of those call sites; the reference interface is cited above
 * each declaration.  The ctypes shim in few_shot_seg_cwt_amd/_lib.py binds exactly these.
 *
 * Conventions
 *  - Plain C types only; no C++ types or exceptions cross the boundary.
 *  - Every device buffer is CALLER-OWNED (e.g. torch tensors via data_ptr()).  The
 *    library owns only packed weights and an internal workspace pool per context.
 *  - Every call is asynchronous on the given stream (a hipStream_t passed as void*;
 *    NULL = the legacy default stream).  Nothing here synchronises the host.
 *  - Return value: 0 on success, a hipError_t value, or a CWT_E* code below.  The
 *    message of the last failure on the calling thread: cwt_last_error().
 *  - One context per device; calls on one context must be externally serialised.
 *  - Activations are fp32 in HBM.  The convs compute in "bf16x3" by default (fp32 operands
 *    split into bf16 hi + lo, three bf16 MFMA products, fp32 accumulation; ~1e-5 relative
 *    per conv); CWT_CONV=f32 selects exact fp32 MFMA.  Feature maps are NHWC ([N][h][w][C], C contiguous), which
 *    is torch's channels_last memory format of an [N,C,h,w] tensor.
 */
#ifndef CWT_H_
#define CWT_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CWT_OK 0
#define CWT_EARG 1001      /* invalid argument / shape (reference: shape asserts, pspnet.py:74-76,150) */
#define CWT_ESTATE 1002    /* weights not loaded / wrong call order */
#define CWT_ENOFG 1003     /* support mask has no foreground (reference: ZeroDivisionError, test.py:174) */

/* Bits of the context's asynchronous status word (cwt_ctx_status). */
#define CWT_STATUS_ADAPT_BARRIER 1u  /* the persistent inner loop's grid barrier timed out: W is wrong */
#define CWT_STATUS_TAIL_BARRIER 2u   /* cwt_episode_tail's grid barrier timed out: its outputs are wrong */

typedef struct cwt_ctx cwt_ctx;
typedef struct cwt_backbone cwt_backbone;  /* one loaded (frozen) PSPNet extractor */

/* Version string of the library build. */
const char* cwt_version(void);

/* Thread-local message of the last failing call on this thread ("" if none). */
const char* cwt_last_error(void);

/* Create / destroy a context bound to HIP device `device`. */
int cwt_ctx_create(int device, cwt_ctx** out);
int cwt_ctx_destroy(cwt_ctx* ctx);

/*
 * Load the frozen PSPNet feature extractor from a state dict given by name.
 * Replaces: get_model(args) (pspnet.py:15) + PSPNet.__init__ (pspnet.py:70-141) +
 *           model.load_state_dict(...) (test.py:61-81; train.py:57-75).
 * names/host_data/numel: n_tensors entries of the reference's PSPNet.state_dict()
 * (keys as in the reference, e.g. "layer1.0.conv1.weight", "ppm.features.0.2.running_var",
 * "bottleneck.0.weight"); host_data are host fp32 pointers (integer entries such as
 * num_batches_tracked may be passed with host_data == NULL and are ignored).
 * layers: 50 or 101.  BatchNorm (eval mode, eps bn_eps) is folded to per-channel
 * scale/shift and conv weights are repacked [Co][kh][kw][Ci] on the device of ctx.
 * *out receives an independent handle (several backbones may coexist on one context);
 * release it with cwt_backbone_destroy.
 */
int cwt_backbone_load(cwt_ctx* ctx, int layers, int n_tensors, const char* const* names,
                      const float* const* host_data, const int64_t* numel, float bn_eps,
                      cwt_backbone** out);
int cwt_backbone_destroy(cwt_backbone* bb);

/*
 * Arithmetic of the extractor's conv stack (SURVEY.md §8(b) `dtype` of cwt_backbone_load;
 * BASELINE.json config #5 "mixed-precision bf16 conv + fp32 CWT").  The reference computes
 * in fp32 only; CWT_CONV_FP32 (the default) matches it to ~1e-5 per conv (bf16x3, see the
 * header comment).  CWT_CONV_BF16 runs every MFMA conv on plain bf16 operands with fp32
 * accumulation and stores the activations between convs as bf16 (the stem conv1, pooling and
 * the PPM branch stay fp32 arithmetic); the returned feature map is fp32 as before, so the
 * inner loop, the CWT and the classifier are unchanged fp32.  Applies to subsequent
 * cwt_extract_features calls with this backbone.  Returns CWT_EARG for an unknown value.
 */
#define CWT_CONV_FP32 0
#define CWT_CONV_BF16 1
int cwt_backbone_set_precision(cwt_backbone* bb, int precision);

/*
 * Frozen feature extractor forward (eval mode).
 * Replaces: PSPNet.extract_features(x) -> (f, []) (pspnet.py:172-181; get_feat_list
 *           pspnet.py:272-287; PPM pspnet.py:33-38; bottleneck pspnet.py:124-129).
 * img:  device fp32 NCHW [N,3,S,S] (S-1 divisible by 8).
 * feat: device fp32 NHWC [N,h,w,512] with h = (S-1)/8+1.
 */
int cwt_extract_features(cwt_ctx* ctx, const cwt_backbone* bb, const float* img, int N, int S,
                         float* feat, void* stream);

/*
 * Feature extractor forward in TRAINING mode (the reference's do_epoch quirk: model.train() at
 * the start of each epoch, model.eval() only before the first query, so the first support
 * extraction of every epoch runs train-mode; train.py:184,219,245).
 * Replaces: PSPNet.extract_features(x) with model.training == True (pspnet.py:172-181):
 *   every BatchNorm2d normalises with the batch statistics over N*h*w (PPM bins: N*b*b),
 *   then moves its running statistics by `momentum` (torch: unbiased variance) -- the
 *   backbone's eval-mode folds (and the PPM-branch weights) are rewritten on the device, so
 *   later cwt_extract_features calls see the updated statistics;
 *   Dropout2d(dropout_p) zeroes whole (image, channel) planes of the bottleneck output and
 *   scales the rest by 1/(1-dropout_p); mask = counter draw (seed, stream 3, n*512+c).
 * N >= 2 (the PPM bin-1 BatchNorm sees N values; torch raises for 1).  Not thread-safe
 * against concurrent extractions with the same backbone.
 */
/* extract_features with the per-layer features (pspnet.py:172-181 with an rmid of 'l..' /
 * 'mid', get_feat_list :272-287 with all_lr 'l': the last block of each layer): as
 * cwt_extract_features, plus fp32 NHWC copies of the outputs of layer2, layer3 and layer4
 * ([N][h][h][512 / 1024 / 2048], h = the feature side) into l2 / l3 / l4 (each may be NULL).
 * Eval-mode BN. */
int cwt_extract_features_mid(cwt_ctx* ctx, const cwt_backbone* bb, const float* img, int N, int S, float* feat,
                             float* l2, float* l3, float* l4, void* stream);

int cwt_extract_features_train_bn(cwt_ctx* ctx, cwt_backbone* bb, const float* img, int N, int S,
                                  float* feat, float momentum, float dropout_p, uint64_t seed,
                                  void* stream);

/*
 * Read back one BatchNorm2d's parameters as [4][C] floats (weight, bias, running_mean,
 * running_var) into host memory; name = the reference module prefix ("layer0.1",
 * "layer3.5.bn2", "ppm.features.2.2", "bottleneck.1").  Synchronises the device.  Replaces the
 * BN entries of PSPNet.state_dict() after train-mode extractions moved the statistics.
 */
int cwt_backbone_read_bn(const cwt_backbone* bb, const char* name, float* out, int C);

/*
 * Episode preprocessing on the device (the loader's transforms; dataset.py:205-327,
 * transform.py:59-167).  Replaces, per image: [RandomHorizontalFlip / RandomVerticalFlip
 * (flip_h / flip_v, decided by the caller)] -> Resize(S) (aspect kept, sides floored to a
 * multiple of 8, cv2 INTER_LINEAR, top-left placement, pad value `pad` (NULL: 0; 'avg'
 * padding: mean*255)) -> ToTensor (/255) -> Normalize(mean, std).
 * src: device HWC RGB, uint8 (CWT_U8) or fp32 (CWT_F32), H x W.  dst: device fp32 [3][S][S].
 * mean, std, pad: HOST float[3].
 */
#define CWT_U8 0
#define CWT_F32 1
int cwt_preprocess_image(cwt_ctx* ctx, const void* src, int src_dtype, int H, int W, int S,
                         const float* mean, const float* std_, const float* pad, int flip_h,
                         int flip_v, float* dst, void* stream);
/*
 * The episode label: chosen class -> 1, 255 kept, every other value -> 0 (dataset.py:222-228,
 * 261-266; class_chosen < 0 keeps the raw values), the same flips, cv2 INTER_NEAREST resize
 * to the Resize target and 255 padding to S x S.  src: device uint8 H x W; dst: device int64
 * [S][S].
 */
int cwt_preprocess_label(cwt_ctx* ctx, const uint8_t* src, int H, int W, int S, int class_chosen,
                         int flip_h, int flip_v, int64_t* dst, void* stream);

/* Bytes of device workspace the context holds (activations etc.; shared by all backbones). */
size_t cwt_workspace_bytes(cwt_ctx* ctx);

/*
 * Support-set inner loop: `iters` SGD steps of a bias-free 2-way 1x1 classifier on f_s,
 * loss = weighted CrossEntropy(ignore 255, mean) of the bilinear(align_corners=True)
 * upsampled logits vs s_label; class weight [1, #bg/#fg] counted on the device.
 * Replaces: test.py:164-187 and train.py:206-231 (nn.Conv2d(512,2,1) + F.interpolate +
 *           nn.CrossEntropyLoss(weight, ignore_index=255) + backward + optim.SGD(lr)).
 * f_s:     device fp32 NHWC [n,h,w,C];  s_label: device int64 [n,S,S] (0, 1, 255).
 * W_inout: device fp32 [2,C] — W0 on entry, adapted weights on return.
 * Returns CWT_EARG on bad shapes. A mask without foreground yields an infinite class
 * weight exactly like the reference; the caller checks counts if it needs to raise.
 */
int cwt_inner_adapt(cwt_ctx* ctx, const float* f_s, const int64_t* s_label, int n, int h, int w,
                    int C, int S, float lr, int iters, float* W_inout, void* stream);

/*
 * E independent inner loops (E episodes of n shots each) in the same launches: f_s NHWC
 * [E*n,h,w,C] (episode-major), s_label int64 [E*n,S,S], W_inout [E,2,C].  Episode e's result
 * is exactly what cwt_inner_adapt gives for its slices alone (its own class weight, W and
 * gradient accumulators).  Throughput form of test.py:164-187 for several episodes in flight
 * per GPU (the 200 dependent step launches are shared).  1 <= E <= 64.
 */
int cwt_inner_adapt_batch(cwt_ctx* ctx, const float* f_s, const int64_t* s_label, int E, int n, int h,
                          int w, int C, int S, float lr, int iters, float* W_inout, void* stream);

/* Per-pixel L2 normalisation over channels, F.normalize(f, dim=1) (test.py:194,
 * train.py:250): out[p,:] = f[p,:] / max(||f[p,:]||_2, 1e-12).  NHWC [P,C] -> [P,C].
 * If W0 (device [B,2,C]) and logits0 (device [B,2,P/B]) are non-NULL, also writes the
 * un-normalised baseline logits W0 . f (test.py:192 pred_q0) in the same pass. */
int cwt_normalize(cwt_ctx* ctx, const float* f, int B, int P_per_b, int C, float* out,
                  const float* W0, float* logits0, void* stream);

/*
 * Classifier Weight Transformer forward: MultiHeadAttentionOne(H, C, C, C).forward(q, k, v)
 * with k = v = f (transformer.py:54-83, ScaledDotProductAttention transformer.py:23-30),
 * eval mode (dropouts identity).  Computed in the re-associated form
 * scores_h = (W_h^T W_h q) . f / sqrt(C), out_h = W_h (softmax . f)  (DESIGN.md §CWT).
 * q:       device fp32 [B,2,C]         (classifier weights, transformer.py:66 residual)
 * f:       device fp32 NHWC [B,hw,C]   (normalised query features = keys = values)
 * w_qkvs:  device fp32 [H*C, C]; fc_w [C, H*C]; fc_b [C]; ln_w [C]; ln_b [C]
 * out:     device fp32 [B,2,C]
 * saved:   device fp32 buffer of cwt_attention_saved_floats(B,hw,C,H) floats kept for the
 *          backward pass, or NULL for inference.
 */
int cwt_attention_fwd(cwt_ctx* ctx, const float* q, const float* f, int B, int hw, int C, int H,
                      const float* w_qkvs, const float* fc_w, const float* fc_b, const float* ln_w,
                      const float* ln_b, float* out, float* saved, void* stream);
size_t cwt_attention_saved_floats(int B, int hw, int C, int H);

/*
 * Backward of cwt_attention_fwd w.r.t. the transformer parameters (q and f carry no
 * gradient in the reference: train.py:252-257 passes .data weights and no_grad features).
 * d_out: device [B,2,C].  Gradients are ACCUMULATED (+=) into g_* (device, same shapes as
 * the parameters), like autograd's .grad.
 */
int cwt_attention_bwd(cwt_ctx* ctx, const float* q, const float* f, int B, int hw, int C, int H,
                      const float* w_qkvs, const float* fc_w, const float* fc_b, const float* ln_w,
                      const float* ln_b, const float* saved, const float* d_out,
                      float* g_w_qkvs, float* g_fc_w, float* g_fc_b, float* g_ln_w, float* g_ln_b,
                      void* stream);

/*
 * Training-mode forms of the two calls above (MultiHeadAttentionOne.train(): transformer.py:17,28
 * nn.Dropout(0.1) on the attention probabilities after the softmax, transformer.py:52,80
 * nn.Dropout(dropout) on the fc output before the residual).  Kept elements are scaled by
 * 1/(1-p).  The masks come from a counter-based generator keyed by `seed` (include/cwt.h has no
 * state): pass the same seed to the backward call to regenerate them.  They are NOT torch's
 * Philox masks, so a training run matches the reference in distribution, not bit for bit; with
 * both probabilities 0 these are exactly cwt_attention_fwd / _bwd.
 */
int cwt_attention_fwd_train(cwt_ctx* ctx, const float* q, const float* f, int B, int hw, int C, int H,
                            const float* w_qkvs, const float* fc_w, const float* fc_b, const float* ln_w,
                            const float* ln_b, float* out, float* saved, float attn_dropout, float out_dropout,
                            uint64_t seed, void* stream);
int cwt_attention_bwd_train(cwt_ctx* ctx, const float* q, const float* f, int B, int hw, int C, int H,
                            const float* w_qkvs, const float* fc_w, const float* fc_b, const float* ln_w,
                            const float* ln_b, const float* saved, const float* d_out, float* g_w_qkvs,
                            float* g_fc_w, float* g_fc_b, float* g_ln_w, float* g_ln_b, float attn_dropout,
                            float out_dropout, uint64_t seed, void* stream);

/*
 * The inference episode's tail before the classifier as ONE call over the RAW query features:
 * f_hat = F.normalize(f_q) (test.py:194), pred_q0 = W . f_q (test.py:192) and
 * W' = MultiHeadAttentionOne(H, C, C, C).eval()(W, f_hat, f_hat) (test.py:195-197,
 * transformer.py:54-83), with the normalisation fused into the single pass over the tokens:
 * no normalised copy of f is written; inv_norm [B,hw] = 1 / max(||f_p||, 1e-12) is returned for
 * cwt_classify_scaled.  For fixed parameters the projections fold into per-head matrices
 * (W_h^T W_h and fc_h W_h), computed on this context's stream once per parameter identity --
 * (w_qkvs, fc_w, params_version): the caller bumps params_version whenever it modifies the
 * parameters in place (torch's tensor._version does).  Same function as cwt_normalize +
 * cwt_attention_fwd up to fp32 rounding (re-associated).  H must be 4.
 * q: device fp32 [B,2,C] (the adapted classifier, also the baseline's weights); f: NHWC [B,hw,C];
 * out [B,2,C]; inv_norm [B,hw]; logits0 [B,2,hw] or NULL.
 */
int cwt_attention_infer(cwt_ctx* ctx, const float* q, const float* f, int B, int hw, int C, int H,
                        const float* w_qkvs, const float* fc_w, const float* fc_b, const float* ln_w,
                        const float* ln_b, int64_t params_version, float* out, float* inv_norm, float* logits0,
                        void* stream);

/* logits = (W . f_p) * inv_norm[p] = W . F.normalize(f)_p (test.py:200-204 over the raw features
 * and cwt_attention_infer's inv_norm).  W [B,2,C]; f NHWC [B,P,C]; inv_norm [B,P]; logits [B,2,P]. */
int cwt_classify_scaled(cwt_ctx* ctx, const float* W, const float* f, const float* inv_norm, int B, int P, int C,
                        float* logits, void* stream);

/* Per-pixel classifier logits = W . f (test.py:200-204 Pseudo_cls; train.py:259-261 matmul).
 * W: device [B,2,C]; f: NHWC [B,P,C]; logits: device [B,2,P] (NCHW [B,2,h,w]). */
int cwt_classify(cwt_ctx* ctx, const float* W, const float* f, int B, int P, int C, float* logits,
                 void* stream);

/*
 * The inference episode's whole tail after the inner loop in ONE launch (test.py:190-224):
 * pred_q0 = W . f_q, f_hat = F.normalize(f_q), W' = MultiHeadAttentionOne(4, 512, 512, 512).eval()
 * (W, f_hat, f_hat), pred_q = W' . f_hat, and the upsample / argmax / intersection-union-target /
 * CE of pred_q and pred_q0 against q_label (util.py:237-308) -- what cwt_attention_infer +
 * cwt_classify_scaled + cwt_seg_metrics_pair compute in 8 launches, as one grid of co-resident
 * workgroups with in-kernel grid barriers between the phases.  The folded weights
 * follow (w_qkvs, fc_w, params_version) as in cwt_attention_infer.  C = 512, H = 4, B <= 4,
 * hw = h*w <= 16384, S - 1 == 8 (h - 1).
 * q [B,2,C] (the adapted W); f NHWC [B,hw,C] raw; q_label int64 [B,S,S]; out W' [B,2,C];
 * logits / logits0 [B,2,hw]; iut / iut0 fp32 [B,3,2]; ce fp64 [B,2] (sum of -log p_y, count).
 * A grid barrier that cannot complete sets CWT_STATUS_TAIL_BARRIER.
 */
int cwt_episode_tail(cwt_ctx* ctx, const float* q, const float* f, int B, int h, int w, int S, const int64_t* q_label,
                     const float* w_qkvs, const float* fc_w, const float* fc_b, const float* ln_w, const float* ln_b,
                     int64_t params_version, float* out, float* logits, float* logits0, float* iut, double* ce,
                     float* iut0, void* stream);

/*
 * One episode's inner loop and post-loop tail (test.py:164-224): cwt_inner_adapt on f_s /
 * s_label / W_inout, then cwt_episode_tail with q = the adapted W and B = 1 query (f_q, q_label),
 * with the same outputs.  Where the loop runs as the persistent two-unit form (the episode
 * pipeline's adapt context: cwt_ctx_set_adapt_units 2) the tail is FUSED behind the loop's last
 * step in the same launch: the loop's resident workgroups run the tail's phases instead of a
 * second grid that waits for CUs.  Elsewhere (and with CWT_FUSED_LOOP_TAIL=0) it makes the two
 * calls.  The profile splits a fused launch into its loop part ("inner_adapt_kernel [...]") and
 * its tail part ("episode_tail_kernel", "post_loop_tail") by in-kernel realtime stamps.
 * Status: a loop barrier that cannot complete sets CWT_STATUS_ADAPT_BARRIER (the tail is then
 * skipped), a tail barrier CWT_STATUS_TAIL_BARRIER.
 */
int cwt_inner_adapt_tail(cwt_ctx* ctx, const float* f_s, const int64_t* s_label, int n, int h, int w, int C, int S,
                         float lr, int iters, float* W_inout, const float* f_q, const int64_t* q_label,
                         const float* w_qkvs, const float* fc_w, const float* fc_b, const float* ln_w,
                         const float* ln_b, int64_t params_version, float* out, float* logits, float* logits0,
                         float* iut, double* ce, float* iut0, void* stream);

/*
 * Segmentation metrics of low-res logits against a full-res label:
 * bilinear(align_corners=True) upsample [B,2,h,w] -> [B,2,S,S], argmax over classes,
 * preds[target==255] = 255, histc intersection / union / target over 2 classes
 * (util.py:237-308 batch_intersectionAndUnionGPU / intersectionAndUnionGPU), plus the
 * CrossEntropy(ignore 255) sum and valid-pixel count of the upsampled logits
 * (test.py:222-224 criterion_standard).
 * iut_out: device fp32 [B,3,2] (intersection, union, target per class);
 * ce_out:  device fp64 [B,2] (sum of -log p_y, count) or NULL.
 */
int cwt_seg_metrics(cwt_ctx* ctx, const float* logits, const int64_t* target, int B, int h, int w,
                    int S, float* iut_out, double* ce_out, void* stream);

/*
 * cwt_seg_metrics for an episode's two logits tensors against one target in the same two
 * launches: logits (pred_q: iut_out, ce_out as above) and logits0 (the un-adapted baseline
 * pred_q0, test.py:192,200-204: iut0_out only).  Results equal two cwt_seg_metrics calls.
 */
int cwt_seg_metrics_pair(cwt_ctx* ctx, const float* logits, const float* logits0, const int64_t* target,
                         int B, int h, int w, int S, float* iut_out, double* ce_out, float* iut0_out,
                         void* stream);

/*
 * Weighted CE of upsampled logits and its gradient w.r.t. the low-res logits, for the
 * outer loop (train.py:237-243,261-265): class weight [1, #bg/(#fg+1e-12)] from target,
 * loss = sum_p w_y * nll_p / sum_p w_y over non-ignored p.
 * logits: device [B,2,h,w]; target int64 [B,S,S]; loss_out device fp32 [1];
 * dlogits: device [B,2,h,w] (overwritten).
 */
int cwt_seg_ce_fwd_bwd(cwt_ctx* ctx, const float* logits, const int64_t* target, int B, int h,
                       int w, int S, float* loss_out, float* dlogits, void* stream);

/* intersectionAndUnionGPU on argmax maps (util.py:280-308): preds/target device int64 [n];
 * preds[target==ignore] are ignored; histc over classes 0..num_classes-1 (num_classes <= 16).
 * iut_out: device fp32 [3, num_classes] (intersection, union, target). */
int cwt_iou_preds(cwt_ctx* ctx, const int64_t* preds, const int64_t* target, int64_t n, int num_classes,
                  int ignore_index, float* iut_out, void* stream);

/* dW[b,c,:] += sum_p dlogits[b,c,p] * f[b,p,:]  (backward of cwt_classify w.r.t. W). */
int cwt_classify_bwd(cwt_ctx* ctx, const float* dlogits, const float* f, int B, int P, int C,
                     float* dW, void* stream);

/*
 * Variant heads on the same features.
 *
 * CosCls.forward (src/model/pspnet.py:290-309, cls_type parsed by parse_param_coscls :318-324):
 * x device [B, P, C] (NHWC tokens, C = 512); weight device [n, C] (the stored cls.weight, or
 * cls.weight_v under WeightNorm), g device [n] (cls.weight_g, WeightNorm only), bias device
 * [n] or NULL, scale device [1] (scale_factor: the constant 2.0 or the learnable parameter);
 * mode bit 0 = WeightNorm ('r': W = g v / ||v||), bit 1 = weight_norm ('n': rows of the stored
 * weight normalised in place with eps 1e-5 before use -- no effect under WeightNorm, whose
 * pre-forward hook recomputes the weight, as in the reference).  out device [B, n, P]:
 * scale * (W . x / max(||x||, 1e-5) + bias).  n <= 64.
 * cwt_cos_classify_bwd: the gradients of sum(dscores * out) w.r.t. the head's parameters:
 * d_weight [n, C] (w.r.t. weight_v under WeightNorm), d_g [n] (WeightNorm), d_bias [n] (may be
 * NULL), d_scale [1] (may be NULL); written, not accumulated; fixed-order sums.
 */
int cwt_cos_classify(cwt_ctx* ctx, const float* x, int B, int P, int C, int n, float* weight,
                     const float* g, const float* bias, const float* scale, int mode, float* out,
                     void* stream);
int cwt_cos_classify_bwd(cwt_ctx* ctx, const float* x, int B, int P, int C, int n, float* weight,
                         const float* g, const float* bias, const float* scale, int mode,
                         const float* dscores, float* d_weight, float* d_g, float* d_bias,
                         float* d_scale, void* stream);

/* get_corr (src/model/model_util.py:101-109; the MMN / MatchNet correlation, mmn.py:57):
 * q device [B, Pq, C], k device [B, Pk, C] (NHWC tokens); sim device [B, Pq, Pk] =
 * normalize(q) . normalize(k)^T per token (eps 1e-12), exact fp32 (fp32 MFMA). */
int cwt_corr(cwt_ctx* ctx, const float* q, const float* k, int B, int Pq, int Pk, int C, float* sim,
             void* stream);

/* MutualMatching (src/model/match.py:21-53), per channel: x device [B][NA][NB][C] (channels
 * last: x[b][a][j][c] = corr4d[b, c, a, j] with a, j the flattened query / support positions);
 * y = x * ((x / (max_a x + 1e-5)) * (x / (max_j x + 1e-5))), the maxima per (b, c) over all
 * query positions a (for each j) and all support positions j (for each a).  y may alias x.
 * C <= 64. */
int cwt_mutual_matching(cwt_ctx* ctx, const float* x, int B, int NA, int NB, int C, float* y, void* stream);

/* MatchNet.corr_forward (src/model/match.py:142-163; NeighConsensus :56-85 with the default
 * kernel sizes [3,3,3], channels [10,10,1] and CenterPivotConv4d layers, conv4d.py:11-62):
 * corr device [B][L][h*w][h*w] (the torch [B, L, h, w, h, w] tensor, L = in_channel 1 or 2);
 * nc_params device: per layer l = 0, 1, 2 (channels L -> 10 -> 10 -> 1) conv1.weight [co][ci][3][3],
 * conv1.bias [co], conv2.weight [co][ci][3][3], conv2.bias [co], concatenated (the order of
 * NeighConsensus.conv.{0,2,4}.{conv1,conv2}.{weight,bias} in its state_dict); symmetric = the
 * sym_mode flag; temp the softmax temperature.  corr2d device [B][h*w][h*w] receives
 * run_match_model's output (the ret_attn corr2d); with weighted_v non-NULL, v device
 * [B][h*w][Cv] (NHWC tokens of the support feature) gives weighted_v device [B][h*w][Cv] =
 * softmax(temp * corr2d, -1) . v (tokens of bmm(v, attn^T)).  Exact fp32. */
int cwt_match_corr_forward(cwt_ctx* ctx, const float* corr, int B, int L, int h, int w, const float* nc_params,
                           int symmetric, float temp, const float* v, int Cv, float* corr2d, float* weighted_v,
                           void* stream);

/* cwt_match_corr_forward with NeighConsensus over full Conv4d layers (conv='cv4', src/model/
 * conv4d.py:64-138; match.py:15,56-85): nc_params device = per layer (0, 2, 4) the reference's
 * pre-permuted weight [3][co][ci][3][3][3] then its bias [co].  fp32 VALU (no MFMA path: every
 * reference config uses 'red'). */
int cwt_match_corr_forward_cv4(cwt_ctx* ctx, const float* corr, int B, int L, int h, int w, const float* nc_params,
                               int symmetric, float temp, const float* v, int Cv, float* corr2d, float* weighted_v,
                               void* stream);

/* The spatial context descriptor of MatchNet's sce option (src/model/base/spatial_context.py:
 * 13-65, generate_spatial_descriptor + featureL2Norm): x device [B][h][w][C] (NHWC tokens), k odd
 * (the reference uses 25), g device [B][h*w][ldg], ldg >= k*k: the dot products of each pixel's
 * feature with its k x k window (zero padded), divided by sqrt(sum of squares + 1e-6); columns
 * k*k .. ldg-1 are zero.  C + k*k floats must fit 64 KB.  Exact fp32. */
int cwt_sce_descriptor(cwt_ctx* ctx, const float* x, int B, int h, int w, int C, int k, int ldg, float* g,
                       void* stream);

/* MMN's agg 'sum' (src/model/mmn.py:62-63, torch.sum(corr4d, dim=1, keepdim=True)): x device
 * [B][L][P], y device [B][P] = the sum over l, in order of l. */
int cwt_channel_sum(cwt_ctx* ctx, const float* x, int B, int L, int64_t P, float* y, void* stream);

/* MatchNet.forward's support masks on corr2d device [B][NA][NB], in place (src/model/match.py:
 * 117-126 and run_cyc, match.py:165-182).  ig_mask device [B][NB] uint8 (NULL: none) sets every
 * query row's entry of a masked support position to 1e-4.  With s_mask device [B][NB] int64 (the
 * support label map; NULL: no cycle mask), after the ig mask: k2q[j] = argmax over the queries,
 * q2k[a] = argmax over the supports (first index on ties, as torch's CPU max), inconsistent
 * device [B][NB] = s_mask[j] != s_mask[q2k[k2q[j]]] as 0 / 1, and corr2d += inconsistent * -1000.
 * The reference's Dropout(0.1) on the mask is its eval-mode identity. */
int cwt_match_masks(cwt_ctx* ctx, float* corr2d, int B, int NA, int NB, const uint8_t* ig_mask,
                    const int64_t* s_mask, float* inconsistent, void* stream);
/* The same in training mode (match.py:97,181 ass_drop = nn.Dropout(0.1) on the cycle mask):
 * inconsistent[b][j] is scaled by the counter-based dropout draw (common.h dropout_scale, stream 5,
 * index b NB + j; kept entries 1 / (1 - drop_p)) before corr2d += inconsistent * -1000. */
int cwt_match_masks_train(cwt_ctx* ctx, float* corr2d, int B, int NA, int NB, const uint8_t* ig_mask,
                          const int64_t* s_mask, float* inconsistent, float drop_p, uint64_t seed, void* stream);

/* MatchNet's readout (match.py:128-130): weighted_v device [B][NA][Cv] = softmax(temp * corr2d,
 * -1) . v, v device [B][NB][Cv] (NHWC tokens).  Exact fp32. */
int cwt_match_readout(cwt_ctx* ctx, const float* corr2d, int B, int NA, int NB, float temp, const float* v, int Cv,
                      float* weighted_v, void* stream);
/* Its backward (MatchNet.forward under autograd with the support masks, match.py:117-130):
 * corr2d the masked corr2d the readout saw, d_weighted_v device [B][NA][Cv] -> d_corr2d device
 * [B][NA][NB] += the softmax readout's gradient, then zeroed on the ig-masked support columns
 * (those entries were overwritten by a constant; the -1000 * inconsistent shift passes the
 * gradient unchanged); d_v device [B][NB][Cv] = attn^T . d_weighted_v (NULL: skipped).  Cv % 4 == 0.
 * d_weighted_v NULL: only the ig columns of d_corr2d are zeroed. */
int cwt_match_readout_backward(cwt_ctx* ctx, const float* corr2d, int B, int NA, int NB, float temp, const float* v,
                               int Cv, const float* d_weighted_v, const uint8_t* ig_mask, float* d_corr2d, float* d_v,
                               void* stream);

/* WeightAverage (src/model/msm/msm_func.py:50-104, R = 3; the MMN head's wa_<layer> modules,
 * mmn.py:27-34,53-55): x device [N][h][w][C] (NHWC tokens), C = c_in in {512, 1024, 2048};
 * w_tpg device [3 C/2][C] = conv_theta.weight, conv_phi.weight, conv_g.weight stacked (each
 * [C/2][C]); b_theta / b_phi / b_g device [C/2]; w_back device [C][C/2], b_back device [C].
 * out device [N][h][w][C] = x + conv_back(sum_r softmax_r(cos(phi(x_r), theta(x))) g(x_r)) over
 * the 3x3 replicate-padded neighbourhood r (CosineSimilarity: dot / (max|a| max|b|), eps 1e-8).
 * Dropouts are identities (att_drop / proj_drop default 0, eval).  Exact fp32. */
int cwt_weight_average(cwt_ctx* ctx, const float* x, int N, int h, int w, int C, const float* w_tpg,
                       const float* b_theta, const float* b_phi, const float* b_g, const float* w_back,
                       const float* b_back, float* out, void* stream);

/* MMN.forward's tail (src/model/mmn.py:65-67): att_fq device [B][n] (the B support rows'
 * weighted query features, n = h*w*C), f_q device [n]; att_mean device [n] = mean over B;
 * fq_out device [n] = f_q * (1 - att_wt) + att_mean * att_wt. */
int cwt_mmn_blend(cwt_ctx* ctx, const float* f_q, const float* att_fq, int B, int64_t n, float att_wt,
                  float* att_mean, float* fq_out, void* stream);

/* ---- MatchNet / MMN training: the backward the reference's autograd runs through the head ----
 * (MMN trained end to end by src/train_cca.py:101-196 and src/train_aug.py:102; DeTr's MatchNet
 * cross attention by src/train_trans.py:100).  Every gradient is exact fp32 with fixed-order
 * reductions (deterministic); outputs are overwritten unless an accumulate flag says otherwise. */

/* Scheduling query of the episode pipeline (no reference counterpart; test.py:164-187 is the loop
 * it sizes): the number of workgroups -- each holding one whole CU for the whole loop -- of the
 * persistent inner loop cwt_inner_adapt_batch would launch on this context for E episodes of n
 * shots with h x w features (0: it would use the per-step launches).  EpisodePipeline runs a
 * burst's last two loops side by side only when the two grids fit on the chip together. */
int cwt_adapt_workgroups(cwt_ctx* ctx, int E, int n, int h, int w, int iters, int* G);

/* 1 if cwt_inner_adapt_tail on this context runs the episode tail inside the inner loop's own
 * launch (the two-unit persistent form, EpisodePipeline's adapt context), else 0 (it then launches
 * the tail as a grid of its own, which needs CUs beside the loop). */
int cwt_adapt_fuses_tail(cwt_ctx* ctx, int n, int h, int w, int iters, int* fused);

/* Floats of the activations cwt_match_corr_forward_train keeps for the backward (CenterPivotConv4d
 * layers): the MutualMatching output, each branch's three ReLU outputs, their sum and, with
 * readout != 0, the attention [B][h*w][ld] (ld = h*w rounded up to 32). */
int cwt_match_corr_saved_floats(int B, int L, int h, int w, int symmetric, int readout, int64_t* n);

/* cwt_match_corr_forward (match.py:142-163, 'red' layers) keeping its activations in saved
 * device [cwt_match_corr_saved_floats]: the forward of MatchNet.corr_forward under autograd. */
int cwt_match_corr_forward_train(cwt_ctx* ctx, const float* corr, int B, int L, int h, int w,
                                 const float* nc_params, int symmetric, float temp, const float* v, int Cv,
                                 float* corr2d, float* weighted_v, float* saved, void* stream);

/* Its backward: d_corr2d device [B][h*w][h*w] (the gradient at corr2d, or NULL) and d_weighted_v
 * device [B][h*w][Cv] (at weighted_v, or NULL) -> d_corr device [B][L][h*w][h*w] (or NULL), d_params
 * device (nc_params' layout: every conv1 / conv2 weight and bias of the three layers, both branches
 * summed), d_v device [B][h*w][Cv] (or NULL).  MutualMatching's maxima route their gradient to the
 * first maximal position (torch.max's single index); Cv % 4 == 0. */
int cwt_match_corr_backward(cwt_ctx* ctx, const float* corr, int B, int L, int h, int w, const float* nc_params,
                            int symmetric, float temp, const float* v, int Cv, const float* saved,
                            const float* d_corr2d, const float* d_weighted_v, float* d_corr, float* d_params,
                            float* d_v, void* stream);

/* get_corr's backward (src/model/model_util.py:101-109: sim = normalize(q) . normalize(k)^T,
 * F.normalize eps 1e-12): q device [B][Pq][C], k device [B][Pk][C] (tokens), d_sim device
 * [B][Pq][Pk] -> dq device [B][Pq][C] and dk device [B][Pk][C] (either may be NULL), added into
 * when accum_q / accum_k != 0 (a query feature shared by the B support rows, mmn.py:50). */
int cwt_corr_backward(cwt_ctx* ctx, const float* q, const float* k, int B, int Pq, int Pk, int C, const float* d_sim,
                      float* dq, float* dk, int accum_q, int accum_k, void* stream);

/* cwt_weight_average keeping tpg device [N*h*w][3 C/2] (theta | phi | g before their biases) and
 * wavg device [N*h*w][C/2] (the softmax-weighted g) for the backward. */
int cwt_weight_average_train(cwt_ctx* ctx, const float* x, int N, int h, int w, int C, const float* w_tpg,
                             const float* b_theta, const float* b_phi, const float* b_g, const float* w_back,
                             const float* b_back, float* out, float* tpg, float* wavg, void* stream);

/* WeightAverage's backward (msm_func.py:66-104): d_out device [N][h][w][C] -> d_x device
 * [N][h][w][C] (or NULL), d_w_tpg device [3 C/2][C], d_b_theta / d_b_phi / d_b_g [C/2], d_w_back
 * [C][C/2], d_b_back [C]; tpg / wavg from cwt_weight_average_train. */
int cwt_weight_average_backward(cwt_ctx* ctx, const float* x, int N, int h, int w, int C, const float* w_tpg,
                                const float* b_theta, const float* b_phi, const float* b_g, const float* w_back,
                                const float* tpg, const float* wavg, const float* d_out, float* d_x,
                                float* d_w_tpg, float* d_b_theta, float* d_b_phi, float* d_b_g, float* d_w_back,
                                float* d_b_back, void* stream);

/* cwt_mmn_blend's backward: d_fq device [n] (at fq_out, or NULL), d_att_mean device [n] (at
 * att_mean, or NULL) -> d_att device [B][n], d_fq_in device [n] (or NULL). */
int cwt_mmn_blend_backward(cwt_ctx* ctx, const float* d_fq, const float* d_att_mean, int B, int64_t n, float att_wt,
                           float* d_att, float* d_fq_in, void* stream);

/* cwt_linear's backward (nn.Linear / the 1x1 nn.Conv2d of detr.py:22, ms_deform_attn.py:56-59):
 * x device [P][K], w device [N][K], out device [P][N] the forward's output when it ended in a ReLU
 * (its > 0 mask gates d_out) or NULL, d_out device [P][N] -> d_x device [P][K], d_w device [N][ldw]
 * (a column slice of a wider weight when ldw > K: adjust_feature's per-layer segments), d_b device
 * [N]; each may be NULL. */
int cwt_linear_backward(cwt_ctx* ctx, const float* x, int64_t P, int K, const float* w, int N, const float* out,
                        const float* d_out, float* d_x, float* d_w, int ldw, float* d_b, void* stream);

/* cwt_deform_attn's backward (ms_deform_attn.py:99-117, ms_deform_attn_func.py:41-61 under autograd;
 * one level, DeTr's pixel-centre reference points): d_out device [B][H*W][n_heads*d_head] ->
 * d_value (same shape; the reference CUDA op scatters it with float atomics, run-to-run
 * nondeterministic: here in 64-bit fixed point with integer atomics, deterministic),
 * d_offsets device [B][H*W][n_heads][n_points][2], d_logits device [B][H*W][n_heads][n_points]. */
int cwt_deform_attn_backward(cwt_ctx* ctx, const float* value, const float* offsets, const float* logits, int B, int H,
                             int W, int n_heads, int n_points, int d_head, const float* d_out, float* d_value,
                             float* d_offsets, float* d_logits, void* stream);

/* cwt_norm_blend's backward (detr.py:41,45): d_out device [T][C] -> d_a, d_b device [T][C] (either
 * may be NULL). */
int cwt_norm_blend_backward(cwt_ctx* ctx, const float* a, const float* b, int64_t T, int C, float wt, const float* d_out,
                            float* d_a, float* d_b, void* stream);

/* ---- DeTr head (src/model/detr.py:13-151), forward only; tokens are [B][hw][C] (NHWC) ---- */

/* nn.Linear / 1x1 nn.Conv2d over tokens (detr.py:22 adjust_feature, ms_deform_attn.py:56-59
 * value_proj / sampling_offsets / attention_weights / output_proj): x device [P][K] (K % 4 == 0),
 * w device [N][K] (the module's weight), bias device [N] or NULL; out device [P][N] =
 * relu?(x w^T + bias (+ out when accumulate != 0: a second input segment of a channel concat,
 * detr.py:56-59)).  Exact fp32 (f32 MFMA). */
int cwt_linear(cwt_ctx* ctx, const float* x, int64_t P, int K, const float* w, const float* bias, int N, int relu,
               int accumulate, float* out, void* stream);

/* query + SinePositionalEncoding(C/2, temperature, normalize, scale, eps)(mask) with the mask
 * DeformAtt.get_qry_flatten_input builds without a padding mask (detr.py:135: a zero LONG tensor,
 * so ~mask = -1 and the cumulative embeddings run -1, -2, ...; positional_encoding.py:44-74):
 * x, out device [B][h][w][C]. */
int cwt_sine_pos_add(cwt_ctx* ctx, const float* x, int B, int h, int w, int C, float temperature, int normalize,
                     float scale, float eps, float* out, void* stream);

/* MSDeformAttn's core over one level (ms_deform_attn.py:84-117 with ms_deform_attn_core_pytorch,
 * ms_deform_attn_func.py:41-61; DeformAtt's reference points, detr.py:98-110): value device
 * [B][H*W][n_heads*d_head] (value_proj output), offsets device [B][H*W][n_heads][n_points][2]
 * (sampling_offsets output, (x, y)), logits device [B][H*W][n_heads][n_points] (attention_weights
 * output, before the softmax); out device [B][H*W][n_heads*d_head] = sum_p softmax_p(logits)
 * grid_sample(value_head, 2 (ref + off / (W, H)) - 1) (bilinear, zeros, align_corners False).
 * n_points <= 16, d_head <= 64. */
int cwt_deform_attn(cwt_ctx* ctx, const float* value, const float* offsets, const float* logits, int B, int H, int W,
                    int n_heads, int n_points, int d_head, float* out, void* stream);

/* DeTr's blends (detr.py:41,45): out[t] = F.normalize(a[t]) + F.normalize(b[t]) * wt over T
 * tokens of C channels (eps 1e-12); a, b, out device [T][C]. */
int cwt_norm_blend(cwt_ctx* ctx, const float* a, const float* b, int64_t T, int C, float wt, float* out,
                   void* stream);

/* torch.optim.SGD(momentum, dampening 0, weight_decay, nesterov) step over one flat
 * fp32 parameter buffer (optimizer.py:8-15): buf = m*buf + (g + wd*p) (buf = g+wd*p on
 * the first step, first_step != 0); p -= lr * (nesterov ? g + wd*p + m*buf : buf). */
int cwt_sgd_step(cwt_ctx* ctx, float* param, const float* grad, float* momentum_buf, int64_t n,
                 float lr, float momentum, float weight_decay, int nesterov, int first_step,
                 void* stream);

/*
 * Stage-1 pretraining of the whole PSPNet (reference src/pretrain.py).
 * A cwt_pretrain holds the trainable model: every parameter, its gradient and SGD momentum
 * buffer in one flat fp32 device buffer each (layer0-4 = SGD group 1, ppm / bottleneck /
 * classifier = group 2, pretrain.py:60-72), the BN running statistics, and the activations
 * of the last forward.  All arithmetic is exact fp32 (f32 MFMA convs, weight gradients and
 * input gradients), BN in training mode as model.train() (pretrain.py:106).
 */
typedef struct cwt_pretrain cwt_pretrain;

typedef struct cwt_pretrain_hparams {
  float lr;            /* group 1 (layer0-4): args.lr (scheduler value of this iteration) */
  float lr_head;       /* group 2 (ppm, bottleneck, classifier): args.lr * args.scale_lr */
  float momentum;      /* args.momentum (SGD, dampening 0) */
  float weight_decay;  /* args.weight_decay (applied to every parameter, as torch.optim.SGD) */
  int nesterov;        /* args.nesterov */
  int smoothing;       /* args.smoothing: one-hot smoothed to 0.9 / 0.1 / (C - 1) (pretrain.py:197-199) */
  float bn_momentum;   /* nn.BatchNorm2d momentum (0.1) */
  float drop_p;        /* Dropout2d of the bottleneck (args.dropout; counter-based masks, seed below) */
  uint64_t seed;
  int ignore_index;    /* 255 */
} cwt_pretrain_hparams;

#define CWT_PT_PARAM 0
#define CWT_PT_GRAD 1
#define CWT_PT_MOMENTUM 2
#define CWT_PT_RUNNING 3

/* Replaces: get_model(args) + the SGD param groups (pretrain.py:60-72), from a PSPNet
 * state_dict given by name as in cwt_backbone_load (classifier.weight [num_classes, 512, 1, 1],
 * num_classes = args.num_classes_tr: 2, 16 or 61). */
int cwt_pretrain_create(cwt_ctx* ctx, int layers, int num_classes, int n_tensors, const char* const* names,
                        const float* const* host_data, const int64_t* numel, float bn_eps, cwt_pretrain** out);
int cwt_pretrain_destroy(cwt_pretrain* pt);

/* One training iteration (pretrain.py:104-121): model.train(); loss = compute_loss(...)
 * (:182-219, mixup off); optimizer.zero_grad(); loss.backward(); optimizer.step().
 * images device [N, 3, S, S] fp32 (NCHW, as the reference's loader yields), labels device
 * [N, S, S] int64 (255 = ignore); N >= 2; (S - 1) % 8 == 0.  *loss_out (device float) = the
 * loss before the step.  Gradients are left in place (CWT_PT_GRAD) until the next step. */
int cwt_pretrain_step(cwt_ctx* ctx, cwt_pretrain* pt, const float* images, const int64_t* labels, int N, int S,
                      const cwt_pretrain_hparams* hp, float* loss_out, void* stream);

/* model(images) before the upsample (pspnet.py:147-156 with classify's conv only): logits
 * device [N, h, h, num_classes] (NHWC), h = (S - 1) / 8 + 1.  train = 0: eval mode (running
 * statistics); train = 1: batch statistics, running statistics untouched, no dropout. */
int cwt_pretrain_forward(cwt_ctx* ctx, cwt_pretrain* pt, const float* images, int N, int S, int train,
                         float* logits, void* stream);

/* Evaluation pass of pretrain.py:223-250 (standard_validate) / :123-131 (the logging block) for
 * one batch: logits = model(images) (train = 0: eval mode as model.eval(); 1: batch statistics,
 * running statistics untouched), nn.CrossEntropyLoss(ignore_index=255) of the upsampled logits ->
 * loss_out device float[2] = {mean loss, valid pixels}; intersectionAndUnionGPU(logits.argmax(1),
 * gt, num_classes, 255) (util.py:280-308) -> iu_out device float[3][num_classes] = intersection,
 * union, target.  labels device [N, S, S] int64. */
int cwt_pretrain_evaluate(cwt_ctx* ctx, cwt_pretrain* pt, const float* images, const int64_t* labels, int N, int S,
                          int train, float* loss_out, float* iu_out, void* stream);

/* Host copy of one tensor in PyTorch layout by state_dict name: what = CWT_PT_PARAM, _GRAD,
 * _MOMENTUM (a parameter name) or CWT_PT_RUNNING ("<bn>.running_mean" / ".running_var").
 * Synchronises the device. */
int cwt_pretrain_get(cwt_pretrain* pt, const char* name, int what, float* host_out, int64_t numel);
/* The inverse of cwt_pretrain_get (what = CWT_PT_PARAM, _MOMENTUM or _RUNNING; PyTorch layout):
 * model.load_state_dict / optimizer.load_state_dict when training resumes from a checkpoint
 * (pretrain.py:147-152 writes {'epoch', 'state_dict', 'optimizer'}).  Setting a momentum buffer
 * marks the optimizer as started (no first-step initialisation of the buffers).  Synchronises. */
int cwt_pretrain_set(cwt_pretrain* pt, const char* name, int what, const float* host_in, int64_t numel);
int cwt_pretrain_num_params(const cwt_pretrain* pt, int64_t* total, int64_t* backbone);

/*
 * Per-launch profiling (no reference counterpart; measurement support for bench.py).
 * level 1: the context records a hipEvent pair on the call's stream around each whole
 *          cwt_extract_features, its bottleneck conv (the largest single launch), the whole
 *          cwt_inner_adapt loop and cwt_attention_fwd;
 * level 2: additionally around every conv / stem / maxpool / PPM launch (adds ~10 us of
 *          event overhead per launch: use for per-layer tables, not for timing);
 * each record carries the algorithmic FLOPs and minimal HBM bytes of the bracket
 * (SURVEY.md §8(d)).  Enabling (level > 0) clears the records; 0 stops recording.
 * cwt_profile_record waits for record i's stop event and returns its elapsed time.
 */
/*
 * Scheduling knob (no reference counterpart): how many 64-pixel units of the support map one
 * workgroup of the persistent inner loop holds (0 = automatic, 1, 2 or 3).  2 halves the CUs the
 * loop occupies, for contexts whose inner loops run beside another stream's extractor pass
 * (few_shot_seg_cwt_amd.episode.EpisodePipeline); results are the same either way.
 */
int cwt_ctx_set_adapt_units(cwt_ctx* ctx, int units_per_workgroup);

/*
 * Asynchronous failures of work already enqueued on this context (no reference counterpart:
 * the reference's torch ops fail synchronously).  A kernel that detects a failure it cannot
 * return -- today the persistent inner loop whose grid barrier does not complete within its
 * bound (co-residency lost), leaving W unadapted -- ORs a CWT_STATUS_* bit into a word in
 * mapped host memory.  Read it after the caller has synchronised the stream (e.g. after the
 * episode's IoU readback): *status receives the word; clear != 0 resets it.  No GPU call.
 */
int cwt_ctx_status(cwt_ctx* ctx, uint32_t* status, int clear);

/*
 * Arithmetic of this context's fp32 conv stack (no reference counterpart; the reference's
 * torch convs are fp32, src/model/resnet.py:57-96, pspnet.py:124-129):
 *   CWT_CONV_ARITH_BF16X6 (default, or CWT_CONV=x6) = fp32 width on the bf16 matrix cores: fp32
 *     activations and weights, each operand split exactly into bf16 hi + mid + lo in registers,
 *     the six products >= 2^-24 |a||b| summed with fp32 accumulation;
 *   CWT_CONV_ARITH_F32 (CWT_CONV=f32) = exact fp32 MFMA over fp32 activations;
 *   CWT_CONV_ARITH_BF16X3 (CWT_CONV=x3s) = a declared approximation: operands rounded to 16
 *     significant bits (bf16 hi + lo), three bf16 MFMA products.
 * Every packing is built at cwt_backbone_load, so this switches between calls.  A bf16
 * backbone (cwt_backbone_set_precision) is unaffected.
 */
#define CWT_CONV_ARITH_BF16X3 0
#define CWT_CONV_ARITH_F32 1
#define CWT_CONV_ARITH_BF16X6 2
int cwt_ctx_set_conv_arith(cwt_ctx* ctx, int arith);

int cwt_profile_enable(cwt_ctx* ctx, int level);
int cwt_profile_count(cwt_ctx* ctx);
int cwt_profile_record(cwt_ctx* ctx, int i, char* name, int name_len, double* flops, double* bytes,
                       float* ms);

#ifdef __cplusplus
}
#endif
#endif /* CWT_H_ */

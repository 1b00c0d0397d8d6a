/*
 * libcwt test and measurement hooks -- NOT part of the drop-in boundary (include/cwt.h).
 *
 * These entry points exist for the parity tests (tests/test_gpu_conv*.py run single convs
 * with forced plans), the timing studies (tools/persist_stamps.py, tools/adapt_stamps.py)
 * and the CU-partition probe.  A reference-side binding never needs them; they are exported
 * by the same libcwt.so so the tests exercise the shipped kernels.
 */
#ifndef CWT_DEBUG_H_
#define CWT_DEBUG_H_
#include "cwt.h"

#ifdef __cplusplus
extern "C" {
#endif

/*
 * Test hook: one exact-fp32 implicit-GEMM conv (CWT_CONV=f32, the training-mode-BN pass) +
 * folded BN (+residual) (+ReLU), NHWC, with the tile (bm x bn in {128x128, 128x64, 64x64}; 0 =
 * automatic) and split-K count (0 = automatic) forced, so every plan can be checked against a
 * reference conv.  precision must be 0 (the bf16x3 plans: cwt_debug_conv_s).  w_packed: device
 * [Co][k][k][Ci]; scale/shift: device [Co]; res: NHWC (pixel stride res_ld) or NULL.
 */
int cwt_debug_conv(cwt_ctx* ctx, const float* x, int N, int Hi, int Wi, int Ci, int x_ld,
                   const float* w_packed, const float* scale, const float* shift, int Co, int k,
                   int stride, int pad, int dil, const float* res, int res_ld, int relu, float* y,
                   int y_ld, int y_off, int bm, int bn, int nsplit, int precision, void* stream);

/*
 * Test hooks of the split-activation conv (conv_x3s.hip).  S-layout = [rows][C/32][64 bf16]:
 * per 32-channel block 32 x hi = bf16_rne(v) then 32 x lo = bf16_rne(v - hi).
 * cwt_debug_split_act: fp32 [P][C] (pixel stride ld) -> S-layout; cwt_debug_unsplit_act the
 * inverse (hi + lo).  cwt_debug_pack_wsplit: weights [Co][k][k][Ci] fp32 -> S-layout rows of
 * K = k*k*Ci in the library's K order.  cwt_debug_conv_s: one conv on S-layout input and
 * weights, folded BN, optional fp32 (res) or S-layout (res_s) residual, ReLU; writes fp32 NHWC
 * y (pixel stride y_ld, channel offset y_off) and/or S-layout ys; bm/bn/nsplit force the plan
 * (0 = automatic); bm = 1000 * variant + rows also forces the main-loop variant (0 base,
 * 1 fragment prefetch, 2 prefetch with 8 waves, 4 = 128x128 with a 2-stage ring; 8 .. 11 timing
 * study: 64x64 without MFMAs / without operand loads, 128x128 8-wave prefetch the same).
 */
int cwt_debug_split_act(cwt_ctx* ctx, const float* x, int64_t P, int C, int ld, void* out, void* stream);
int cwt_debug_unsplit_act(cwt_ctx* ctx, const void* s, int64_t P, int C, float* out, int ld, void* stream);
int cwt_debug_pack_wsplit(cwt_ctx* ctx, const float* w, int Co, int k, int Ci, void* out, void* stream);
int cwt_debug_conv_s(cwt_ctx* ctx, const void* xs, int N, int Hi, int Wi, int Ci, const void* ws,
                     const float* scale, const float* shift, int Co, int k, int stride, int pad,
                     int dil, const float* res, int res_ld, const void* res_s, int relu, float* y,
                     int y_ld, int y_off, void* ys, int bm, int bn, int nsplit, void* stream);
/* The same conv on plain bf16 operands (the CWT_CONV_BF16 kernel): xs bf16 NHWC [N*Hi*Wi][Ci]
 * (Ci % 64 == 0), ws bf16 [Co][K] with K ordered (64-channel block, tap, channel in block),
 * res_s / ys bf16 NHWC [M][Co]. */
int cwt_debug_conv_b16(cwt_ctx* ctx, const void* xs, int N, int Hi, int Wi, int Ci, const void* ws,
                       const float* scale, const float* shift, int Co, int k, int stride, int pad,
                       int dil, const float* res, int res_ld, const void* res_s, int relu, float* y,
                       int y_ld, int y_off, void* ys, int bm, int bn, int nsplit, void* stream);

/* The exact-fp32 conv on the LDS-DMA body (conv_igemm_f32d, the eval-mode exact path of
 * cwt_ctx_set_conv_arith(CWT_CONV_ARITH_F32)): x fp32 NHWC [N][Hi][Wi][Ci] (Ci % 32 == 0,
 * pixel stride Ci), w_packed fp32 [Co][K] in the packed_k order (32-channel block, tap, channel),
 * res fp32 [M][res_ld] or NULL, y fp32 [M][y_ld] at channel offset y_off.  bm / bn / nsplit as
 * cwt_debug_conv_s (bm = 1000 * variant + rows; 0 = the library's plan). */
int cwt_debug_conv_f32d(cwt_ctx* ctx, const float* x, int N, int Hi, int Wi, int Ci, const float* w_packed,
                        const float* scale, const float* shift, int Co, int k, int stride, int pad, int dil,
                        const float* res, int res_ld, int relu, float* y, int y_ld, int y_off, int bm, int bn,
                        int nsplit, void* stream);

/* The same conv at fp32 width on the bf16 matrix cores (conv_igemm_x6, the conv of
 * cwt_ctx_set_conv_arith(CWT_CONV_ARITH_BF16X6)): arguments and layouts as cwt_debug_conv_f32d. */
int cwt_debug_conv_x6(cwt_ctx* ctx, const float* x, int N, int Hi, int Wi, int Ci, const float* w_packed,
                      const float* scale, const float* shift, int Co, int k, int stride, int pad, int dil,
                      const float* res, int res_ld, int relu, float* y, int y_ld, int y_off, int bm, int bn,
                      int nsplit, void* stream);

/* The same conv in the Winograd F(2x2, 3x3) form on the x6 arithmetic (wino.hip; the form the
 * x6 stack takes for stride-1 3x3 layers with Ci >= 256): k == 3, stride 1, pad == dil; the weights
 * are transformed and split on the device each call; bm / bn pick the 16 batched GEMMs' tile
 * (nsplit ignored: the batch fills the chip). */
int cwt_debug_conv_x6w(cwt_ctx* ctx, const float* x, int N, int Hi, int Wi, int Ci, const float* w_packed,
                       const float* scale, const float* shift, int Co, int k, int stride, int pad, int dil,
                       const float* res, int res_ld, int relu, float* y, int y_ld, int y_off, int bm, int bn,
                       int nsplit, void* stream);

/* One CenterPivotConv4d layer + ReLU (src/model/conv4d.py:40-62) on the channels-last 4-D
 * tensor x [B][hA*wA][hB*wB][cin] -> y [B][hA*wA][hB*wB][cout]: Wa / Wb [cout][cin][3][3] the
 * a-plane / b-plane filters, ba / bb their biases.  variant 0: the library's kernel choice, 1:
 * never the rolling-window kernel (cp4d_roll_kernel), 2: only it (CWT_EARG where it has no form). */
int cwt_debug_cp4d_layer(cwt_ctx* ctx, const float* x, int B, int hA, int wA, int hB, int wB, int cin, int cout,
                         const float* Wa, const float* ba, const float* Wb, const float* bb, float* y, int variant,
                         void* stream);

/* Timing-study hook of cwt_episode_tail: with CWT_TAIL_STAMPS=1 in the environment the tail runs a
 * separately compiled instantiation whose workgroups record s_memtime at each phase edge
 * ([G][16]: 0 entry, 2k-1 / 2k before / after grid barrier k, 11 the partials written, 14 / 15
 * s_memrealtime at entry / before the ticket; tools/tail_stamps.py).  Copies up to max_count of
 * the last stamped launch's values to host_out; *count = G * 16 (0 if none). */
int cwt_debug_tail_stamps(cwt_ctx* ctx, unsigned long long* host_out, int64_t max_count, int64_t* count);

/* Timing-study hook: hold nwg CUs for about `us` microseconds (nwg workgroups of 1024 threads, each
 * taking a whole CU's LDS, spinning on the realtime clock with s_sleep, bounded), so a kernel timed
 * on another stream meanwhile sees the CUs the pipeline's resident inner loop leaves it.  nwg <= 256,
 * us <= 100000. */
int cwt_debug_occupy(cwt_ctx* ctx, int nwg, int us, void* stream);

/* Timing-study hook of the inner loop: with CWT_ADAPT_DBG=32 in the environment, the inner
 * loop runs a separately compiled instantiation that records clock stamps per step and
 * workgroup (persistent loop: tools/persist_stamps.py; per-step launches with
 * CWT_ADAPT_PERSIST=0: tools/adapt_stamps.py).  Copies up to max_count of them to host_out
 * (may be NULL) and stores the number available in *count. */
int cwt_debug_adapt_stamps(cwt_ctx* ctx, unsigned long long* host_out, int64_t max_count, int64_t* count);

/* Test hook: the persistent inner loop's per-barrier spin bound on this context (polls before
 * the grid gives up and raises CWT_STATUS_ADAPT_BARRIER); 0 restores the default (~4 s).  A
 * bound of 1 makes nearly every barrier time out, to exercise the error path. */
int cwt_debug_adapt_spin_limit(cwt_ctx* ctx, int64_t limit);

/* Test hooks of the pretraining step's teacher-forced per-block parity test
 * (tests/test_gpu_pretrain_chain.py).  capture != 0: the next cwt_pretrain_step keeps copies of
 * its transient backward gradients ("dlogits" [M][nc], "dcat" [M][2048] = the gradient at
 * layer4's output, "dx:l<layer>.<block>" = a ResNet block's input gradient [M][Ci]).
 * cwt_debug_pretrain_tensor copies one of those, or a forward tensor of the last step
 * ("in:l<layer>.<block>" = a block's input [M][Ci], "a:l<layer>.<block>.c<1|2|3>" = a conv's
 * BN (+ residual) + ReLU output, "a:stem<i>", "a:ppm<i>", "fpre" = the bottleneck's output before
 * Dropout2d, "cat" = layer4's output, "mp" = the stem's max-pool output, "logits" [M][nc]), to
 * host_out (numel floats, NHWC rows). */
int cwt_debug_pretrain_capture(cwt_pretrain* pt, int on);
int cwt_debug_pretrain_tensor(cwt_pretrain* pt, const char* name, float* host_out, int64_t numel);

/* Test hook: per workgroup of a 64-thread grid, the raw HW_REG_HW_ID and HW_REG_XCC_ID of the
 * CU it ran on (out[2*b], out[2*b+1]); with a CU-masked stream this maps mask bits to CUs. */
int cwt_debug_census(cwt_ctx* ctx, int nblocks, unsigned* out, void* stream);

/*
 * CU-partitioned streams (probe of episode pipelining, tools/cu_partition_probe.py): a HIP
 * stream whose kernels (including replays of graphs launched on it) only run on the CUs whose
 * bits are set in mask (mask_words 32-bit words, bit i = CU i of the device).
 * cwt_cu_count returns the device's CU count.
 */
int cwt_cu_count(cwt_ctx* ctx, int* count);
int cwt_stream_create_masked(cwt_ctx* ctx, const uint32_t* mask, int mask_words, void** stream);
int cwt_stream_destroy(void* stream);

/* Single steps of the pretraining iteration on caller buffers (tests/test_gpu_pretrain_ops.py):
 * op 0 conv weight gradient, 1 conv input gradient (b = dy, x | w, out; ia = N Hi Ci Co k stride
 * pad dil; NHWC fp32, weights packed [Co][K] as conv.hip), 2 label-smoothed CE (b = logits
 * [N][h][h][nc], int64 target, dlogits, loss; ia = N S h nc; fa = on off), 3 training BN + ReLU
 * forward and backward (b = y gamma beta out dout dy dgamma dbeta; ia = M C; fa = eps), 4 max
 * pool 3x3 s2 p1 forward and adjoint (b = in out dout din; ia = N H C), 5 the folded PPM field of
 * the bottleneck conv and its adjoint (b = P dF F dP W dW; ia = N h; P [cells][512] bin-major,
 * W / dW packed [512][4096 * 9], only dW's PPM columns written). */
int cwt_debug_pretrain_op(cwt_ctx* ctx, int op, void* const* bufs, const int64_t* iargs, const float* fargs,
                          void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CWT_DEBUG_H_ */

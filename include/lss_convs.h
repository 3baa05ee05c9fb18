/*
 * lss_convs.h -- C ABI of the conv-stack kernels beside the Lift-Splat hot path (same library,
 * liblss_hip.so). Not part of the reference's hot-path boundary (lss_hip.h): these replace MIOpen
 * for the depthwise convolutions of CamEncode's EfficientNet-B0 trunk (src/models.py:43, 63-84),
 * which MIOpen runs on naive kernels for bf16 NCHW.
 *
 * Depthwise (groups = C) 2-D convolution, no bias, dilation 1, NCHW contiguous activations of
 * element type dtype (fp32 or bf16), fp32 weights (C, 1, K, K), fp32 accumulation; K in {3, 5},
 * stride in {1, 2}. Padding is given as the top / left pads; the bottom / right pads are implied
 * by (Ho, Wo): taps that fall outside the input read zero (TF "same" static padding, asymmetric
 * for the stride-2 layers). Asynchronous on the stream; 0 on success, a positive hipError_t on a
 * launch failure, LSS_CONV_EINVAL for bad arguments.
 */
#ifndef LSS_CONVS_H
#define LSS_CONVS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { LSS_CONV_F32 = 0, LSS_CONV_BF16 = 1 };
enum { LSS_CONV_NCHW = 0, LSS_CONV_NHWC = 1 };
enum { LSS_ACT_NONE = 0, LSS_ACT_RELU = 1, LSS_ACT_SWISH = 2 };
enum { LSS_CONV_EINVAL = -1 };

/* y (N, C, Ho, Wo) = depthwise_conv(x (N, C, Hi, Wi), w) */
int lss_dwconv_fwd(const void* x, int32_t dtype, const float* w, int32_t N, int32_t C, int32_t Hi, int32_t Wi,
                   int32_t K, int32_t stride, int32_t pad_top, int32_t pad_left, int32_t Ho, int32_t Wo, void* y,
                   void* stream);

/* dx (N, C, Hi, Wi) = d loss / d x given dy (N, C, Ho, Wo); shapes and pads of the forward conv */
int lss_dwconv_bwd_data(const void* dy, int32_t dtype, const float* w, int32_t N, int32_t C, int32_t Hi, int32_t Wi,
                        int32_t K, int32_t stride, int32_t pad_top, int32_t pad_left, int32_t Ho, int32_t Wo, void* dx,
                        void* stream);

/* partial (C, ngroups, K*K) fp32: the weight gradient of images [N*q/ngroups, N*(q+1)/ngroups) in
 * slot q (1 <= ngroups <= N); the caller sums the groups (fixed order, deterministic). */
int lss_dwconv_bwd_weight(const void* x, const void* dy, int32_t dtype, int32_t N, int32_t C, int32_t Hi, int32_t Wi,
                          int32_t K, int32_t stride, int32_t pad_top, int32_t pad_left, int32_t Ho, int32_t Wo,
                          int32_t ngroups, float* partial, void* stream);
/* (ABI 23) lss_dwconv_bwd_weight that also folds the partials: the last of each channel's ngroups blocks
 * to finish sums them in group order into dw (C, K*K) fp32 -- no separate reduction launch. sync: the
 * batch-norm sync workspace (lss_bn_sync_words int32, zero-filled; left zero-filled), C <= 4096. */
int lss_dwconv_bwd_weight2(const void* x, const void* dy, int32_t dtype, int32_t N, int32_t C, int32_t Hi,
                           int32_t Wi, int32_t K, int32_t stride, int32_t pad_top, int32_t pad_left, int32_t Ho,
                           int32_t Wo, int32_t ngroups, float* partial, uint32_t* sync, float* dw, void* stream);

/* 1x1 convolution to one output channel (BevEncode's last conv, up2.4: 128 -> outC = 1,
 * src/models.py:115) over channels-last bf16 rows x (P, C), C % 8 == 0 and 64 % (C / 8) == 0:
 * y[r] = bf16(sum_c x[r, c] * w[c] + bias[0]) (fp32 accumulation; w holds the bf16-rounded weights
 * as fp32, as autocast's conv operands; bias is a device scalar, nullable). Backward: dx[r, c] = bf16(dy[r] * w[c]) and partial
 * (lss_head1_blocks(P), C + 1) fp32 = per block of rows, sum_r dy[r] * x[r, c] (columns 0..C-1) and
 * sum_r dy[r] (column C); the caller sums the blocks (fixed order). */
int lss_head1_blocks(int32_t P);
int lss_head1_fwd(const void* x, const float* w, const float* bias, int32_t P, int32_t C, void* y, void* stream);
int lss_head1_bwd(const void* x, const void* dy, const float* w, int32_t P, int32_t C, void* dx, float* partial,
                  void* stream);
/* (ABI 23) BevEncode's up2 tail -- BN + ReLU + the one-channel head -- without the normalised map:
 * lss_head1_fwd2 / lss_head1_bwd2 with bn_stats = the batch norm's saved (4, C) statistics (mean, rstd,
 * scale, shift; from lss_bn_fwd2 with y = NULL) read x as the batch norm's INPUT and use
 * bf16(relu(fmaf(x, scale, shift))) -- the value lss_bn_fwd's ReLU apply would have stored -- in its
 * place (bn_stats = NULL: lss_head1_fwd / lss_head1_bwd). lss_head1_bwd2 with dx = NULL writes no input
 * gradient (bn_stats required): lss_bn_bwd_rank1 takes it as bf16(dy[r] w[c]) itself. Bit-identical to
 * the unfused sequence (tests/test_gpu_convs.py). */
int lss_head1_fwd2(const void* x, const float* w, const float* bias, int32_t P, int32_t C, const float* bn_stats,
                   void* y, void* stream);
int lss_head1_bwd2(const void* x, const void* dy, const float* w, int32_t P, int32_t C, const float* bn_stats,
                   void* dx, float* partial, void* stream);

/* Weight gradient of a 1x1 convolution (no bias, stride 1) over NCHW contiguous bf16 activations:
 * dw (Cout, Cin) = sum over n < N, q < HW of dy[n][co][q] * x[n][ci][q], fp32 accumulation, written as
 * dw_dtype (LSS_CONV_BF16: rounded once; LSS_CONV_F32). HW % 4 == 0, 8-B aligned x / dy. workspace:
 * at least lss_pw_wrw_workspace_bytes(N, Cin, Cout, HW) bytes of device memory (per-split fp32
 * partials, summed in split order: deterministic). Two launches on the stream. */
int64_t lss_pw_wrw_workspace_bytes(int32_t N, int32_t Cin, int32_t Cout, int32_t HW);
int lss_pw_wrw(const void* x, const void* dy, int32_t N, int32_t Cin, int32_t Cout, int32_t HW, void* dw,
               int32_t dw_dtype, void* workspace, int64_t workspace_bytes, void* stream);

/* 1x1 convolution (no bias, stride 1) over NCHW contiguous bf16 activations, fp32 accumulation:
 * y[n][m][q] = bf16(sum_k A(m, k) * x[n][k][q]) for n < N, m < M, q < HW, with A(m, k) = a[m * K + k]
 * (LSS_PW_MK: the conv weight (M, K), the forward) or a[k * M + m] (LSS_PW_KM: the weight (K, M) read
 * transposed, the backward-data dx = W^T dy). HW % 4 == 0, K % 8 == 0, M % 8 == 0, 16-B aligned pointers. */
enum { LSS_PW_MK = 0, LSS_PW_KM = 1 };
int lss_pw_conv(const void* x, const void* a, int32_t a_layout, int32_t N, int32_t K, int32_t M, int32_t HW, void* y,
                void* stream);

/* Per-sample scale (+ residual) over N samples of `per` contiguous bf16 elements each (any memory
 * format that is sample-major: NCHW or channels-last), per % 8 == 0, 16-B aligned pointers:
 * y = bf16(x * scale[n] + res) (res nullable: y = bf16(x * scale[n])), scale[n] = mask[n] / keep with
 * mask[n] = floor(bf16(keep + u[n])), u the N bf16 uniform draws (torch.rand in the activations'
 * dtype), 0 < keep <= 1. The MBConv residual with stochastic depth (efficientnet_pytorch
 * drop_connect: inputs / keep_prob * floor(keep_prob + rand), then the skip add; the reference's
 * trunk, src/models.py:43) in one pass, the mask computed in the kernel; its backward is the
 * res == NULL form on the output gradient with the same draws. */
int lss_scale_add(const void* x, const void* u, float keep, const void* res, int64_t N, int64_t per, void* y,
                  void* stream);

/* (ABI 23) The weight of a stride-1, padding-(K-1)/2 transposed convolution as a forward one:
 * wt[i][o][a][b] = w[o][i][K-1-a][K-1-b], written channels-last ((I, O, K, K) with memory order
 * i, a, b, o). w is (O, I, K, K), NCHW (contiguous) or NHWC (channels-last) per w_layout; dtype fp32 or
 * bf16. dx = conv2d(dy, wt) is the backward-data of y = conv2d(x, w) (models._Conv3x3: MIOpen's forward
 * kernels instead of its backward-data ones). Replaces w.transpose(0, 1).flip(2, 3).contiguous(...),
 * two torch kernels. */
int lss_conv_flip_weight(const void* w, int32_t dtype, int32_t O, int32_t I, int32_t K, int32_t w_layout,
                         void* wt, void* stream);

/* Dropout (CamEncode.dropout = nn.Dropout(0.2), src/models.py:44, 53), training mode: y = x / keep where
 * a counter-based draw keeps the element (probability keep), else 0; n elements of dtype (fp32 or bf16)
 * in memory order (any memory format), n * sizeof(dtype) % 16 == 0, 16-B aligned. The mask is a pure
 * function of (*seed, element index) -- Philox4x32-10, key = the 64-bit seed (device memory, so a
 * captured graph draws a new one per replay), counter = (16-B vector index, block) -- so the backward is
 * the same call on dy with the same seed. Blocks write the tensor in 8 XCD-contiguous eighths (the
 * fused lift's layout) and, when `prefetch` is non-NULL, also read its `prefetch_bytes` (the lift's
 * packed depthnet weights) into every XCD's L2. */
int lss_dropout(const void* x, int32_t dtype, int64_t n, const uint64_t* seed, float keep, void* y,
                const void* prefetch, int64_t prefetch_bytes, void* stream);

/* SimpleLoss (src/tools.py:222-230: BCEWithLogitsLoss(pos_weight=[pos_weight]), reduction mean) and its
 * input gradient in one pass: loss[0] = mean over the n elements of
 *   (1 - t) x + (1 + (pw - 1) t) (log1p(exp(-|x|)) + max(-x, 0)),
 * grad = ((1 + (pw - 1) t) sigmoid(x) - pw t) / n (the gradient for d loss = 1; the caller scales it by
 * the incoming gradient). x, grad: n logits of dtype (fp32 or bf16), 16-B aligned; target: n fp32,
 * 16-B aligned; arithmetic fp32. partial: lss_bce_partials(n) fp32 scratch. Deterministic (fixed-order
 * sums). Two launches, no host synchronisation. */
int lss_bce_logits(const void* x, int32_t dtype, const float* target, int64_t n, float pos_weight, float* partial,
                   float* loss, void* grad, void* stream);
int64_t lss_bce_partials(int64_t n);
/* Backward of lss_bce_logits: dx = grad * grad_loss[0] (grad_loss: the loss's incoming gradient, one fp32
 * in device memory), computed in fp32 and rounded once to dtype; grad and dx 16-B aligned. */
int lss_bce_logits_bwd(const void* grad, int32_t dtype, int64_t n, const float* grad_loss, void* dx, void* stream);

/* out[c] = sum over (n, pixel) of x[n][c][pixel] (fp32, fixed order), x (N, C, HW) NCHW fp32 or bf16: the
 * bias gradient of the fused lift's depthnet conv (src/models.py:47) from d(logits). One launch. */
int lss_channel_sums(const void* x, int32_t dtype, int32_t N, int32_t C, int32_t HW, float* out, void* stream);

/* The training step's update (train_simbev.py:245-248): clip_grad_norm_(params, max_norm) fused with
 * torch.optim.Adam (L2 weight_decay added to the clipped gradient, no amsgrad) over `count` fp32 tensors
 * (params[k], grads[k], exp_avg[k], exp_avg_sq[k]: numel[k] elements each; step[k]: the tensor's
 * device-resident fp32 step count, advanced by one; all distinct). The clip factor is
 * min(max_norm / (||all grads||_2 + 1e-6), 1); the gradients are not modified. partial:
 * lss_clip_adam_partials() fp32 scratch. Two launches, no host synchronisation (graph-capturable);
 * deterministic. */
#define LSS_ADAM_MAX_TENSORS 32
int lss_clip_adam_partials(void);
int lss_clip_adam(int32_t count, float* const* params, const float* const* grads, float* const* exp_avg,
                  float* const* exp_avg_sq, float* const* step, const int64_t* numel, float max_norm, float lr,
                  float beta1, float beta2, float eps, float weight_decay, float* partial, void* stream);

/* Training-mode batch norm fused with an activation (and, for ReLU, a residual add), for
 * nn.BatchNorm2d followed by swish (EfficientNet-B0, src/models.py:68 and the MBConv blocks) or
 * ReLU (CamEncode.up1, BevEncode, src/models.py:15-34, 92-130):
 *   y = act(x * scale_c + shift_c [+ residual]),  scale_c = gamma_c / sqrt(var_c + eps),
 *   shift_c = beta_c - mean_c * scale_c, mean / biased var over (N, H, W); running_mean / running_var
 *   (nullable) updated with `momentum` and the unbiased variance, as nn.BatchNorm2d does.
 * x, residual, y: (N, C, H, W) with HW = H*W, NCHW or channels-last (LSS_CONV_NHWC: C a multiple
 * of 8 with 256 % (C / 8) == 0), element type dtype; gamma, beta and every statistic fp32.
 * partial: (C, ngroups, 2) fp32 scratch, ngroups from lss_bn_groups. save_mean, save_rstd, scale,
 * shift are the four rows of one (4, C) fp32 array (outputs kept for lss_bn_bwd).
 * num_batches_tracked (nullable): the module's int64 counter, incremented on the device (no
 * separate launch per BN layer). */
int lss_bn_groups(int32_t N, int32_t C, int32_t HW, int32_t layout);
int lss_bn_fwd(const void* x, const void* residual, int32_t dtype, int32_t layout, int32_t N, int32_t C, int32_t HW,
               const float* gamma, const float* beta, float eps, float momentum, float* running_mean,
               float* running_var, long long* num_batches_tracked, int32_t act, int32_t ngroups, float* partial,
               float* save_mean, float* save_rstd, float* scale, float* shift, void* y, void* stream);

/* Backward of lss_bn_fwd: dx (and dresidual = the gradient of the residual, nullable) of element
 * type dtype; dgamma, dbeta fp32 (nullable). y is the forward output (needed for ReLU). With
 * LSS_CONV_NHWC and a forward WITHOUT a residual, y may be NULL for ReLU: the kernels then recompute
 * it from x and the saved scale / shift exactly as the forward rounded it (one tensor read less).
 * coef: (C, 2) fp32 scratch. */
int lss_bn_bwd(const void* dy, const void* x, const void* y, int32_t dtype, int32_t layout, int32_t N, int32_t C,
               int32_t HW, const float* scale, const float* shift, const float* save_mean, const float* save_rstd,
               int32_t act, int32_t ngroups, float* partial, float* coef, float* dgamma, float* dbeta, void* dx,
               void* dresidual, void* stream);

/* lss_bn_fwd / lss_bn_bwd with a sync workspace (lss_bn_sync_words() uint32, zero-filled once; every
 * call leaves it zero-filled; one call at a time per workspace; NULL = the calls above). For NCHW bf16
 * maps with several groups per channel (lss_bn_groups > 1), statistics and apply then run in ONE launch:
 * the blocks of a channel hold their groups in registers and meet on the channel's counters in the
 * workspace (bounded waits; a block that gives up recomputes the statistics itself). Same outputs,
 * bit for bit. The workspace's last word overrides the wait bound (0: built in; s > 0: s - 1 polls). */
int lss_bn_sync_words(void);
int lss_bn_fwd2(const void* x, const void* residual, int32_t dtype, int32_t layout, int32_t N, int32_t C, int32_t HW,
                const float* gamma, const float* beta, float eps, float momentum, float* running_mean,
                float* running_var, long long* num_batches_tracked, int32_t act, int32_t ngroups, float* partial,
                float* save_mean, float* save_rstd, float* scale, float* shift, void* y, uint32_t* sync,
                void* stream);
int lss_bn_bwd2(const void* dy, const void* x, const void* y, int32_t dtype, int32_t layout, int32_t N, int32_t C,
                int32_t HW, const float* scale, const float* shift, const float* save_mean, const float* save_rstd,
                int32_t act, int32_t ngroups, float* partial, float* coef, float* dgamma, float* dbeta, void* dx,
                void* dresidual, uint32_t* sync, void* stream);
/* (ABI 23) NHWC bf16 batch-norm backward whose incoming gradient is the rank-1 product
 * dy[p][c] = bf16(g1[p] * w1[c]) (g1: N*HW bf16, w1: C fp32), computed in the kernels instead of read --
 * the gradient the one-channel head hands back (lss_head1_bwd2 with dx = NULL). Otherwise lss_bn_bwd's
 * NHWC path with y = NULL, no residual; act LSS_ACT_NONE or LSS_ACT_RELU. And lss_bn_fwd / lss_bn_fwd2
 * accept y = NULL for LSS_CONV_NHWC: statistics, saved stats and running stats only, no apply pass. */
int lss_bn_bwd_rank1(const void* g1, const float* w1, const void* x, int32_t N, int32_t C, int32_t HW,
                     const float* scale, const float* shift, const float* save_mean, const float* save_rstd,
                     int32_t act, int32_t ngroups, float* partial, float* coef, float* dgamma, float* dbeta, void* dx,
                     void* stream);

/* Bilinear upsampling with align_corners=True (nn.Upsample(mode="bilinear", align_corners=True),
 * src/models.py:19, 109) fused with Up's channel concatenation (torch.cat([x2, x1], 1),
 * src/models.py:33). All tensors channels-last bf16, 16-byte aligned, C1 and C2 multiples of 8,
 * upsampling only (Ho >= Hi > 1, Wo >= Wi > 1):
 *   y (N, Ho, Wo, C2 + C1) = cat([skip (N, Ho, Wo, C2), up(x (N, Hi, Wi, C1))]) -- skip may be NULL
 *   when C2 == 0; the blend is fp32 in PyTorch's order, rounded to bf16 once (the value the bf16
 *   autocast cast of the reference's fp32 upsample + cat produces). */
int lss_upsample_cat_fwd(const void* x, const void* skip, int32_t N, int32_t Hi, int32_t Wi, int32_t C1, int32_t C2,
                         int32_t Ho, int32_t Wo, void* y, void* stream);

/* dx (N, Hi, Wi, C1) bf16 = the upsample's backward applied to channels [C2, C2 + C1) of dy
 * (N, Ho, Wo, C2 + C1) bf16: a gather (each input element sums its weighted output gradients in
 * fp32, fixed order), no atomics. The skip's gradient is dy's first C2 channels (a view). */
int lss_upsample_bwd(const void* dy, int32_t N, int32_t Hi, int32_t Wi, int32_t C1, int32_t C2, int32_t Ho,
                     int32_t Wo, void* dx, void* stream);
/* (ABI 23) The same with chan_scale (nullable, N x C1 fp32): x's channel c of image n scaled by
 * chan_scale[n C1 + c] after the interpolation, and the input gradient by the same factor -- BevEncode's
 * Dropout2d (src/models.py:110: a per-(image, channel) 0 or 1 / (1 - p)) folded into up2's upsample. */
int lss_upsample_cat_fwd2(const void* x, const void* skip, int32_t N, int32_t Hi, int32_t Wi, int32_t C1, int32_t C2,
                          int32_t Ho, int32_t Wo, const float* chan_scale, void* y, void* stream);
int lss_upsample_bwd2(const void* dy, int32_t N, int32_t Hi, int32_t Wi, int32_t C1, int32_t C2, int32_t Ho,
                      int32_t Wo, const float* chan_scale, void* dx, void* stream);

/* Squeeze-and-excitation of an MBConv block (efficientnet_pytorch MBConvBlock, used by CamEncode's
 * trunk, src/models.py:43): y = x * sigmoid(W2 swish(W1 mean_hw(x) + b1) + b2), x / y (N, C, HW)
 * NCHW bf16 (HW % 4 == 0, C <= 2048, sq <= 64), W1 (sq, C), b1 (sq), W2 (C, sq), b2 (C) fp32
 * masters. Weights and values are rounded to bf16 where bf16 autocast rounds them (conv operands,
 * pooled map, both conv outputs, swish, sigmoid). Saved for the backward: m (N, C) pooled means, r / h (N, sq) reduce-conv output and
 * its swish, sig (N, C); all fp32 buffers. */
int lss_se_fwd(const void* x, int32_t N, int32_t C, int32_t HW, const float* w1, const float* b1, const float* w2,
               const float* b2, int32_t sq, float* m, float* r, float* h, float* sig, void* y, void* stream);

/* Backward: dx (bf16) = dy * sig + dm / HW (the excitation and the pooling paths), and the
 * per-image gradients the caller turns into parameter gradients with small GEMMs: de (N, C) =
 * d(expand-conv output), dr (N, sq) = d(reduce-conv output), dm (N, C) = d(pooled means).
 * Scratch: t (N, C) fp32 (sum over HW of dy * x), dh_part (N, ceil(C / 64), sq) fp32. */
int lss_se_bwd(const void* dy, const void* x, int32_t N, int32_t C, int32_t HW, const float* w1, const float* w2,
               int32_t sq, const float* r, const float* sig, float* t, float* dh_part, float* de, float* dr, float* dm,
               void* dx, void* stream);

/* The SE convs' parameter gradients from the backward's per-image values, in one launch (fp32, the N
 * images summed in order): dw1 (sq, C) = dr^T m, db1 (sq) = sum_n dr, dw2 (C, sq) = de^T h,
 * db2 (C) = sum_n de. */
int lss_se_wgrad(const float* de, const float* h, const float* dr, const float* m, int32_t N, int32_t C, int32_t sq,
                 float* dw1, float* db1, float* dw2, float* db2, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* LSS_CONVS_H */

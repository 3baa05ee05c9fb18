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

#ifdef __cplusplus
}
#endif
#endif /* LSS_CONVS_H */

// lss_resample.hip -- the Up stages' bilinear upsampling (nn.Upsample(mode="bilinear",
// align_corners=True), src/models.py:19, 109) fused with the channel concatenation that follows it
// (Up.forward: torch.cat([x2, x1], dim=1), src/models.py:33), for channels-last bf16 maps.
//
// Under bf16 autocast the reference runs the upsample in fp32 (an fp32-listed op), concatenates in
// fp32 and casts back to bf16 for the next conv: at config 3 BevEncode.up2 alone materialises a
// 327 MB fp32 map and a 164 MB bf16 copy of it, and PyTorch's backward scatters with fp32 atomics
// (0.6 ms per launch). Here the forward blends in fp32 and writes the bf16 concatenation directly
// (the same values the cast produces), and the backward is a gather: each thread owns one input
// pixel x 8 channels and sums, in fp32, the weighted bf16 output gradients of the output pixels whose
// 2 x 2 stencil touches it -- no atomics, deterministic, every input gradient written once.
//
// Layout: x (N, Hi, Wi, C1), skip (N, Ho, Wo, C2), y / dy (N, Ho, Wo, C2 + C1), all channels-last
// bf16 with C1, C2 multiples of 8: a thread moves 8 channels (16 bytes) per access, and the lanes of
// a wave cover consecutive channel octets of one pixel, so every wave access is contiguous.

#include <hip/hip_runtime.h>
#include <limits.h>
#include <math.h>
#include <stdint.h>

#include "lss_convs.h"

// The library is built with -ffp-contract=off for the geometry's reference op order (lss_hip.hip);
// the conv-stack kernels here have no bit-exact contract, so they keep FMA contraction.
#pragma clang fp contract(fast)

namespace {

using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
constexpr int kBlock = 256;

struct UpGeo {
    int N, Hi, Wi, C1, C2, Ho, Wo;
    float rh, rw;  // (in - 1) / (out - 1) in fp32, as PyTorch's area_pixel_compute_scale (align_corners)
};

__device__ __forceinline__ void unpack8(u32x4 v, float f[8]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        f[2 * k] = __uint_as_float(v[k] << 16);
        f[2 * k + 1] = __uint_as_float(v[k] & 0xffff0000u);
    }
}

// fp32 -> bf16 bits, round to nearest even (c10::BFloat16's rounding; NaN kept quiet)
__device__ __forceinline__ unsigned bf16_bits(float x) {
    unsigned u = __float_as_uint(x);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (u >> 16) | 0x40u;
    u += 0x7fffu + ((u >> 16) & 1u);
    return u >> 16;
}

__device__ __forceinline__ u32x4 pack8(const float f[8]) {
    u32x4 v;
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = bf16_bits(f[2 * k]) | (bf16_bits(f[2 * k + 1]) << 16);
    return v;
}

// source row/column of output index o: i0 = trunc(r * o), step ip (0 on the last input line),
// fraction l1 (PyTorch's area_pixel_compute_source_index with align_corners=True)
struct Src {
    int i0, ip;
    float l1;
};
__device__ __forceinline__ Src source(float r, int o, int in) {
    const float s = r * (float)o;
    Src q;
    q.i0 = (int)s;
    q.ip = q.i0 < in - 1 ? 1 : 0;
    q.l1 = s - (float)q.i0;
    return q;
}

// weight of input line i in the stencil of output line o (0 if untouched)
__device__ __forceinline__ float line_weight(float r, int o, int in, int i) {
    const Src q = source(r, o, in);
    float w = 0.f;
    if (q.i0 == i) w += 1.f - q.l1;
    if (q.i0 + q.ip == i) w += q.l1;
    return w;
}

// cs (nullable): a per-(image, channel) scale of x's channels (N x C1 fp32): BevEncode's Dropout2d mask
// (src/models.py:110), applied to the interpolated values (and to the input gradient in the backward)
__global__ __launch_bounds__(kBlock) void k_up_cat_fwd(const u32x4* __restrict__ x, const u32x4* __restrict__ skip,
                                                       UpGeo g, u32x4* __restrict__ y, const float* __restrict__ cs) {
    const int c8s = g.C2 >> 3, c81 = g.C1 >> 3, c8t = c8s + c81;
    const int total = g.N * g.Ho * g.Wo * c8t;
    const int t = blockIdx.x * kBlock + threadIdx.x;
    if (t >= total) return;
    const int c8 = t % c8t;
    const int pix = t / c8t;
    if (c8 < c8s) {
        y[t] = skip[pix * c8s + c8];
        return;
    }
    const int ow = pix % g.Wo;
    const int r = pix / g.Wo;
    const int oh = r % g.Ho;
    const int n = r / g.Ho;
    const Src h = source(g.rh, oh, g.Hi), w = source(g.rw, ow, g.Wi);
    const float h1l = h.l1, h0l = 1.f - h.l1, w1l = w.l1, w0l = 1.f - w.l1;
    const u32x4* xb = x + (n * g.Hi * g.Wi) * c81 + (c8 - c8s);
    const int r0 = h.i0 * g.Wi, r1 = (h.i0 + h.ip) * g.Wi;
    float a[8], b[8], c[8], d[8], o[8];
    unpack8(xb[(r0 + w.i0) * c81], a);
    unpack8(xb[(r0 + w.i0 + w.ip) * c81], b);
    unpack8(xb[(r1 + w.i0) * c81], c);
    unpack8(xb[(r1 + w.i0 + w.ip) * c81], d);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = h0l * (w0l * a[k] + w1l * b[k]) + h1l * (w0l * c[k] + w1l * d[k]);
    if (cs) {
        const float* m = cs + (size_t)n * g.C1 + (c8 - c8s) * 8;
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] *= m[k];
    }
    y[t] = pack8(o);
}

// candidate output lines whose stencil can touch input line i: trunc(r * o) in {i - 1, i}
__device__ __forceinline__ void out_range(float r, int i, int out, int& lo, int& hi) {
    lo = max(0, (int)floorf((float)(i - 1) / r) - 1);
    hi = min(out - 1, (int)ceilf((float)(i + 1) / r) + 1);
}

// d x of input pixel (i, j) from every output pixel whose stencil touches it, nonzero weights only,
// output rows then columns ascending (k_up_bwd's order; k_up_bwd_taps adds the same terms in the same order)
__device__ __forceinline__ void up_bwd_sum(const u32x4* __restrict__ db, const UpGeo& g, int i, int j, int oh0,
                                           int oh1, int ow0, int ow1, int c8t, float acc[8]) {
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = 0.f;
    for (int oh = oh0; oh <= oh1; ++oh) {
        const float wy = line_weight(g.rh, oh, g.Hi, i);
        if (wy == 0.f) continue;
        for (int ow = ow0; ow <= ow1; ++ow) {
            const float wx = line_weight(g.rw, ow, g.Wi, j);
            if (wx == 0.f) continue;
            const float wgt = wy * wx;
            float v[8];
            unpack8(db[(oh * g.Wo + ow) * c8t], v);
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[k] += wgt * v[k];
        }
    }
}

__device__ __forceinline__ void up_scale(const float* __restrict__ cs, const UpGeo& g, int n, int c8, float acc[8]) {
    if (!cs) return;
    const float* m = cs + (size_t)n * g.C1 + c8 * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] *= m[k];
}

__global__ __launch_bounds__(kBlock) void k_up_bwd(const u32x4* __restrict__ dy, UpGeo g, u32x4* __restrict__ dx,
                                                   const float* __restrict__ cs) {
    const int c8s = g.C2 >> 3, c81 = g.C1 >> 3, c8t = c8s + c81;
    const int total = g.N * g.Hi * g.Wi * c81;
    const int t = blockIdx.x * kBlock + threadIdx.x;
    if (t >= total) return;
    const int c8 = t % c81;
    const int pix = t / c81;
    const int j = pix % g.Wi;
    const int r = pix / g.Wi;
    const int i = r % g.Hi;
    const int n = r / g.Hi;
    int oh0, oh1, ow0, ow1;
    out_range(g.rh, i, g.Ho, oh0, oh1);
    out_range(g.rw, j, g.Wo, ow0, ow1);
    float acc[8];
    up_bwd_sum(dy + (n * g.Ho * g.Wo) * c8t + c8s + c8, g, i, j, oh0, oh1, ow0, ow1, c8t, acc);
    up_scale(cs, g, n, c8, acc);
    dx[t] = pack8(acc);
}

// k_up_bwd with every load of an output row's taps in flight: the output lines with a nonzero weight
// for this input line / column are listed first (at most T per axis: T >= 2 / r + 1), then each output
// row's T loads are issued unconditionally (clamped addresses, weight 0 past the list) before they are
// summed -- the loop above waits for each load behind a data-dependent branch. Same order of the
// nonzero terms (a zero-weight term adds 0), so the same bits for finite values.
#ifndef LSS_UP_BWD_V2
#define LSS_UP_BWD_V2 1
#endif
template <int T>
__global__ __launch_bounds__(kBlock) void k_up_bwd_taps(const u32x4* __restrict__ dy, UpGeo g, u32x4* __restrict__ dx,
                                                        const float* __restrict__ cs) {
    const int c8s = g.C2 >> 3, c81 = g.C1 >> 3, c8t = c8s + c81;
    const int total = g.N * g.Hi * g.Wi * c81;
    const int t = blockIdx.x * kBlock + threadIdx.x;
    if (t >= total) return;
    const int c8 = t % c81;
    const int pix = t / c81;
    const int j = pix % g.Wi;
    const int r = pix / g.Wi;
    const int i = r % g.Hi;
    const int n = r / g.Hi;
    int oh0, oh1, ow0, ow1;
    out_range(g.rh, i, g.Ho, oh0, oh1);
    out_range(g.rw, j, g.Wo, ow0, ow1);
    int hl[T], wl[T];
    float hw[T], ww[T];
    int nh = 0, nw = 0;
#pragma unroll
    for (int q = 0; q < T; ++q) {
        hl[q] = oh0; hw[q] = 0.f;
        wl[q] = ow0; ww[q] = 0.f;
    }
    for (int oh = oh0; oh <= oh1; ++oh) {
        const float wy = line_weight(g.rh, oh, g.Hi, i);
        if (wy != 0.f) {
#pragma unroll
            for (int q = 0; q < T; ++q)
                if (q == nh) { hl[q] = oh; hw[q] = wy; }
            ++nh;
        }
    }
    for (int ow = ow0; ow <= ow1; ++ow) {
        const float wx = line_weight(g.rw, ow, g.Wi, j);
        if (wx != 0.f) {
#pragma unroll
            for (int q = 0; q < T; ++q)
                if (q == nw) { wl[q] = ow; ww[q] = wx; }
            ++nw;
        }
    }
    float acc[8];
    const u32x4* db = dy + (n * g.Ho * g.Wo) * c8t + c8s + c8;
    if (nh > T || nw > T) {
        // more nonzero lines than the host's bound allowed for (float rounding of r * o): the plain
        // loop, same terms in the same order -- never a dropped tap
        up_bwd_sum(db, g, i, j, oh0, oh1, ow0, ow1, c8t, acc);
        up_scale(cs, g, n, c8, acc);
        dx[t] = pack8(acc);
        return;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = 0.f;
    for (int a = 0; a < nh; ++a) {
        int row = 0;
        float wy = 0.f;
#pragma unroll
        for (int q = 0; q < T; ++q)
            if (q == a) { row = hl[q]; wy = hw[q]; }
        u32x4 v[T];
#pragma unroll
        for (int b = 0; b < T; ++b) v[b] = db[(row * g.Wo + wl[b]) * c8t];
#pragma unroll
        for (int b = 0; b < T; ++b) {
            if (b < nw) {
                float f[8];
                unpack8(v[b], f);
                const float wgt = wy * ww[b];
#pragma unroll
                for (int k = 0; k < 8; ++k) acc[k] += wgt * f[k];
            }
        }
    }
    up_scale(cs, g, n, c8, acc);
    dx[t] = pack8(acc);
}

inline int launch_status() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

inline bool up_ok(int N, int Hi, int Wi, int C1, int C2, int Ho, int Wo) {
    // upsampling only (Ho >= Hi, Wo >= Wi), > 1 line on both sides (align_corners scale defined)
    return N > 0 && Hi > 1 && Wi > 1 && Ho >= Hi && Wo >= Wi && C1 > 0 && C1 % 8 == 0 && C2 >= 0 &&
           C2 % 8 == 0 && (long)N * Ho * Wo * (C1 + C2) / 8 < INT_MAX - kBlock &&
           (long)N * Hi * Wi * (C1 + C2) < INT_MAX;
}

inline bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

UpGeo make_geo(int N, int Hi, int Wi, int C1, int C2, int Ho, int Wo) {
    UpGeo g;
    g.N = N; g.Hi = Hi; g.Wi = Wi; g.C1 = C1; g.C2 = C2; g.Ho = Ho; g.Wo = Wo;
    g.rh = (float)(Hi - 1) / (float)(Ho - 1);
    g.rw = (float)(Wi - 1) / (float)(Wo - 1);
    return g;
}

}  // namespace

extern "C" {

int lss_upsample_cat_fwd(const void* x, const void* skip, int32_t N, int32_t Hi, int32_t Wi, int32_t C1, int32_t C2,
                         int32_t Ho, int32_t Wo, void* y, void* stream) {
    return lss_upsample_cat_fwd2(x, skip, N, Hi, Wi, C1, C2, Ho, Wo, nullptr, y, stream);
}

int lss_upsample_cat_fwd2(const void* x, const void* skip, int32_t N, int32_t Hi, int32_t Wi, int32_t C1, int32_t C2,
                          int32_t Ho, int32_t Wo, const float* chan_scale, void* y, void* stream) {
    if (!x || !y || !up_ok(N, Hi, Wi, C1, C2, Ho, Wo) || (C2 > 0 && !skip)) return LSS_CONV_EINVAL;
    if (!aligned16(x) || !aligned16(y) || (C2 > 0 && !aligned16(skip))) return LSS_CONV_EINVAL;
    const UpGeo g = make_geo(N, Hi, Wi, C1, C2, Ho, Wo);
    const int total = N * Ho * Wo * ((C1 + C2) / 8);
    hipLaunchKernelGGL(k_up_cat_fwd, dim3((total + kBlock - 1) / kBlock), dim3(kBlock), 0, (hipStream_t)stream,
                       (const u32x4*)x, (const u32x4*)skip, g, (u32x4*)y, chan_scale);
    return launch_status();
}

int lss_upsample_bwd(const void* dy, int32_t N, int32_t Hi, int32_t Wi, int32_t C1, int32_t C2, int32_t Ho,
                     int32_t Wo, void* dx, void* stream) {
    return lss_upsample_bwd2(dy, N, Hi, Wi, C1, C2, Ho, Wo, nullptr, dx, stream);
}

int lss_upsample_bwd2(const void* dy, int32_t N, int32_t Hi, int32_t Wi, int32_t C1, int32_t C2, int32_t Ho,
                      int32_t Wo, const float* chan_scale, void* dx, void* stream) {
    if (!dy || !dx || !up_ok(N, Hi, Wi, C1, C2, Ho, Wo) || !aligned16(dy) || !aligned16(dx)) return LSS_CONV_EINVAL;
    const UpGeo g = make_geo(N, Hi, Wi, C1, C2, Ho, Wo);
    const int total = N * Hi * Wi * (C1 / 8);
    // output lines with a nonzero weight per input line: those with r * o in (i - 1, i + 1), <= 2 / r + 1
    const int need = (int)(2.f / fminf(g.rh, g.rw)) + 2;
    const dim3 gr((total + kBlock - 1) / kBlock), bl(kBlock);
    if (LSS_UP_BWD_V2 && need <= 6)
        hipLaunchKernelGGL(k_up_bwd_taps<6>, gr, bl, 0, (hipStream_t)stream,
                       (const u32x4*)dy, g, (u32x4*)dx, chan_scale);
    else if (LSS_UP_BWD_V2 && need <= 10)
        hipLaunchKernelGGL(k_up_bwd_taps<10>, gr, bl, 0, (hipStream_t)stream,
                       (const u32x4*)dy, g, (u32x4*)dx, chan_scale);
    else
        hipLaunchKernelGGL(k_up_bwd, gr, bl, 0, (hipStream_t)stream,
                       (const u32x4*)dy, g, (u32x4*)dx, chan_scale);
    return launch_status();
}

}  // extern "C"

// lss_se.hip -- squeeze-and-excitation of the EfficientNet-B0 MBConv blocks (efficientnet_pytorch
// MBConvBlock: x * sigmoid(se_expand(swish(se_reduce(avg_pool(x))))), used by CamEncode's trunk,
// src/models.py:43, 63-84), NCHW bf16 activations as the trunk runs under bf16 autocast.
//
// PyTorch runs it as ~7 forward and ~20 backward launches per block (pooling, two 1x1 convs on
// 1x1 maps with MIOpen's set/cast kernels, swish, sigmoid, the broadcast multiply, its two-sided
// backward with a materialised g*x, the pooling backward and a gradient add). Here:
//   forward   k_se_mean (one wave per (n, c) plane) -> k_se_mlp1 / k_se_mlp2 (both 1x1 convs,
//             swish, sigmoid; values rounded to bf16 where autocast rounds them) ->
//             k_se_scale (y = x * sig)
//   backward  k_se_dot (t = sum_hw g*x per plane) -> k_se_mlpb1 / k_se_mlpb2 (sigmoid, expand,
//             swish, reduce backward -> de, dr, dm) -> k_se_dx (dx = g*sig + dm/HW);
//             k_se_wgrad: the four weight / bias gradients in one launch.
// All sums fp32 in a fixed order (deterministic).

#include <hip/hip_runtime.h>
#include <limits.h>
#include <math.h>
#include <stdint.h>

#include "lss_convs.h"

// The library is built with -ffp-contract=off for the geometry's reference op order (lss_hip.hip);
// the conv-stack kernels here have no bit-exact contract, so they keep FMA contraction.
#pragma clang fp contract(fast)

namespace {

constexpr int kBlock = 256;
constexpr int kWave = 64;
constexpr int kMaxC = 2048;  // channels of the widest MBConv block: 1152

__device__ __forceinline__ float bf(unsigned short b) { return __uint_as_float((unsigned)b << 16); }
// fp32 -> bf16 bits, round to nearest even (NaN kept quiet)
__device__ __forceinline__ unsigned short bfbits(float x) {
    unsigned u = __float_as_uint(x);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (unsigned short)((u >> 16) | 0x40u);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (unsigned short)(u >> 16);
}
__device__ __forceinline__ float rbf(float x) { return bf(bfbits(x)); }  // round through bf16
__device__ __forceinline__ float sigm(float z) { return 1.f / (1.f + __expf(-z)); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}

// 4 consecutive bf16 (8 bytes) <-> fp32
__device__ __forceinline__ void ld4(const unsigned short* p, float* o) {
    const uint2 u = *reinterpret_cast<const uint2*>(p);
    o[0] = __uint_as_float(u.x << 16); o[1] = __uint_as_float(u.x & 0xffff0000u);
    o[2] = __uint_as_float(u.y << 16); o[3] = __uint_as_float(u.y & 0xffff0000u);
}
__device__ __forceinline__ void st4(unsigned short* p, const float* v) {
    uint2 u;
    u.x = (unsigned)bfbits(v[0]) | ((unsigned)bfbits(v[1]) << 16);
    u.y = (unsigned)bfbits(v[2]) | ((unsigned)bfbits(v[3]) << 16);
    *reinterpret_cast<uint2*>(p) = u;
}

// one wave per (n, c) plane of HW elements (HW % 4 == 0): mean, rounded to bf16 (the pooled map's type)
__global__ __launch_bounds__(kBlock) void k_se_mean(const unsigned short* __restrict__ x, int planes, int HW,
                                                    float* __restrict__ m) {
    const int pl = blockIdx.x * (kBlock / kWave) + (int)(threadIdx.x >> 6);
    if (pl >= planes) return;
    const int lane = threadIdx.x & 63;
    const unsigned short* xp = x + (size_t)pl * HW;
    float s = 0.f;
    for (int i = lane * 4; i < HW; i += kWave * 4) {
        float v[4];
        ld4(xp + i, v);
        s += (v[0] + v[1]) + (v[2] + v[3]);
    }
    s = wave_sum(s);
    if (lane == 0) m[pl] = rbf(s / (float)HW);
}

// The two 1x1 convs on the pooled (N, C) map, split so that every weight read is coalesced:
//   k_se_mlp1: one block per image, waves over the sq outputs, lanes over C (rows of W1 (sq, C)):
//              r = bf16(W1 m + b1), h = bf16(swish(r))
//   k_se_mlp2: one block per (image, 256 channels), the block's rows of W2 (C, sq) staged in LDS:
//              e = bf16(W2 h + b2), sig = bf16(sigmoid(e))
// Weights are fp32 masters, used rounded to bf16 as the autocast conv uses them.
constexpr int kMlpC = 256;  // channels per k_se_mlp2 / k_se_mlpb2 block
constexpr int kMlpbC = 64;  // channels per k_se_mlpb1 block (16 per wave: short dependent chains)
constexpr int kMaxSq = kWave;

__global__ __launch_bounds__(kBlock) void k_se_mlp1(const float* __restrict__ m, const float* __restrict__ w1,
                                                    const float* __restrict__ b1, int C, int sq,
                                                    float* __restrict__ r_out, float* __restrict__ h_out) {
    // one wave per (image, output j); four independent partial sums keep four loads in flight
    const int wpi = (sq + 3) / 4;  // blocks per image
    const int n = blockIdx.x / wpi, j = (blockIdx.x % wpi) * 4 + (int)(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (j >= sq) return;
    const float* mn = m + (size_t)n * C;
    const float* wr = w1 + (size_t)j * C;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int c = lane;
    for (; c + 3 * kWave < C; c += 4 * kWave) {
        a0 = fmaf(rbf(wr[c]), mn[c], a0);
        a1 = fmaf(rbf(wr[c + kWave]), mn[c + kWave], a1);
        a2 = fmaf(rbf(wr[c + 2 * kWave]), mn[c + 2 * kWave], a2);
        a3 = fmaf(rbf(wr[c + 3 * kWave]), mn[c + 3 * kWave], a3);
    }
    for (; c < C; c += kWave) a0 = fmaf(rbf(wr[c]), mn[c], a0);
    const float a = wave_sum((a0 + a1) + (a2 + a3));
    if (lane == 0) {
        const float r = rbf(a + rbf(b1[j]));
        r_out[(size_t)n * sq + j] = r;
        h_out[(size_t)n * sq + j] = rbf(r * sigm(r));
    }
}

__global__ __launch_bounds__(kBlock) void k_se_mlp2(const float* __restrict__ h, const float* __restrict__ w2,
                                                    const float* __restrict__ b2, int C, int sq,
                                                    float* __restrict__ sig) {
    __shared__ float s_w[kMlpC * (kMaxSq + 1)];  // rows of W2, padded
    __shared__ float s_h[kMaxSq];
    const int nchunk = (C + kMlpC - 1) / kMlpC;
    const int n = blockIdx.x / nchunk, c0 = (blockIdx.x % nchunk) * kMlpC;
    const int nc = min(kMlpC, C - c0);
    for (int i = threadIdx.x; i < nc * sq; i += kBlock) {
        const int cl = i / sq, j = i - cl * sq;
        s_w[cl * (sq + 1) + j] = rbf(w2[(size_t)c0 * sq + i]);
    }
    if ((int)threadIdx.x < sq) s_h[threadIdx.x] = h[(size_t)n * sq + threadIdx.x];
    __syncthreads();
    if ((int)threadIdx.x < nc) {
        const int c = c0 + threadIdx.x;
        const float* wr = s_w + threadIdx.x * (sq + 1);
        float e = 0.f;
        for (int j = 0; j < sq; ++j) e = fmaf(wr[j], s_h[j], e);
        e = rbf(e + rbf(b2[c]));
        sig[(size_t)n * C + c] = rbf(sigm(e));
    }
}

// y = bf16(x * sig[plane]), 4 elements per thread
__global__ __launch_bounds__(kBlock) void k_se_scale(const unsigned short* __restrict__ x,
                                                     const float* __restrict__ sig, int HW, int n4,
                                                     unsigned short* __restrict__ y) {
    const int t = blockIdx.x * kBlock + threadIdx.x;
    if (t >= n4) return;
    const int i = t * 4;
    const float s = sig[i / HW];
    float v[4];
    ld4(x + i, v);
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] *= s;
    st4(y + i, v);
}

// t[plane] = sum_hw g * x (fp32), one wave per plane
__global__ __launch_bounds__(kBlock) void k_se_dot(const unsigned short* __restrict__ g,
                                                   const unsigned short* __restrict__ x, int planes, int HW,
                                                   float* __restrict__ t) {
    const int pl = blockIdx.x * (kBlock / kWave) + (int)(threadIdx.x >> 6);
    if (pl >= planes) return;
    const int lane = threadIdx.x & 63;
    const size_t off = (size_t)pl * HW;
    float s = 0.f;
    for (int i = lane * 4; i < HW; i += kWave * 4) {
        float a[4], b[4];
        ld4(g + off + i, a);
        ld4(x + off + i, b);
#pragma unroll
        for (int k = 0; k < 4; ++k) s = fmaf(a[k], b[k], s);
    }
    s = wave_sum(s);
    if (lane == 0) t[pl] = s;
}

// MLP backward, coalesced like the forward, one block per (image, 64 channels):
//   k_se_mlpb1: de = t sig (1 - sig) for the block's channels; partial dh = W2^T de over them
//               (waves over 64-channel ranges, lanes over j = rows of W2; wave order fixed)
//   k_se_mlpb2: dh = sum of the image's partials (chunk order), dr = dh swish'(r) (the first block
//               of an image stores it), dm = W1^T dr for the block's 64 channels (lanes over C)
__global__ __launch_bounds__(kBlock) void k_se_mlpb1(const float* __restrict__ t, const float* __restrict__ sig,
                                                     const float* __restrict__ w2, int C, int sq,
                                                     float* __restrict__ de, float* __restrict__ dh_part) {
    __shared__ float s_de[kMlpbC];
    __shared__ float s_part[kBlock / kWave][kMaxSq];
    const int nchunk = (C + kMlpbC - 1) / kMlpbC;
    const int n = blockIdx.x / nchunk, k = blockIdx.x % nchunk, c0 = k * kMlpbC;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if ((int)threadIdx.x < kMlpbC) {
        const int c = c0 + (int)threadIdx.x;
        float d = 0.f;
        if (c < C) {
            const float s = sig[(size_t)n * C + c];
            d = t[(size_t)n * C + c] * s * (1.f - s);
            de[(size_t)n * C + c] = d;
        }
        s_de[threadIdx.x] = d;
    }
    __syncthreads();
    constexpr int kPer = kMlpbC / (kBlock / kWave);
    float a[kPer];
    const int cb = wave * kPer;
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
        const int ca = c0 + cb + i;
        a[i] = (lane < sq && ca < C) ? rbf(w2[(size_t)ca * sq + lane]) * s_de[cb + i] : 0.f;
    }
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < kPer; ++i) sum += a[i];
    s_part[wave][lane] = sum;
    __syncthreads();
    if ((int)threadIdx.x < sq) {
        const int j = threadIdx.x;
        dh_part[((size_t)n * nchunk + k) * sq + j] = (s_part[0][j] + s_part[1][j]) + (s_part[2][j] + s_part[3][j]);
    }
}

__global__ __launch_bounds__(kBlock) void k_se_mlpb2(const float* __restrict__ dh_part, const float* __restrict__ r,
                                                     const float* __restrict__ w1, int C, int sq,
                                                     float* __restrict__ dr, float* __restrict__ dm) {
    __shared__ float s_dr[kMaxSq];
    __shared__ float s_acc[kBlock / kWave][kWave];
    const int nchunk = (C + kMlpbC - 1) / kMlpbC, npart = nchunk;
    const int n = blockIdx.x / nchunk, k = blockIdx.x % nchunk;
    if ((int)threadIdx.x < sq) {
        const int j = threadIdx.x;
        float dh = 0.f;
        for (int q = 0; q < npart; ++q) dh += dh_part[((size_t)n * npart + q) * sq + j];
        const float rv = r[(size_t)n * sq + j];
        const float s = sigm(rv);
        const float d = dh * s * (1.f + rv * (1.f - s));
        s_dr[j] = d;
        if (k == 0) dr[(size_t)n * sq + j] = d;
    }
    __syncthreads();
    // 64 channels per block: lane = channel, wave w sums the j in [w sq / 4, (w+1) sq / 4); waves
    // combined in order
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int c = k * kMlpbC + lane;
    const int j0 = wave * sq / 4, j1 = (wave + 1) * sq / 4;
    float a = 0.f;
    if (c < C)
        for (int j = j0; j < j1; ++j) a = fmaf(rbf(w1[(size_t)j * C + c]), s_dr[j], a);
    s_acc[wave][lane] = a;
    __syncthreads();
    if (wave == 0 && c < C)
        dm[(size_t)n * C + c] = (s_acc[0][lane] + s_acc[1][lane]) + (s_acc[2][lane] + s_acc[3][lane]);
}

// dx = bf16(g * sig + dm / HW), 4 elements per thread
__global__ __launch_bounds__(kBlock) void k_se_dx(const unsigned short* __restrict__ g, const float* __restrict__ sig,
                                                  const float* __restrict__ dm, int HW, int n4,
                                                  unsigned short* __restrict__ dx) {
    const int t = blockIdx.x * kBlock + threadIdx.x;
    if (t >= n4) return;
    const int i = t * 4;
    const int pl = i / HW;
    const float s = sig[pl], b = dm[pl] / (float)HW;
    float v[4];
    ld4(g + i, v);
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = fmaf(v[k], s, b);
    st4(dx + i, v);
}

// The four parameter gradients of the two 1x1 convs in one launch, one thread per output, the N
// images summed in order (deterministic; the loops unrolled so 16 images' loads are in flight at once,
// the sums still one dependent chain in image order): dw2[c][j] = sum_n de[n][c] h[n][j] (C, sq),
// dw1[j][c] = sum_n dr[n][j] m[n][c] (sq, C), db1[j] = sum_n dr[n][j], db2[c] = sum_n de[n][c].
__global__ __launch_bounds__(kBlock) void k_se_wgrad(const float* __restrict__ de, const float* __restrict__ h,
                                                     const float* __restrict__ dr, const float* __restrict__ m,
                                                     int N, int C, int sq, float* __restrict__ dw1,
                                                     float* __restrict__ db1, float* __restrict__ dw2,
                                                     float* __restrict__ db2) {
    const int t = blockIdx.x * kBlock + threadIdx.x;
    const int cs = C * sq;
    float a = 0.f;
    if (t < cs) {  // dw2, lanes over j: de broadcast, h coalesced
        const int c = t / sq, j = t - c * sq;
#pragma unroll 16
        for (int n = 0; n < N; ++n) a = fmaf(de[(size_t)n * C + c], h[(size_t)n * sq + j], a);
        dw2[t] = a;
    } else if (t < 2 * cs) {  // dw1, lanes over c: m coalesced
        const int u = t - cs, j = u / C, c = u - j * C;
#pragma unroll 16
        for (int n = 0; n < N; ++n) a = fmaf(dr[(size_t)n * sq + j], m[(size_t)n * C + c], a);
        dw1[u] = a;
    } else if (t < 2 * cs + sq) {
        const int j = t - 2 * cs;
#pragma unroll 16
        for (int n = 0; n < N; ++n) a += dr[(size_t)n * sq + j];
        db1[j] = a;
    } else if (t < 2 * cs + sq + C) {
        const int c = t - 2 * cs - sq;
#pragma unroll 16
        for (int n = 0; n < N; ++n) a += de[(size_t)n * C + c];
        db2[c] = a;
    }
}

inline int launch_status() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

inline bool se_ok(int N, int C, int HW, int sq) {
    return N > 0 && C > 0 && C <= kMaxC && sq > 0 && sq <= kWave && HW > 0 && HW % 4 == 0 &&
           (long)N * C * HW < INT_MAX;
}

inline int blocks(long n, int per) { return (int)((n + per - 1) / per); }

}  // namespace

extern "C" {

int lss_se_fwd(const void* x, int32_t N, int32_t C, int32_t HW, const float* w1, const float* b1, const float* w2,
               const float* b2, int32_t sq, float* m, float* r, float* h, float* sig, void* y, void* stream) {
    if (!x || !w1 || !b1 || !w2 || !b2 || !m || !r || !h || !sig || !y || !se_ok(N, C, HW, sq)) return LSS_CONV_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    const int planes = N * C, n4 = planes * HW / 4;
    hipLaunchKernelGGL(k_se_mean, dim3(blocks(planes, kBlock / kWave)), dim3(kBlock), 0, s,
                       (const unsigned short*)x, planes, HW, m);
    const int nchunk = (C + kMlpC - 1) / kMlpC;
    hipLaunchKernelGGL(k_se_mlp1, dim3(N * ((sq + 3) / 4)), dim3(kBlock), 0, s, m, w1, b1, C, sq, r, h);
    hipLaunchKernelGGL(k_se_mlp2, dim3(N * nchunk), dim3(kBlock), 0, s, h, w2, b2, C, sq, sig);
    hipLaunchKernelGGL(k_se_scale, dim3(blocks(n4, kBlock)), dim3(kBlock), 0, s, (const unsigned short*)x, sig, HW, n4,
                       (unsigned short*)y);
    return launch_status();
}

int lss_se_bwd(const void* dy, const void* x, int32_t N, int32_t C, int32_t HW, const float* w1, const float* w2,
               int32_t sq, const float* r, const float* sig, float* t, float* dh_part, float* de, float* dr, float* dm,
               void* dx, void* stream) {
    if (!dy || !x || !w1 || !w2 || !r || !sig || !t || !dh_part || !de || !dr || !dm || !dx || !se_ok(N, C, HW, sq))
        return LSS_CONV_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    const int planes = N * C, n4 = planes * HW / 4;
    hipLaunchKernelGGL(k_se_dot, dim3(blocks(planes, kBlock / kWave)), dim3(kBlock), 0, s,
                       (const unsigned short*)dy, (const unsigned short*)x, planes, HW, t);
    const int nchunk = (C + kMlpbC - 1) / kMlpbC;
    hipLaunchKernelGGL(k_se_mlpb1, dim3(N * nchunk), dim3(kBlock), 0, s, t, sig, w2, C, sq, de, dh_part);
    hipLaunchKernelGGL(k_se_mlpb2, dim3(N * nchunk), dim3(kBlock), 0, s, dh_part, r, w1, C, sq, dr, dm);
    hipLaunchKernelGGL(k_se_dx, dim3(blocks(n4, kBlock)), dim3(kBlock), 0, s, (const unsigned short*)dy, sig, dm, HW,
                       n4, (unsigned short*)dx);
    return launch_status();
}

int lss_se_wgrad(const float* de, const float* h, const float* dr, const float* m, int32_t N, int32_t C, int32_t sq,
                 float* dw1, float* db1, float* dw2, float* db2, void* stream) {
    if (!de || !h || !dr || !m || !dw1 || !db1 || !dw2 || !db2 || N <= 0 || C <= 0 || C > kMaxC || sq <= 0 ||
        sq > kWave)
        return LSS_CONV_EINVAL;
    const int total = 2 * C * sq + sq + C;
    hipLaunchKernelGGL(k_se_wgrad, dim3(blocks(total, kBlock)), dim3(kBlock), 0, (hipStream_t)stream, de, h, dr, m, N,
                       C, sq, dw1, db1, dw2, db2);
    return launch_status();
}

}  // extern "C"

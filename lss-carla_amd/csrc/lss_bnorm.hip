// lss_bnorm.hip -- gfx950 training-mode batch norm (+ activation, + residual) for the conv stacks
// around the Lift-Splat hot path: the EfficientNet-B0 trunk's BN + swish (src/models.py:68 and the
// MBConv blocks), CamEncode.up1 / BevEncode's BN + ReLU (src/models.py:15-34, 92-130).
//
// Activations fp32 or bf16, NCHW or channels-last (NHWC); statistics, affine parameters and all
// arithmetic fp32. Two launches per direction (one for NCHW maps small enough for one block per
// channel: k_bn_fused_nchw / k_bn_bwd_fused_nchw):
//   forward  1. per-group shifted sums of x - K_c and (x - K_c)^2 (K_c = the channel's first
//               element, so the one-pass variance does not cancel);
//            2. every block folds the group sums of its channel(s) in a fixed order (all blocks
//               get identical statistics; the first block of a channel also writes the running
//               statistics and the saved mean / rstd / scale / shift) and writes
//               y = act(x * scale_c + shift_c [+ residual]).
//   backward 1. per-group sums of g and g * xhat, g = dy * act'(.) (ReLU from y; swish from the
//               pre-activation recomputed from x);
//            2. fold as above (first block writes dgamma, dbeta), dx = scale_c (g - mean g -
//               xhat mean(g xhat)), d residual = g.
// NCHW: block = (channel, group of images), the channel is block-uniform (scalar loads / SGPR
// operands), V consecutive elements per thread. NHWC: block = group of pixels x all channels,
// 8 consecutive channels per thread, per-channel coefficients staged in LDS.

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <limits.h>
#include <math.h>
#include <stdint.h>

#include <type_traits>

#include "lss_convs.h"

// The library is built with -ffp-contract=off for the geometry's reference op order (lss_hip.hip);
// the conv-stack kernels here have no bit-exact contract, so they keep FMA contraction.
#pragma clang fp contract(fast)

namespace {

using bf16 = __hip_bfloat16;
constexpr int kBlock = 256;
constexpr int kWave = 64;
#ifndef LSS_BN_GMAX
#define LSS_BN_GMAX 4096
#endif
#ifndef LSS_BN_NHWC_ELEMS
#define LSS_BN_NHWC_ELEMS 32768  // NHWC statistics: elements per block (128 per thread; 8 K: 1013 vs 966-978 us of NHWC BN per c3 step, profiles/r06/bn_nhwc_groups_ab.txt)
#endif
#ifndef LSS_BN_NHWC_GMIN
#define LSS_BN_NHWC_GMIN 512  // ... but at least this many blocks where each still gets >= 8 K elements
#endif
constexpr int kMaxGroupsNhwc = 4096;  // partial groups the ABI accepts (NHWC)
constexpr int kGroupsNhwc = LSS_BN_GMAX;  // groups lss_bn_groups picks at most (NHWC)

__device__ __forceinline__ float ld(const float* p) { return *p; }
__device__ __forceinline__ float ld(const bf16* p) { return __bfloat162float(*p); }

// V consecutive elements <-> fp32 (V in {1, 4, 8})
template <int V> __device__ __forceinline__ void ldv(const float* p, float* o) {
    if constexpr (V == 1) {
        o[0] = *p;
    } else {
#pragma unroll
        for (int i = 0; i < V; i += 4) {
            const float4 a = *reinterpret_cast<const float4*>(p + i);
            o[i] = a.x; o[i + 1] = a.y; o[i + 2] = a.z; o[i + 3] = a.w;
        }
    }
}
template <int V> __device__ __forceinline__ void ldv(const bf16* p, float* o) {
    if constexpr (V == 1) {
        o[0] = __bfloat162float(*p);
    } else {
        unsigned w[V / 2];
        if constexpr (V == 8) {
            const uint4 u = *reinterpret_cast<const uint4*>(p);
            w[0] = u.x; w[1] = u.y; w[2] = u.z; w[3] = u.w;
        } else {
            const uint2 u = *reinterpret_cast<const uint2*>(p);
            w[0] = u.x; w[1] = u.y;
        }
#pragma unroll
        for (int i = 0; i < V / 2; ++i) {
            o[2 * i] = __uint_as_float(w[i] << 16);
            o[2 * i + 1] = __uint_as_float(w[i] & 0xFFFF0000u);
        }
    }
}
template <int V> __device__ __forceinline__ void stv(float* p, const float* v) {
    if constexpr (V == 1) {
        *p = v[0];
    } else {
#pragma unroll
        for (int i = 0; i < V; i += 4) *reinterpret_cast<float4*>(p + i) = make_float4(v[i], v[i + 1], v[i + 2], v[i + 3]);
    }
}
template <int V> __device__ __forceinline__ void stv(bf16* p, const float* v) {
    if constexpr (V == 1) {
        *p = __float2bfloat16(v[0]);
    } else {
        bf16 b[V];
#pragma unroll
        for (int i = 0; i < V; ++i) b[i] = __float2bfloat16(v[i]);
        if constexpr (V == 8) *reinterpret_cast<uint4*>(p) = *reinterpret_cast<const uint4*>(b);
        else *reinterpret_cast<uint2*>(p) = *reinterpret_cast<const uint2*>(b);
    }
}

__device__ __forceinline__ float sigmoidf(float z) { return 1.f / (1.f + __expf(-z)); }

__device__ __forceinline__ float act_fwd(float z, int act) {
    if (act == LSS_ACT_RELU) return fmaxf(z, 0.f);
    if (act == LSS_ACT_SWISH) return z * sigmoidf(z);
    return z;
}

// dy -> g = dy * act'(pre-activation z); ReLU: from the output (y > 0), swish: from z
__device__ __forceinline__ float grad_pre(float dy, float y, float z, int act) {
    if (act == LSS_ACT_RELU) return y > 0.f ? dy : 0.f;
    if (act == LSS_ACT_SWISH) {
        const float s = sigmoidf(z);
        return dy * s * (1.f + z * (1.f - s));
    }
    return dy;
}

// the forward's stored ReLU output for a pre-activation z without a residual: relu(z) rounded to T
// (the NHWC backward's stand-in for y when the caller passes none -- the same value the forward's
// apply wrote, so the mask y > 0 is the same; one tensor read less in both backward passes)
template <typename T> __device__ __forceinline__ float relu_out(float z);
template <> __device__ __forceinline__ float relu_out<float>(float z) { return fmaxf(z, 0.f); }
template <> __device__ __forceinline__ float relu_out<bf16>(float z) {
    return __bfloat162float(__float2bfloat16(fmaxf(z, 0.f)));
}

struct BnGeo {
    int N, C, HW;
};

template <typename T>
__device__ __forceinline__ float first_nchw(const T* x, int c, const BnGeo& g) { return ld(x + (size_t)c * g.HW); }

// sum of a pair over a block, fixed order (wave shuffles, then waves in order); result valid in thread 0
__device__ __forceinline__ void block_pair_sum(float& a, float& b, float (*s_red)[kBlock / kWave]) {
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) {
        a += __shfl_xor(a, o, kWave);
        b += __shfl_xor(b, o, kWave);
    }
    const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
    if (lane == 0) {
        s_red[0][wave] = a;
        s_red[1][wave] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        a = 0.f;
        b = 0.f;
#pragma unroll
        for (int j = 0; j < kBlock / kWave; ++j) {
            a += s_red[0][j];
            b += s_red[1][j];
        }
    }
}

// fold G pairs partial[(c * G + q) * 2 + k] (NCHW layout of the partials) with one wave, lanes over
// groups, fixed order; returns the sums in every lane of wave 0 (others: undefined)
__device__ __forceinline__ void fold_groups(const float* __restrict__ partial, int c, int G, float& a, float& b) {
    a = 0.f;
    b = 0.f;
    for (int q = threadIdx.x; q < G; q += kWave) {
        a += partial[((size_t)c * G + q) * 2];
        b += partial[((size_t)c * G + q) * 2 + 1];
    }
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) {
        a += __shfl_xor(a, o, kWave);
        b += __shfl_xor(b, o, kWave);
    }
}

// ============================================================================= NCHW
// block (c, q): images [N q / G, N (q+1) / G) of channel c; V elements per thread (HW % V == 0)
template <int V, typename T, typename F>
__device__ __forceinline__ void for_chunk_nchw(const BnGeo& g, int G, int c, int q, F&& f) {
    const int n0 = (int)((long)g.N * q / G), n1 = (int)((long)g.N * (q + 1) / G);
    const int per = g.HW / V;
    const int count = per * (n1 - n0);
    for (int e = threadIdx.x; e < count; e += kBlock) {
        const int nl = e / per, p = (e - nl * per) * V;
        f(((size_t)(n0 + nl) * g.C + c) * g.HW + p);
    }
}

template <int V, typename T>
__global__ __launch_bounds__(kBlock) void k_bn_stats_nchw(const T* __restrict__ x, BnGeo g, int G,
                                                          float* __restrict__ partial) {
    __shared__ float s_red[2][kBlock / kWave];
    const int c = blockIdx.x % g.C, q = blockIdx.x / g.C;
    const float k = first_nchw(x, c, g);
    float s1 = 0.f, s2 = 0.f;
    for_chunk_nchw<V, T>(g, G, c, q, [&](size_t i) {
        float v[V];
        ldv<V>(x + i, v);
#pragma unroll
        for (int j = 0; j < V; ++j) {
            const float d = v[j] - k;
            s1 += d;
            s2 = fmaf(d, d, s2);
        }
    });
    block_pair_sum(s1, s2, s_red);
    if (threadIdx.x == 0) {
        partial[((size_t)c * G + q) * 2] = s1;
        partial[((size_t)c * G + q) * 2 + 1] = s2;
    }
}

struct BnParams {
    const float* gamma;
    const float* beta;
    float eps, momentum;
    float* run_mean;
    float* run_var;
    float* stats;  // (4, C): save_mean, save_rstd, scale, shift
    long long* batches;  // nn.BatchNorm2d.num_batches_tracked (nullable), +1 per forward
};

// statistics of channel c from its folded sums; the writer block stores running / saved values
__device__ __forceinline__ void finalize_channel(float s1, float s2, float k, float n, int c, int C,
                                                 const BnParams& P, bool writer, float& scale, float& shift) {
    const float d = s1 / n;
    const float mean = k + d;
    const float var = fmaxf(s2 / n - d * d, 0.f);  // biased, used to normalise
    const float rstd = rsqrtf(var + P.eps);
    scale = (P.gamma ? P.gamma[c] : 1.f) * rstd;
    shift = (P.beta ? P.beta[c] : 0.f) - mean * scale;
    if (writer) {
        if (c == 0 && P.batches) *P.batches += 1;
        if (P.run_mean) P.run_mean[c] = (1.f - P.momentum) * P.run_mean[c] + P.momentum * mean;
        if (P.run_var)
            P.run_var[c] = (1.f - P.momentum) * P.run_var[c] + P.momentum * (n > 1.f ? var * n / (n - 1.f) : var);
        P.stats[c] = mean;
        P.stats[C + c] = rstd;
        P.stats[2 * C + c] = scale;
        P.stats[3 * C + c] = shift;
    }
}

template <int V, typename T>
__global__ __launch_bounds__(kBlock) void k_bn_apply_nchw(const T* __restrict__ x, const T* __restrict__ res, BnGeo g,
                                                          int G, const float* __restrict__ partial, BnParams P, int act,
                                                          T* __restrict__ y) {
    __shared__ float s_coef[2];
    const int c = blockIdx.x % g.C, q = blockIdx.x / g.C;
    if (threadIdx.x < kWave) {
        float s1, s2;
        fold_groups(partial, c, G, s1, s2);
        float sc, sh;
        finalize_channel(s1, s2, first_nchw(x, c, g), (float)g.N * (float)g.HW, c, g.C, P, q == 0 && threadIdx.x == 0,
                         sc, sh);
        if (threadIdx.x == 0) {
            s_coef[0] = sc;
            s_coef[1] = sh;
        }
    }
    __syncthreads();
    const float sc = s_coef[0], sh = s_coef[1];
    for_chunk_nchw<V, T>(g, G, c, q, [&](size_t i) {
        float v[V], r[V];
        ldv<V>(x + i, v);
        if (res) ldv<V>(res + i, r);
#pragma unroll
        for (int j = 0; j < V; ++j) {
            float z = fmaf(v[j], sc, sh);
            if (res) z += r[j];
            v[j] = act_fwd(z, act);
        }
        stv<V>(y + i, v);
    });
}

template <int V, typename T>
__global__ __launch_bounds__(kBlock) void k_bn_bwd_stats_nchw(const T* __restrict__ dy, const T* __restrict__ x,
                                                              const T* __restrict__ y, BnGeo g, int G,
                                                              const float* __restrict__ stats, int act,
                                                              float* __restrict__ partial) {
    __shared__ float s_red[2][kBlock / kWave];
    const int c = blockIdx.x % g.C, q = blockIdx.x / g.C;
    const float mean = stats[c], rstd = stats[g.C + c], sc = stats[2 * g.C + c], sh = stats[3 * g.C + c];
    float sg = 0.f, sgx = 0.f;
    for_chunk_nchw<V, T>(g, G, c, q, [&](size_t i) {
        float d[V], xv[V], yv[V];
        ldv<V>(dy + i, d);
        ldv<V>(x + i, xv);
        if (act == LSS_ACT_RELU) ldv<V>(y + i, yv);
#pragma unroll
        for (int j = 0; j < V; ++j) {
            const float gr = grad_pre(d[j], act == LSS_ACT_RELU ? yv[j] : 0.f, fmaf(xv[j], sc, sh), act);
            sg += gr;
            sgx = fmaf(gr, (xv[j] - mean) * rstd, sgx);
        }
    });
    block_pair_sum(sg, sgx, s_red);
    if (threadIdx.x == 0) {
        partial[((size_t)c * G + q) * 2] = sg;
        partial[((size_t)c * G + q) * 2 + 1] = sgx;
    }
}

template <int V, typename T>
__global__ __launch_bounds__(kBlock) void k_bn_bwd_apply_nchw(const T* __restrict__ dy, const T* __restrict__ x,
                                                              const T* __restrict__ y, BnGeo g, int G,
                                                              const float* __restrict__ stats,
                                                              const float* __restrict__ partial, int act,
                                                              float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                              T* __restrict__ dx, T* __restrict__ dres) {
    __shared__ float s_coef[2];
    const int c = blockIdx.x % g.C, q = blockIdx.x / g.C;
    if (threadIdx.x < kWave) {
        float sg, sgx;
        fold_groups(partial, c, G, sg, sgx);
        if (threadIdx.x == 0) {
            if (q == 0) {
                if (dgamma) dgamma[c] = sgx;
                if (dbeta) dbeta[c] = sg;
            }
            const float n = (float)g.N * (float)g.HW;
            s_coef[0] = sg / n;
            s_coef[1] = sgx / n;
        }
    }
    __syncthreads();
    const float mg = s_coef[0], mgx = s_coef[1];
    const float mean = stats[c], rstd = stats[g.C + c], sc = stats[2 * g.C + c], sh = stats[3 * g.C + c];
    for_chunk_nchw<V, T>(g, G, c, q, [&](size_t i) {
        float d[V], xv[V], yv[V], o[V], gr[V];
        ldv<V>(dy + i, d);
        ldv<V>(x + i, xv);
        if (act == LSS_ACT_RELU) ldv<V>(y + i, yv);
#pragma unroll
        for (int j = 0; j < V; ++j) {
            gr[j] = grad_pre(d[j], act == LSS_ACT_RELU ? yv[j] : 0.f, fmaf(xv[j], sc, sh), act);
            o[j] = sc * (gr[j] - mg - (xv[j] - mean) * rstd * mgx);
        }
        stv<V>(dx + i, o);
        if (dres) stv<V>(dres + i, gr);
    });
}

// ---- one group per channel (G == 1: every map of 8 x 22 pixels or less at B*N = 48): statistics and
// apply in ONE launch, a block per channel -- the second pass re-reads the channel (<= 17 KB at c3)
// from the cache the first pass filled. Same sums, same fold, same bits as the two launches above.
template <int V, typename T>
__global__ __launch_bounds__(kBlock) void k_bn_fused_nchw(const T* __restrict__ x, const T* __restrict__ res, BnGeo g,
                                                          BnParams P, int act, T* __restrict__ y) {
    __shared__ float s_red[2][kBlock / kWave];
    __shared__ float s_coef[2];
    const int c = blockIdx.x;
    const float k = first_nchw(x, c, g);
    float s1 = 0.f, s2 = 0.f;
    for_chunk_nchw<V, T>(g, 1, c, 0, [&](size_t i) {
        float v[V];
        ldv<V>(x + i, v);
#pragma unroll
        for (int j = 0; j < V; ++j) {
            const float d = v[j] - k;
            s1 += d;
            s2 = fmaf(d, d, s2);
        }
    });
    block_pair_sum(s1, s2, s_red);
    if (threadIdx.x == 0) {
        float sc, sh;
        finalize_channel(s1, s2, k, (float)g.N * (float)g.HW, c, g.C, P, true, sc, sh);
        s_coef[0] = sc;
        s_coef[1] = sh;
    }
    __syncthreads();
    const float sc = s_coef[0], sh = s_coef[1];
    for_chunk_nchw<V, T>(g, 1, c, 0, [&](size_t i) {
        float v[V], r[V];
        ldv<V>(x + i, v);
        if (res) ldv<V>(res + i, r);
#pragma unroll
        for (int j = 0; j < V; ++j) {
            float z = fmaf(v[j], sc, sh);
            if (res) z += r[j];
            v[j] = act_fwd(z, act);
        }
        stv<V>(y + i, v);
    });
}

template <int V, typename T>
__global__ __launch_bounds__(kBlock) void k_bn_bwd_fused_nchw(const T* __restrict__ dy, const T* __restrict__ x,
                                                              const T* __restrict__ y, BnGeo g,
                                                              const float* __restrict__ stats, int act,
                                                              float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                              T* __restrict__ dx, T* __restrict__ dres) {
    __shared__ float s_red[2][kBlock / kWave];
    __shared__ float s_coef[2];
    const int c = blockIdx.x;
    const float mean = stats[c], rstd = stats[g.C + c], sc = stats[2 * g.C + c], sh = stats[3 * g.C + c];
    float sg = 0.f, sgx = 0.f;
    for_chunk_nchw<V, T>(g, 1, c, 0, [&](size_t i) {
        float d[V], xv[V], yv[V];
        ldv<V>(dy + i, d);
        ldv<V>(x + i, xv);
        if (act == LSS_ACT_RELU) ldv<V>(y + i, yv);
#pragma unroll
        for (int j = 0; j < V; ++j) {
            const float gr = grad_pre(d[j], act == LSS_ACT_RELU ? yv[j] : 0.f, fmaf(xv[j], sc, sh), act);
            sg += gr;
            sgx = fmaf(gr, (xv[j] - mean) * rstd, sgx);
        }
    });
    block_pair_sum(sg, sgx, s_red);
    if (threadIdx.x == 0) {
        if (dgamma) dgamma[c] = sgx;
        if (dbeta) dbeta[c] = sg;
        const float n = (float)g.N * (float)g.HW;
        s_coef[0] = sg / n;
        s_coef[1] = sgx / n;
    }
    __syncthreads();
    const float mg = s_coef[0], mgx = s_coef[1];
    for_chunk_nchw<V, T>(g, 1, c, 0, [&](size_t i) {
        float d[V], xv[V], yv[V], o[V], gr[V];
        ldv<V>(dy + i, d);
        ldv<V>(x + i, xv);
        if (act == LSS_ACT_RELU) ldv<V>(y + i, yv);
#pragma unroll
        for (int j = 0; j < V; ++j) {
            gr[j] = grad_pre(d[j], act == LSS_ACT_RELU ? yv[j] : 0.f, fmaf(xv[j], sc, sh), act);
            o[j] = sc * (gr[j] - mg - (xv[j] - mean) * rstd * mgx);
        }
        stv<V>(dx + i, o);
        if (dres) stv<V>(dres + i, gr);
    });
}

// (IT = 5 for the trunk's 8 x 22 maps at B*N = 48: 1,056 vectors, one over IT = 4's reach; with IT = 8
// the backward's 130 VGPRs held 3 blocks per CU, 1.5 rounds for 1,152 channels)
// bf16, one group per channel, at most IT vectors of V elements per thread: the same two launches'
// work with every load of the channel issued up front and the channel held in registers (packed
// bf16) between the statistics and the apply -- one read of x (and dy) instead of two, and no
// round trip per loop iteration. Same sums in the same order as k_bn_fused_nchw (bit-identical).
template <int V> struct PackedBf16;
template <> struct PackedBf16<8> {
    uint4 u;
    __device__ __forceinline__ void load(const bf16* p) { u = *reinterpret_cast<const uint4*>(p); }
    __device__ __forceinline__ void get(float* o) const {
        const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            o[2 * i] = __uint_as_float(w[i] << 16);
            o[2 * i + 1] = __uint_as_float(w[i] & 0xFFFF0000u);
        }
    }
};
template <> struct PackedBf16<4> {
    uint2 u;
    __device__ __forceinline__ void load(const bf16* p) { u = *reinterpret_cast<const uint2*>(p); }
    __device__ __forceinline__ void get(float* o) const {
        o[0] = __uint_as_float(u.x << 16); o[1] = __uint_as_float(u.x & 0xFFFF0000u);
        o[2] = __uint_as_float(u.y << 16); o[3] = __uint_as_float(u.y & 0xFFFF0000u);
    }
};

// the element offset of vector e of channel c (one group: images 0..N-1), e clamped into range
__device__ __forceinline__ size_t chan_vec(const BnGeo& g, int c, int per, int count, int e, int V) {
    const int ec = min(e, count - 1);
    const int nl = ec / per, p = (ec - nl * per) * V;
    return ((size_t)nl * g.C + c) * g.HW + p;
}

template <int V, int IT>
__global__ __launch_bounds__(kBlock) void k_bn_fused_reg_nchw(const bf16* __restrict__ x, const bf16* __restrict__ res,
                                                              BnGeo g, BnParams P, int act, bf16* __restrict__ y) {
    __shared__ float s_red[2][kBlock / kWave];
    __shared__ float s_coef[2];
    const int c = blockIdx.x;
    const int per = g.HW / V, count = per * g.N;
    PackedBf16<V> raw[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) raw[it].load(x + chan_vec(g, c, per, count, (int)threadIdx.x + it * kBlock, V));
    const float k = first_nchw(x, c, g);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        if ((int)threadIdx.x + it * kBlock < count) {
            float v[V];
            raw[it].get(v);
#pragma unroll
            for (int j = 0; j < V; ++j) {
                const float d = v[j] - k;
                s1 += d;
                s2 = fmaf(d, d, s2);
            }
        }
    }
    block_pair_sum(s1, s2, s_red);
    if (threadIdx.x == 0) {
        float sc, sh;
        finalize_channel(s1, s2, k, (float)g.N * (float)g.HW, c, g.C, P, true, sc, sh);
        s_coef[0] = sc;
        s_coef[1] = sh;
    }
    __syncthreads();
    const float sc = s_coef[0], sh = s_coef[1];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int e = (int)threadIdx.x + it * kBlock;
        if (e < count) {
            const size_t i = chan_vec(g, c, per, count, e, V);
            float v[V], r[V];
            raw[it].get(v);
            if (res) ldv<V>(res + i, r);
#pragma unroll
            for (int j = 0; j < V; ++j) {
                float z = fmaf(v[j], sc, sh);
                if (res) z += r[j];
                v[j] = act_fwd(z, act);
            }
            stv<V>(y + i, v);
        }
    }
}

template <int V, int IT>
__global__ __launch_bounds__(kBlock) void k_bn_bwd_fused_reg_nchw(const bf16* __restrict__ dy, const bf16* __restrict__ x,
                                                                  const bf16* __restrict__ y, BnGeo g,
                                                                  const float* __restrict__ stats, int act,
                                                                  float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                                  bf16* __restrict__ dx, bf16* __restrict__ dres) {
    __shared__ float s_red[2][kBlock / kWave];
    __shared__ float s_coef[2];
    const int c = blockIdx.x;
    const int per = g.HW / V, count = per * g.N;
    const bool relu = act == LSS_ACT_RELU;
    PackedBf16<V> rd[IT], rx[IT], ry[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const size_t i = chan_vec(g, c, per, count, (int)threadIdx.x + it * kBlock, V);
        rd[it].load(dy + i);
        rx[it].load(x + i);
        ry[it].load((relu ? y : x) + i);  // (unconditional: a load under a branch waits for the worst case)
    }
    const float mean = stats[c], rstd = stats[g.C + c], sc = stats[2 * g.C + c], sh = stats[3 * g.C + c];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        if ((int)threadIdx.x + it * kBlock < count) {
            float d[V], xv[V], yv[V];
            rd[it].get(d);
            rx[it].get(xv);
            ry[it].get(yv);
#pragma unroll
            for (int j = 0; j < V; ++j) {
                const float gr = grad_pre(d[j], relu ? yv[j] : 0.f, fmaf(xv[j], sc, sh), act);
                sg += gr;
                sgx = fmaf(gr, (xv[j] - mean) * rstd, sgx);
            }
        }
    }
    block_pair_sum(sg, sgx, s_red);
    if (threadIdx.x == 0) {
        if (dgamma) dgamma[c] = sgx;
        if (dbeta) dbeta[c] = sg;
        const float n = (float)g.N * (float)g.HW;
        s_coef[0] = sg / n;
        s_coef[1] = sgx / n;
    }
    __syncthreads();
    const float mg = s_coef[0], mgx = s_coef[1];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int e = (int)threadIdx.x + it * kBlock;
        if (e < count) {
            const size_t i = chan_vec(g, c, per, count, e, V);
            float d[V], xv[V], yv[V], o[V], gr[V];
            rd[it].get(d);
            rx[it].get(xv);
            ry[it].get(yv);
#pragma unroll
            for (int j = 0; j < V; ++j) {
                gr[j] = grad_pre(d[j], relu ? yv[j] : 0.f, fmaf(xv[j], sc, sh), act);
                o[j] = sc * (gr[j] - mg - (xv[j] - mean) * rstd * mgx);
            }
            stv<V>(dx + i, o);
            if (dres) stv<V>(dres + i, gr);
        }
    }
}

// ---- NCHW with G > 1 groups per channel, bf16: statistics and apply in ONE launch (lss_bn_fwd2 /
// lss_bn_bwd2 with a sync workspace). Block b = (channel c = b / G, group q = b % G), so the G blocks of
// a channel are consecutive in dispatch order (a cluster). Each block holds its group of the channel
// (images [N q / G, N (q + 1) / G)) in registers, publishes its partial pair with an agent-scope store,
// arrives on the channel's counter and waits for the other G - 1 blocks of its cluster, folds the G
// pairs in group order and applies from its registers: x (and dy) read once instead of twice, one
// launch instead of two. Same sums in the same order as k_bn_stats_nchw + k_bn_apply_nchw (and the
// backward pair), so the same bits. The wait is bounded: a block that gives up recomputes every
// group's pair from memory itself (same code, same order: exact), so a cluster whose blocks are not
// all resident only costs time. The last block to leave re-zeroes the channel's two counters.
constexpr unsigned kBnSpinLimit = 1u << 20;
constexpr int kBnClusterMaxG = 64;  // (the timeout path's LDS pairs)
constexpr int kBnClusterIT = 8;     // 16-B vectors per thread held in registers
constexpr int kBnSyncMaxC = 4096;   // channels a sync workspace covers (+ the spin word)
constexpr int kBnSyncStride = 32;   // words per channel: its two counters alone in a 128-B line (a line
                                    // shared by the counters of many channels serialised every poll)

__device__ __forceinline__ void st_pair_agent(float* p, float a, float b) {
    const unsigned long long v = ((unsigned long long)__float_as_uint(b) << 32) | __float_as_uint(a);
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float2 ld_pair_agent(const float* p) {
    const unsigned long long v =
        __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return make_float2(__uint_as_float((unsigned)v), __uint_as_float((unsigned)(v >> 32)));
}

// thread 0: publish (a, b) as group q's pair, arrive, wait for the cluster; true = all G arrived.
// limit_word (the workspace's last word): 0 = kBnSpinLimit polls, s > 0 = s - 1 (tests of the timeout path)
__device__ __forceinline__ bool cluster_publish_wait(float* __restrict__ partial, size_t at, float a, float b,
                                                     unsigned* arrive, int G, const unsigned* limit_word) {
    // the R2 hand-off (cdna_hip_programming.md, Guideline 16): the pair written through (sc1) and
    // retired (vmcnt counts stores) before the arrival; readers poll and read with sc1 loads. No fence:
    // an agent-scope fence writes back / invalidates the whole L2 of the XCD, per block
    st_pair_agent(partial + at, a, b);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned lo = *limit_word;
    const unsigned limit = lo ? lo - 1u : kBnSpinLimit;
    for (unsigned spins = 0;; ++spins) {
        if (__hip_atomic_load(arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (unsigned)G) return true;
        if (spins >= limit) return false;
        __builtin_amdgcn_s_sleep(8);
    }
}
__device__ __forceinline__ void cluster_leave(unsigned* arrive, unsigned* leave, int G) {
    if (atomicAdd(leave, 1u) == (unsigned)G - 1u) {
        atomicExch(arrive, 0u);
        atomicExch(leave, 0u);
    }
}

// wave 0: the G pairs of channel c in fold_groups' order (lanes over groups, then a butterfly), from
// the published pairs or, after a timeout, from the block's own recomputation in LDS
__device__ __forceinline__ void fold_cluster(const float* __restrict__ partial, int c, int G, bool published,
                                             const float (*s_pairs)[2], float& a, float& b) {
    a = 0.f;
    b = 0.f;
    for (int q = threadIdx.x; q < G; q += kWave) {
        const float2 v = published ? ld_pair_agent(partial + ((size_t)c * G + q) * 2) : make_float2(s_pairs[q][0], s_pairs[q][1]);
        a += v.x;
        b += v.y;
    }
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) {
        a += __shfl_xor(a, o, kWave);
        b += __shfl_xor(b, o, kWave);
    }
}

template <int V, int IT>
__global__ __launch_bounds__(kBlock) void k_bn_cluster_nchw(const bf16* __restrict__ x, const bf16* __restrict__ res,
                                                            BnGeo g, int G, float* __restrict__ partial, BnParams P,
                                                            int act, unsigned* __restrict__ sync,
                                                            bf16* __restrict__ y) {
    __shared__ float s_red[2][kBlock / kWave];
    __shared__ float s_pairs[kBnClusterMaxG][2];
    __shared__ float s_coef[2];
    __shared__ int s_ok;
    const int c = blockIdx.x / G, q = blockIdx.x - c * G;
    const int n0 = (int)((long)g.N * q / G), n1 = (int)((long)g.N * (q + 1) / G);
    const int per = g.HW / V, count = per * (n1 - n0);
    const bf16* xc = x + ((size_t)n0 * g.C + c) * g.HW;  // (chan_vec over the group's images)
    PackedBf16<V> raw[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it)
        raw[it].load(xc + chan_vec(g, 0, per, count, (int)threadIdx.x + it * kBlock, V) + (size_t)0);
    const float k = first_nchw(x, c, g);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        if ((int)threadIdx.x + it * kBlock < count) {
            float v[V];
            raw[it].get(v);
#pragma unroll
            for (int j = 0; j < V; ++j) {
                const float d = v[j] - k;
                s1 += d;
                s2 = fmaf(d, d, s2);
            }
        }
    }
    block_pair_sum(s1, s2, s_red);
    unsigned* arrive = sync + (size_t)c * kBnSyncStride;
    if (threadIdx.x == 0)
        s_ok = cluster_publish_wait(partial, ((size_t)c * G + q) * 2, s1, s2, arrive, G,
                                    sync + (size_t)kBnSyncMaxC * kBnSyncStride);
    __syncthreads();
    const bool ok = s_ok;
    if (!ok) {  // (never expected) every group's pair from memory, in k_bn_stats_nchw's order
        for (int qq = 0; qq < G; ++qq) {
            float a = 0.f, b = 0.f;
            for_chunk_nchw<V, bf16>(g, G, c, qq, [&](size_t i) {
                float v[V];
                ldv<V>(x + i, v);
#pragma unroll
                for (int j = 0; j < V; ++j) {
                    const float d = v[j] - k;
                    a += d;
                    b = fmaf(d, d, b);
                }
            });
            block_pair_sum(a, b, s_red);
            if (threadIdx.x == 0) {
                s_pairs[qq][0] = a;
                s_pairs[qq][1] = b;
            }
            __syncthreads();
        }
    }
    if (threadIdx.x < kWave) {
        float f1, f2;
        fold_cluster(partial, c, G, ok, s_pairs, f1, f2);
        float sc, sh;
        finalize_channel(f1, f2, k, (float)g.N * (float)g.HW, c, g.C, P, q == 0 && threadIdx.x == 0, sc, sh);
        if (threadIdx.x == 0) {
            s_coef[0] = sc;
            s_coef[1] = sh;
            cluster_leave(arrive, arrive + 1, G);
        }
    }
    __syncthreads();
    const float sc = s_coef[0], sh = s_coef[1];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int e = (int)threadIdx.x + it * kBlock;
        if (e < count) {
            const size_t i = ((size_t)n0 * g.C + c) * g.HW + chan_vec(g, 0, per, count, e, V);
            float v[V], r[V];
            raw[it].get(v);
            if (res) ldv<V>(res + i, r);
#pragma unroll
            for (int j = 0; j < V; ++j) {
                float z = fmaf(v[j], sc, sh);
                if (res) z += r[j];
                v[j] = act_fwd(z, act);
            }
            stv<V>(y + i, v);
        }
    }
}

template <int V, int IT, bool RELU>
__global__ __launch_bounds__(kBlock) void k_bn_bwd_cluster_nchw(const bf16* __restrict__ dy, const bf16* __restrict__ x,
                                                                const bf16* __restrict__ y, BnGeo g, int G,
                                                                const float* __restrict__ stats, float* __restrict__ partial,
                                                                int act, unsigned* __restrict__ sync,
                                                                float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                                bf16* __restrict__ dx, bf16* __restrict__ dres) {
    __shared__ float s_red[2][kBlock / kWave];
    __shared__ float s_pairs[kBnClusterMaxG][2];
    __shared__ float s_coef[2];
    __shared__ int s_ok;
    const int c = blockIdx.x / G, q = blockIdx.x - c * G;
    const int n0 = (int)((long)g.N * q / G), n1 = (int)((long)g.N * (q + 1) / G);
    const int per = g.HW / V, count = per * (n1 - n0);
    const size_t base = ((size_t)n0 * g.C + c) * g.HW;
    PackedBf16<V> rd[IT], rx[IT], ry[RELU ? IT : 1];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const size_t i = base + chan_vec(g, 0, per, count, (int)threadIdx.x + it * kBlock, V);
        rd[it].load(dy + i);
        rx[it].load(x + i);
        if constexpr (RELU) ry[it].load(y + i);
    }
    const float mean = stats[c], rstd = stats[g.C + c], sc = stats[2 * g.C + c], sh = stats[3 * g.C + c];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        if ((int)threadIdx.x + it * kBlock < count) {
            float d[V], xv[V], yv[V];
            rd[it].get(d);
            rx[it].get(xv);
            if constexpr (RELU) ry[it].get(yv);
#pragma unroll
            for (int j = 0; j < V; ++j) {
                const float gr = grad_pre(d[j], RELU ? yv[j] : 0.f, fmaf(xv[j], sc, sh), act);
                sg += gr;
                sgx = fmaf(gr, (xv[j] - mean) * rstd, sgx);
            }
        }
    }
    block_pair_sum(sg, sgx, s_red);
    unsigned* arrive = sync + (size_t)c * kBnSyncStride;
    if (threadIdx.x == 0)
        s_ok = cluster_publish_wait(partial, ((size_t)c * G + q) * 2, sg, sgx, arrive, G,
                                    sync + (size_t)kBnSyncMaxC * kBnSyncStride);
    __syncthreads();
    const bool ok = s_ok;
    if (!ok) {
        for (int qq = 0; qq < G; ++qq) {
            float a = 0.f, b = 0.f;
            for_chunk_nchw<V, bf16>(g, G, c, qq, [&](size_t i) {
                float d[V], xv[V], yv[V];
                ldv<V>(dy + i, d);
                ldv<V>(x + i, xv);
                if constexpr (RELU) ldv<V>(y + i, yv);
#pragma unroll
                for (int j = 0; j < V; ++j) {
                    const float gr = grad_pre(d[j], RELU ? yv[j] : 0.f, fmaf(xv[j], sc, sh), act);
                    a += gr;
                    b = fmaf(gr, (xv[j] - mean) * rstd, b);
                }
            });
            block_pair_sum(a, b, s_red);
            if (threadIdx.x == 0) {
                s_pairs[qq][0] = a;
                s_pairs[qq][1] = b;
            }
            __syncthreads();
        }
    }
    if (threadIdx.x < kWave) {
        float fg, fgx;
        fold_cluster(partial, c, G, ok, s_pairs, fg, fgx);
        if (threadIdx.x == 0) {
            if (q == 0) {
                if (dgamma) dgamma[c] = fgx;
                if (dbeta) dbeta[c] = fg;
            }
            const float n = (float)g.N * (float)g.HW;
            s_coef[0] = fg / n;
            s_coef[1] = fgx / n;
            cluster_leave(arrive, arrive + 1, G);
        }
    }
    __syncthreads();
    const float mg = s_coef[0], mgx = s_coef[1];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int e = (int)threadIdx.x + it * kBlock;
        if (e < count) {
            const size_t i = base + chan_vec(g, 0, per, count, e, V);
            float d[V], xv[V], yv[V], o[V], gr[V];
            rd[it].get(d);
            rx[it].get(xv);
            if constexpr (RELU) ry[it].get(yv);
#pragma unroll
            for (int j = 0; j < V; ++j) {
                gr[j] = grad_pre(d[j], RELU ? yv[j] : 0.f, fmaf(xv[j], sc, sh), act);
                o[j] = sc * (gr[j] - mg - (xv[j] - mean) * rstd * mgx);
            }
            stv<V>(dx + i, o);
            if (dres) stv<V>(dres + i, gr);
        }
    }
}

// ============================================================================= NHWC (channels-last)
// block q: pixels [M q / G, M (q+1) / G) x all C channels; thread = 8 consecutive channels of a pixel.
// Partials (C, G, 2) as in NCHW; a separate fold kernel (one wave per channel) turns them into the
// per-channel coefficients the apply passes read.
// A thread keeps one channel octet (kBlock % (C/8) == 0) and walks the block's pixels with a stride
// of kBlock / (C/8) rows, four rows per iteration so four 16-byte loads are in flight; 32-bit
// offsets (the host checks N*HW*C < 2^31).

// f(idx, n) over the block's rows, R rows' loads in flight per iteration (n of the R row offsets valid)
template <int R, typename F>
__device__ __forceinline__ void for_rows_nhwc(const BnGeo& g, int G, int q, F&& f) {
    const int M = g.N * g.HW;
    const int r0 = (int)((long)M * q / G), r1 = (int)((long)M * (q + 1) / G);
    const int cg = g.C >> 3, step = kBlock / cg;
    const int c0 = ((int)threadIdx.x % cg) * 8;
    if ((int)threadIdx.x >= step * cg) return;
    int r = r0 + (int)threadIdx.x / cg;
    for (; r + (R - 1) * step < r1; r += R * step) {
        int idx[R];
#pragma unroll
        for (int u = 0; u < R; ++u) idx[u] = (r + u * step) * g.C + c0;
        f(idx, R);
    }
    for (; r < r1; r += step) {
        int idx[R];
#pragma unroll
        for (int u = 0; u < R; ++u) idx[u] = r * g.C + c0;
        f(idx, 1);
    }
}

// rows in flight per thread in the statistics kernels
#ifndef LSS_BN_STATS_R
#define LSS_BN_STATS_R 4
#endif
// per-thread 8-channel sums -> per-channel block sums -> partial[c][q][2]. The threads sharing a channel
// octet are lane, lane + cg, ... (cg = C / 8 divides kBlock, a power of two): a butterfly over those
// lanes inside each wave, then the waves' rows in LDS ([wave][C][2], zero where a wave holds none of
// a channel) added in wave order -- fixed association, two barriers (a serial round per thread of an
// octet took kBlock / cg barriers: 32 at C = 64).
// dynamic LDS floats per channel of nhwc_block_sums' [wave][C][2] rows (stats kernels, both directions)
constexpr int kNhwcStatsLds = (kBlock / kWave) * 2;
__device__ __forceinline__ void nhwc_block_sums(const BnGeo& g, int G, int q, float* a, float* b, int c0,
                                                bool active, float* s_acc, float* __restrict__ partial) {
    const int cg = g.C / 8;
    const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
    constexpr int NW = kBlock / kWave;
    if (!active) {
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = b[j] = 0.f;
    }
    for (int o = cg; o < kWave; o <<= 1) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            a[j] += __shfl_xor(a[j], o, kWave);
            b[j] += __shfl_xor(b[j], o, kWave);
        }
    }
    for (int i = threadIdx.x; i < NW * 2 * g.C; i += kBlock) s_acc[i] = 0.f;
    __syncthreads();
    if (active && lane < cg) {
        float* row = s_acc + (size_t)wave * 2 * g.C;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            row[2 * (c0 + j)] = a[j];
            row[2 * (c0 + j) + 1] = b[j];
        }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < g.C; c += kBlock) {
        float sa = 0.f, sb = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            sa += s_acc[(size_t)w * 2 * g.C + 2 * c];
            sb += s_acc[(size_t)w * 2 * g.C + 2 * c + 1];
        }
        partial[((size_t)c * G + q) * 2] = sa;
        partial[((size_t)c * G + q) * 2 + 1] = sb;
    }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_bn_stats_nhwc(const T* __restrict__ x, BnGeo g, int G,
                                                          float* __restrict__ partial) {
    extern __shared__ float s_dyn[];  // [waves][C][2]
    const int cg = g.C / 8;
    const int c0 = ((int)threadIdx.x % cg) * 8;  // a thread's channel group is fixed (kBlock % cg == 0)
    float k[8];
    ldv<8>(x + c0, k);  // first pixel: the shifts
    float a[8] = {}, b[8] = {};
    constexpr int R = LSS_BN_STATS_R;
    for_rows_nhwc<R>(g, G, blockIdx.x, [&](const int* idx, int n) {
        float v[R][8];
#pragma unroll
        for (int u = 0; u < R; ++u)
            if (u < n) ldv<8>(x + idx[u], v[u]);
#pragma unroll
        for (int u = 0; u < R; ++u) {
            if (u >= n) continue;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float d = v[u][j] - k[j];
                a[j] += d;
                b[j] = fmaf(d, d, b[j]);
            }
        }
    });
    nhwc_block_sums(g, G, blockIdx.x, a, b, c0, (int)threadIdx.x < (kBlock / cg) * cg, s_dyn, partial);
}

// fold kernels (NHWC): one wave per channel, lanes over groups, fixed order
// A lane's pairs of one channel's partials (groups lane, lane + 64, ...) added in that order, kFoldBatch
// loads in flight at a time: the loop that loaded one pair per iteration waited a cache round trip per
// 64 groups (up to 64 of them in sequence: a 14-19 us fold at 2,500-4,096 groups).
constexpr int kFoldBatch = 16;  // (32, one batch per lane at c3, measured no faster: launch-bound)
__device__ __forceinline__ void fold_lane_pairs(const float* __restrict__ p, int G, int lane, float& s1, float& s2) {
    int q = lane;
    for (; q + (kFoldBatch - 1) * kWave < G; q += kFoldBatch * kWave) {
        float2 v[kFoldBatch];
#pragma unroll
        for (int i = 0; i < kFoldBatch; ++i) v[i] = *reinterpret_cast<const float2*>(p + 2 * (q + i * kWave));
#pragma unroll
        for (int i = 0; i < kFoldBatch; ++i) {
            s1 += v[i].x;
            s2 += v[i].y;
        }
    }
    float2 v[kFoldBatch];
#pragma unroll
    for (int i = 0; i < kFoldBatch; ++i)
        v[i] = q + i * kWave < G ? *reinterpret_cast<const float2*>(p + 2 * (q + i * kWave)) : make_float2(0.f, 0.f);
#pragma unroll
    for (int i = 0; i < kFoldBatch; ++i)
        if (q + i * kWave < G) {
            s1 += v[i].x;
            s2 += v[i].y;
        }
}
template <typename T>
__global__ __launch_bounds__(kBlock) void k_bn_fold_nhwc(const float* __restrict__ partial, int G, const T* __restrict__ x,
                                                         BnGeo g, BnParams P) {
    const int c = blockIdx.x * (kBlock / kWave) + (int)threadIdx.x / kWave;
    if (c >= g.C) return;
    float s1 = 0.f, s2 = 0.f;
    fold_lane_pairs(partial + (size_t)c * G * 2, G, (int)threadIdx.x & (kWave - 1), s1, s2);
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) {
        s1 += __shfl_xor(s1, o, kWave);
        s2 += __shfl_xor(s2, o, kWave);
    }
    float sc, sh;
    finalize_channel(s1, s2, ld(x + c), (float)g.N * (float)g.HW, c, g.C, P, (threadIdx.x & (kWave - 1)) == 0, sc, sh);
}

__global__ __launch_bounds__(kBlock) void k_bn_bwd_fold_nhwc(const float* __restrict__ partial, int G, BnGeo g,
                                                             float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                             float* __restrict__ coef) {
    const int c = blockIdx.x * (kBlock / kWave) + (int)threadIdx.x / kWave;
    if (c >= g.C) return;
    float sg = 0.f, sgx = 0.f;
    fold_lane_pairs(partial + (size_t)c * G * 2, G, (int)threadIdx.x & (kWave - 1), sg, sgx);
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) {
        sg += __shfl_xor(sg, o, kWave);
        sgx += __shfl_xor(sgx, o, kWave);
    }
    if ((threadIdx.x & (kWave - 1)) == 0) {
        if (dgamma) dgamma[c] = sgx;
        if (dbeta) dbeta[c] = sg;
        const float n = (float)g.N * (float)g.HW;
        coef[2 * c] = sg / n;
        coef[2 * c + 1] = sgx / n;
    }
}

// y = act(x * scale_c + shift_c [+ residual]), grid-stride over 8-channel vectors
template <typename T>
__global__ __launch_bounds__(kBlock) void k_bn_apply_nhwc(const T* __restrict__ x, const T* __restrict__ res, BnGeo g,
                                                          const float* __restrict__ stats, int act, T* __restrict__ y) {
    extern __shared__ float s_dyn[];  // scale[C], shift[C]
    for (int c = threadIdx.x; c < g.C; c += kBlock) {
        s_dyn[c] = stats[2 * g.C + c];
        s_dyn[g.C + c] = stats[3 * g.C + c];
    }
    __syncthreads();
    const long nv = (long)g.N * g.HW * g.C / 8;
    for (long e = (long)blockIdx.x * kBlock + threadIdx.x; e < nv; e += (long)gridDim.x * kBlock) {
        const size_t i = (size_t)e * 8;
        const int c0 = (int)(i % g.C);
        float v[8], r[8];
        ldv<8>(x + i, v);
        if (res) ldv<8>(res + i, r);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float z = fmaf(v[j], s_dyn[c0 + j], s_dyn[g.C + c0 + j]);
            if (res) z += r[j];
            v[j] = act_fwd(z, act);
        }
        stv<8>(y + i, v);
    }
}

// Rank-1 incoming gradient (R1): dy[p][c] = bf16(g1[p] * w1[c]), computed instead of loaded -- the
// gradient a 1x1 conv to ONE channel (lss_head1_bwd2) hands back, bit for bit, never materialised.
struct Rank1 {
    const bf16* g1;   // per pixel row
    const float* w1;  // per channel
};
template <bool R1, typename T>
__device__ __forceinline__ void load_dy8(const T* __restrict__ dy, int idx, int c0, const BnGeo& g, const Rank1& r1,
                                         const float* w8, float* d) {
    if constexpr (R1) {
        const float gv = __bfloat162float(r1.g1[(idx - c0) / g.C]);
#pragma unroll
        for (int j = 0; j < 8; ++j) d[j] = __bfloat162float(__float2bfloat16(gv * w8[j]));
    } else {
        ldv<8>(dy + idx, d);
    }
}

template <typename T, bool R1 = false>
__global__ __launch_bounds__(kBlock) void k_bn_bwd_stats_nhwc(const T* __restrict__ dy, const T* __restrict__ x,
                                                              const T* __restrict__ y, BnGeo g, int G,
                                                              const float* __restrict__ stats, int act,
                                                              float* __restrict__ partial, Rank1 r1 = {}) {
    extern __shared__ float s_dyn[];  // [waves][C][2]
    const int cg = g.C / 8;
    const int c0 = ((int)threadIdx.x % cg) * 8;
    float mean[8], rstd[8], sc[8], sh[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        mean[j] = stats[c0 + j];
        rstd[j] = stats[g.C + c0 + j];
        sc[j] = stats[2 * g.C + c0 + j];
        sh[j] = stats[3 * g.C + c0 + j];
    }
    float a[8] = {}, b[8] = {};
    float w8[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) w8[j] = R1 ? r1.w1[c0 + j] : 0.f;
    const bool relu = act == LSS_ACT_RELU;
    constexpr int R = LSS_BN_STATS_R;
    for_rows_nhwc<R>(g, G, blockIdx.x, [&](const int* idx, int n) {
        float d[R][8], xv[R][8], yv[R][8];
#pragma unroll
        for (int u = 0; u < R; ++u) {
            if (u >= n) continue;
            load_dy8<R1>(dy, idx[u], c0, g, r1, w8, d[u]);
            ldv<8>(x + idx[u], xv[u]);
            if (relu && y) ldv<8>(y + idx[u], yv[u]);
        }
#pragma unroll
        for (int u = 0; u < R; ++u) {
            if (u >= n) continue;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float z = fmaf(xv[u][j], sc[j], sh[j]);
                const float gr = grad_pre(d[u][j], relu ? (y ? yv[u][j] : relu_out<T>(z)) : 0.f, z, act);
                a[j] += gr;
                b[j] = fmaf(gr, (xv[u][j] - mean[j]) * rstd[j], b[j]);
            }
        }
    });
    nhwc_block_sums(g, G, blockIdx.x, a, b, c0, (int)threadIdx.x < (kBlock / cg) * cg, s_dyn, partial);
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_bn_bwd_apply_nhwc(const T* __restrict__ dy, const T* __restrict__ x,
                                                              const T* __restrict__ y, BnGeo g,
                                                              const float* __restrict__ stats,
                                                              const float* __restrict__ coef, int act,
                                                              T* __restrict__ dx, T* __restrict__ dres) {
    extern __shared__ float s_dyn[];  // mean, rstd, scale, shift, mean(g), mean(g xhat): [6][C]
    for (int c = threadIdx.x; c < g.C; c += kBlock) {
#pragma unroll
        for (int k = 0; k < 4; ++k) s_dyn[k * g.C + c] = stats[k * g.C + c];
        s_dyn[4 * g.C + c] = coef[2 * c];
        s_dyn[5 * g.C + c] = coef[2 * c + 1];
    }
    __syncthreads();
    const long nv = (long)g.N * g.HW * g.C / 8;
    for (long e = (long)blockIdx.x * kBlock + threadIdx.x; e < nv; e += (long)gridDim.x * kBlock) {
        const size_t i = (size_t)e * 8;
        const int c0 = (int)(i % g.C);
        float d[8], xv[8], yv[8], o[8], gr[8];
        ldv<8>(dy + i, d);
        ldv<8>(x + i, xv);
        if (act == LSS_ACT_RELU && y) ldv<8>(y + i, yv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int c = c0 + j;
            const float sc = s_dyn[2 * g.C + c];
            const float z = fmaf(xv[j], sc, s_dyn[3 * g.C + c]);
            gr[j] = grad_pre(d[j], act == LSS_ACT_RELU ? (y ? yv[j] : relu_out<T>(z)) : 0.f, z, act);
            o[j] = sc * (gr[j] - s_dyn[4 * g.C + c] - (xv[j] - s_dyn[c]) * s_dyn[g.C + c] * s_dyn[5 * g.C + c]);
        }
        stv<8>(dx + i, o);
        if (dres) stv<8>(dres + i, gr);
    }
}

// Row-walking forms of the two apply passes (LSS_BN_ROWS, the default): block q of G takes the pixel rows
// [M q / G, M (q+1) / G) like the statistics kernels, a thread keeps one channel octet, so its
// per-channel coefficients sit in registers for all its rows (the grid-stride forms above re-read
// them from LDS for every vector), and R rows' loads are in flight per iteration.
#ifndef LSS_BN_ROWS
#define LSS_BN_ROWS 1
#endif
template <typename T>
__global__ __launch_bounds__(kBlock) void k_bn_apply_rows_nhwc(const T* __restrict__ x, const T* __restrict__ res, BnGeo g,
                                                               const float* __restrict__ stats, int act,
                                                               T* __restrict__ y) {
    constexpr int R = 4;
    const int c0 = ((int)threadIdx.x % (g.C >> 3)) * 8;
    float sc[8], sh[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        sc[j] = stats[2 * g.C + c0 + j];
        sh[j] = stats[3 * g.C + c0 + j];
    }
    for_rows_nhwc<R>(g, (int)gridDim.x, (int)blockIdx.x, [&](const int* idx, int n) {
        float v[R][8], rv[R][8];
#pragma unroll
        for (int u = 0; u < R; ++u)
            if (u < n) {
                ldv<8>(x + idx[u], v[u]);
                if (res) ldv<8>(res + idx[u], rv[u]);
            }
#pragma unroll
        for (int u = 0; u < R; ++u)
            if (u < n) {
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    float z = fmaf(v[u][j], sc[j], sh[j]);
                    if (res) z += rv[u][j];
                    v[u][j] = act_fwd(z, act);
                }
                stv<8>(y + idx[u], v[u]);
            }
    });
}

// dx = scale g + B x + K with B = -scale rstd mean(g xhat), K = -scale (mean(g) - mean rstd mean(g xhat))
// (the grid-stride form's scale (g - mean(g) - (x - mean) rstd mean(g xhat)) regrouped: 4 coefficients
// per channel held in registers)
template <typename T, bool R1 = false>
__global__ __launch_bounds__(kBlock) void k_bn_bwd_apply_rows_nhwc(const T* __restrict__ dy, const T* __restrict__ x,
                                                                   const T* __restrict__ y, BnGeo g,
                                                                   const float* __restrict__ stats,
                                                                   const float* __restrict__ coef, int act,
                                                                   T* __restrict__ dx, T* __restrict__ dres,
                                                                   Rank1 r1 = {}) {
    constexpr int R = 2;
    const int c0 = ((int)threadIdx.x % (g.C >> 3)) * 8;
    float sc[8], sh[8], kb[8], kk[8], w8[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) w8[j] = R1 ? r1.w1[c0 + j] : 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int c = c0 + j;
        const float mean = stats[c], rstd = stats[g.C + c];
        sc[j] = stats[2 * g.C + c];
        sh[j] = stats[3 * g.C + c];
        const float mg = coef[2 * c], mgx = coef[2 * c + 1];
        kb[j] = -sc[j] * rstd * mgx;
        kk[j] = -sc[j] * (mg - mean * rstd * mgx);
    }
    const bool relu = act == LSS_ACT_RELU;
    for_rows_nhwc<R>(g, (int)gridDim.x, (int)blockIdx.x, [&](const int* idx, int n) {
        float d[R][8], xv[R][8], yv[R][8];
#pragma unroll
        for (int u = 0; u < R; ++u)
            if (u < n) {
                load_dy8<R1>(dy, idx[u], c0, g, r1, w8, d[u]);
                ldv<8>(x + idx[u], xv[u]);
                if (relu && y) ldv<8>(y + idx[u], yv[u]);
            }
#pragma unroll
        for (int u = 0; u < R; ++u)
            if (u < n) {
                float o[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float z = fmaf(xv[u][j], sc[j], sh[j]);
                    const float gr = grad_pre(d[u][j], relu ? (y ? yv[u][j] : relu_out<T>(z)) : 0.f, z, act);
                    o[j] = fmaf(sc[j], gr, fmaf(kb[j], xv[u][j], kk[j]));
                    d[u][j] = gr;
                }
                stv<8>(dx + idx[u], o);
                if (dres) stv<8>(dres + idx[u], d[u]);
            }
    });
}

// ============================================================================= host side
inline int launch_status() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

inline bool bn_ok(const BnGeo& g, int layout) {
    if (g.N <= 0 || g.C <= 0 || g.HW <= 0 || (long)g.N * g.C * g.HW >= INT_MAX) return false;
    if (layout == LSS_CONV_NHWC) return g.C % 8 == 0 && g.C / 8 <= kBlock && kBlock % (g.C / 8) == 0;
    return layout == LSS_CONV_NCHW;
}

#ifndef LSS_BN_FUSED
#define LSS_BN_FUSED 1  // NCHW, one group per channel: statistics + apply in one launch (k_bn_fused_nchw)
#endif

// register-resident one-group kernels: bf16, V in {8, 4}, at most 8 vectors per thread
template <typename T> inline bool fused_reg(int V, long cnt) {
    return std::is_same<T, bf16>::value && (V == 8 || V == 4) && cnt <= 8 * kBlock;
}

inline int vec_nchw(int HW) { return HW % 8 == 0 ? 8 : (HW % 4 == 0 ? 4 : 1); }

#ifndef LSS_BN_CLUSTER
#define LSS_BN_CLUSTER 1  // NCHW, G > 1: the cluster kernels when a sync workspace is given (lss_bn_*2)
#endif

// vectors per thread the largest group of a channel needs
inline int cluster_it(int G, int V, const BnGeo& g) {
    const long imgs = (g.N + G - 1) / G;
    return (int)((imgs * (g.HW / V) + kBlock - 1) / kBlock);
}

// NCHW bf16 with several groups per channel, each group's vectors held in registers. Where it pays
// (c3 trunk, per-layer A/B of the step's graph replays against stats + apply, profiles/r06/
// bn_cluster_ab.txt): a block that has published waits for the whole channel, so a grid that does not
// fit the resident slots in one round (4 blocks per CU at the cluster kernels' 100-128 VGPRs) loses
// the overlap two launches give -- forward: 1,536 blocks 31-33 us vs 24-26, 4,608 blocks 86 vs 57;
// at <= 960 blocks 8.5-15.4 vs 11.1-16.9 us. The backward (two tensors read, three written or read
// again) also wins at 1,536-2,304 blocks of 3-12 images per group (30.6-40.6 vs 32.5-44.7 us), not at
// one image per group (G = 48 at 64 x 176: 43.9 vs 39.0; forward 768 blocks: 15.5 vs 14.2).
template <typename T> inline bool cluster_ok(const uint32_t* sync, int G, int V, const BnGeo& g, bool bwd) {
    if (!LSS_BN_CLUSTER || sync == nullptr || !std::is_same<T, bf16>::value || V != 8) return false;
    if (G < 2 || G > kBnClusterMaxG || g.C > kBnSyncMaxC) return false;
    const long blocks = (long)g.C * G;
    if (g.N / G < 2 || blocks > (bwd ? 2304 : 1024)) return false;
    const long imgs = (g.N + G - 1) / G;  // images of the largest group
    return imgs * (g.HW / V) <= (long)kBnClusterIT * kBlock;
}

inline int apply_blocks(const BnGeo& g) {  // grid-stride elementwise passes: up to 8 blocks per CU
    const long nv = (long)g.N * g.HW * g.C / 8;
    const long b = (nv + kBlock - 1) / kBlock;
    return (int)(b < 2048 ? b : 2048);
}

}  // namespace

extern "C" {

int lss_bn_groups(int32_t N, int32_t C, int32_t HW, int32_t layout) {
    const long per_chan = (long)N * HW;
    if (layout == LSS_CONV_NHWC) {
        // ~LSS_BN_NHWC_ELEMS elements per block, but at least LSS_BN_NHWC_GMIN blocks where the tensor
        // has >= 8 K elements for each
        const long tot = per_chan * C;
        long g = tot / LSS_BN_NHWC_ELEMS;
        const long gmin = std::min<long>(LSS_BN_NHWC_GMIN, tot / 8192);
        if (g < gmin) g = gmin;
        return (int)(g < 1 ? 1 : (g > kGroupsNhwc ? kGroupsNhwc : g));
    }
    const long g = per_chan / 8192;  // ~8 K elements of one channel per block
    return (int)(g < 1 ? 1 : (g > N ? N : g));
}

int lss_bn_sync_words(void) { return kBnSyncMaxC * kBnSyncStride + 1; }

int lss_bn_fwd(const void* x, const void* residual, int32_t dtype, int32_t layout, int32_t N, int32_t C, int32_t HW,
               const float* gamma, const float* beta, float eps, float momentum, float* running_mean,
               float* running_var, long long* num_batches_tracked, int32_t act, int32_t ngroups, float* partial,
               float* save_mean, float* save_rstd, float* scale, float* shift, void* y, void* stream) {
    return lss_bn_fwd2(x, residual, dtype, layout, N, C, HW, gamma, beta, eps, momentum, running_mean, running_var,
                       num_batches_tracked, act, ngroups, partial, save_mean, save_rstd, scale, shift, y, nullptr,
                       stream);
}

int lss_bn_fwd2(const void* x, const void* residual, int32_t dtype, int32_t layout, int32_t N, int32_t C, int32_t HW,
                const float* gamma, const float* beta, float eps, float momentum, float* running_mean,
                float* running_var, long long* num_batches_tracked, int32_t act, int32_t ngroups, float* partial,
                float* save_mean, float* save_rstd, float* scale, float* shift, void* y, uint32_t* sync,
                void* stream) {
    const BnGeo g{N, C, HW};
    // y == NULL (NHWC only): statistics and the running-stat update, no apply pass (a consumer that
    // applies scale / shift itself: lss_head1_fwd2)
    if (!x || (!y && layout != LSS_CONV_NHWC) || !partial || !save_mean || !save_rstd || !scale || !shift ||
        ngroups <= 0 || !bn_ok(g, layout))
        return LSS_CONV_EINVAL;
    if (act != LSS_ACT_NONE && act != LSS_ACT_RELU && act != LSS_ACT_SWISH) return LSS_CONV_EINVAL;
    // the saved statistics are one (4, C) array: mean, rstd, scale, shift
    if (save_rstd != save_mean + C || scale != save_mean + 2 * C || shift != save_mean + 3 * C) return LSS_CONV_EINVAL;
    if (layout == LSS_CONV_NHWC && ngroups > kMaxGroupsNhwc) return LSS_CONV_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    const BnParams P{gamma, beta, eps, momentum, running_mean, running_var, save_mean, num_batches_tracked};
    const int G = ngroups;
#define LSS_BN_FWD(T)                                                                                              \
    do {                                                                                                           \
        const T* xx = (const T*)x;                                                                                 \
        const T* rr = (const T*)residual;                                                                          \
        T* yy = (T*)y;                                                                                             \
        if (layout == LSS_CONV_NHWC) {                                                                             \
            const size_t lds = 2 * C * sizeof(float);                                                              \
            hipLaunchKernelGGL(k_bn_stats_nhwc<T>, dim3(G), dim3(kBlock), kNhwcStatsLds * C * sizeof(float), s, xx, \
                               g, G, partial);                                                                     \
            hipLaunchKernelGGL(k_bn_fold_nhwc<T>, dim3((C + 3) / 4), dim3(kBlock), 0, s, partial, G, xx, g, P);   \
            if (!yy) {                                                                                             \
            } else if (LSS_BN_ROWS)                                                                                \
                hipLaunchKernelGGL(k_bn_apply_rows_nhwc<T>, dim3(apply_blocks(g)), dim3(kBlock), 0, s, xx, rr, g,  \
                                   save_mean, (int)act, yy);                                                       \
            else                                                                                                   \
                hipLaunchKernelGGL(k_bn_apply_nhwc<T>, dim3(apply_blocks(g)), dim3(kBlock), lds, s, xx, rr, g,    \
                                   save_mean, (int)act, yy);                                                       \
        } else {                                                                                                   \
            const int V = vec_nchw(HW);                                                                            \
            const dim3 gr(C * G), bl(kBlock);                                                                      \
            const long cnt = (long)N * (HW / V);                                                                   \
            if (cluster_ok<T>(sync, G, V, g, false)) {                                                             \
                if (cluster_it(G, V, g) <= 6)                                                                      \
                    hipLaunchKernelGGL((k_bn_cluster_nchw<8, 6>), gr, bl, 0, s, (const bf16*)xx, (const bf16*)rr,  \
                                       g, G, partial, P, (int)act, (unsigned*)sync, (bf16*)yy);                    \
                else                                                                                               \
                    hipLaunchKernelGGL((k_bn_cluster_nchw<8, 8>), gr, bl, 0, s, (const bf16*)xx, (const bf16*)rr,  \
                                       g, G, partial, P, (int)act, (unsigned*)sync, (bf16*)yy);                    \
            } else if (G == 1 && LSS_BN_FUSED && fused_reg<T>(V, cnt)) {                                           \
                if (V == 8 && cnt <= 4 * kBlock)                                                                   \
                    hipLaunchKernelGGL((k_bn_fused_reg_nchw<8, 4>), gr, bl, 0, s, (const bf16*)xx,                \
                                       (const bf16*)rr, g, P, (int)act, (bf16*)yy);                                \
                else if (V == 8 && cnt <= 5 * kBlock)                                                              \
                    hipLaunchKernelGGL((k_bn_fused_reg_nchw<8, 5>), gr, bl, 0, s, (const bf16*)xx,                \
                                       (const bf16*)rr, g, P, (int)act, (bf16*)yy);                                \
                else if (V == 8)                                                                                   \
                    hipLaunchKernelGGL((k_bn_fused_reg_nchw<8, 8>), gr, bl, 0, s, (const bf16*)xx,                \
                                       (const bf16*)rr, g, P, (int)act, (bf16*)yy);                                \
                else if (cnt <= 4 * kBlock)                                                                        \
                    hipLaunchKernelGGL((k_bn_fused_reg_nchw<4, 4>), gr, bl, 0, s, (const bf16*)xx,                \
                                       (const bf16*)rr, g, P, (int)act, (bf16*)yy);                                \
                else                                                                                               \
                    hipLaunchKernelGGL((k_bn_fused_reg_nchw<4, 8>), gr, bl, 0, s, (const bf16*)xx,                \
                                       (const bf16*)rr, g, P, (int)act, (bf16*)yy);                                \
            } else if (G == 1 && LSS_BN_FUSED) {                                                                   \
                if (V == 8) hipLaunchKernelGGL((k_bn_fused_nchw<8, T>), gr, bl, 0, s, xx, rr, g, P, (int)act, yy); \
                else if (V == 4) hipLaunchKernelGGL((k_bn_fused_nchw<4, T>), gr, bl, 0, s, xx, rr, g, P, (int)act, \
                                                    yy);                                                           \
                else hipLaunchKernelGGL((k_bn_fused_nchw<1, T>), gr, bl, 0, s, xx, rr, g, P, (int)act, yy);        \
            } else if (V == 8) {                                                                                   \
                hipLaunchKernelGGL((k_bn_stats_nchw<8, T>), gr, bl, 0, s, xx, g, G, partial);                     \
                hipLaunchKernelGGL((k_bn_apply_nchw<8, T>), gr, bl, 0, s, xx, rr, g, G, partial, P, (int)act, yy); \
            } else if (V == 4) {                                                                                   \
                hipLaunchKernelGGL((k_bn_stats_nchw<4, T>), gr, bl, 0, s, xx, g, G, partial);                     \
                hipLaunchKernelGGL((k_bn_apply_nchw<4, T>), gr, bl, 0, s, xx, rr, g, G, partial, P, (int)act, yy); \
            } else {                                                                                               \
                hipLaunchKernelGGL((k_bn_stats_nchw<1, T>), gr, bl, 0, s, xx, g, G, partial);                     \
                hipLaunchKernelGGL((k_bn_apply_nchw<1, T>), gr, bl, 0, s, xx, rr, g, G, partial, P, (int)act, yy); \
            }                                                                                                      \
        }                                                                                                          \
    } while (0)
    if (dtype == LSS_CONV_F32) LSS_BN_FWD(float);
    else if (dtype == LSS_CONV_BF16) LSS_BN_FWD(bf16);
    else return LSS_CONV_EINVAL;
#undef LSS_BN_FWD
    return launch_status();
}

int lss_bn_bwd(const void* dy, const void* x, const void* y, int32_t dtype, int32_t layout, int32_t N, int32_t C,
               int32_t HW, const float* scale, const float* shift, const float* save_mean, const float* save_rstd,
               int32_t act, int32_t ngroups, float* partial, float* coef, float* dgamma, float* dbeta, void* dx,
               void* dresidual, void* stream) {
    return lss_bn_bwd2(dy, x, y, dtype, layout, N, C, HW, scale, shift, save_mean, save_rstd, act, ngroups, partial,
                       coef, dgamma, dbeta, dx, dresidual, nullptr, stream);
}

int lss_bn_bwd2(const void* dy, const void* x, const void* y, int32_t dtype, int32_t layout, int32_t N, int32_t C,
                int32_t HW, const float* scale, const float* shift, const float* save_mean, const float* save_rstd,
                int32_t act, int32_t ngroups, float* partial, float* coef, float* dgamma, float* dbeta, void* dx,
                void* dresidual, uint32_t* sync, void* stream) {
    const BnGeo g{N, C, HW};
    if (!dy || !x || !scale || !shift || !save_mean || !save_rstd || !partial || !coef || !dx || ngroups <= 0 ||
        !bn_ok(g, layout))
        return LSS_CONV_EINVAL;
    if (save_rstd != save_mean + C || scale != save_mean + 2 * C || shift != save_mean + 3 * C) return LSS_CONV_EINVAL;
    if (act == LSS_ACT_RELU && !y && layout != LSS_CONV_NHWC) return LSS_CONV_EINVAL;
    if (act != LSS_ACT_NONE && act != LSS_ACT_RELU && act != LSS_ACT_SWISH) return LSS_CONV_EINVAL;
    if (layout == LSS_CONV_NHWC && ngroups > kMaxGroupsNhwc) return LSS_CONV_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    const int G = ngroups;
    const float* stats = save_mean;
#define LSS_BN_BWD(T)                                                                                              \
    do {                                                                                                           \
        const T* d = (const T*)dy;                                                                                 \
        const T* xx = (const T*)x;                                                                                 \
        const T* yy = (const T*)y;                                                                                 \
        T* o = (T*)dx;                                                                                             \
        T* orr = (T*)dresidual;                                                                                    \
        if (layout == LSS_CONV_NHWC) {                                                                             \
            hipLaunchKernelGGL(k_bn_bwd_stats_nhwc<T>, dim3(G), dim3(kBlock), kNhwcStatsLds * C * sizeof(float), s, d, xx, yy, \
                               g, G, stats, (int)act, partial);                                                    \
            hipLaunchKernelGGL(k_bn_bwd_fold_nhwc, dim3((C + 3) / 4), dim3(kBlock), 0, s, partial, G, g, dgamma,  \
                               dbeta, coef);                                                                       \
            if (LSS_BN_ROWS)                                                                                       \
                hipLaunchKernelGGL(k_bn_bwd_apply_rows_nhwc<T>, dim3(apply_blocks(g)), dim3(kBlock), 0, s, d, xx, yy, \
                                   g, stats, coef, (int)act, o, orr);                                              \
            else                                                                                                   \
                hipLaunchKernelGGL(k_bn_bwd_apply_nhwc<T>, dim3(apply_blocks(g)), dim3(kBlock), 6 * C * sizeof(float), \
                                   s, d, xx, yy, g, stats, coef, (int)act, o, orr);                                \
        } else {                                                                                                   \
            const int V = vec_nchw(HW);                                                                            \
            const dim3 gr(C * G), bl(kBlock);                                                                      \
            const long cnt = (long)N * (HW / V);                                                                   \
            if (cluster_ok<T>(sync, G, V, g, true)) {                                                              \
                const bf16 *db = (const bf16*)d, *xb = (const bf16*)xx, *yb = (const bf16*)yy;                     \
                const bool it6 = cluster_it(G, V, g) <= 6;                                                         \
                if (act == LSS_ACT_RELU && it6)                                                                    \
                    hipLaunchKernelGGL((k_bn_bwd_cluster_nchw<8, 6, true>), gr, bl, 0, s, db, xb, yb, g, G, stats, \
                                       partial, (int)act, (unsigned*)sync, dgamma, dbeta, (bf16*)o, (bf16*)orr);   \
                else if (act == LSS_ACT_RELU)                                                                      \
                    hipLaunchKernelGGL((k_bn_bwd_cluster_nchw<8, 8, true>), gr, bl, 0, s, db, xb, yb, g, G, stats, \
                                       partial, (int)act, (unsigned*)sync, dgamma, dbeta, (bf16*)o, (bf16*)orr);   \
                else if (it6)                                                                                      \
                    hipLaunchKernelGGL((k_bn_bwd_cluster_nchw<8, 6, false>), gr, bl, 0, s, db, xb, yb, g, G,       \
                                       stats, partial, (int)act, (unsigned*)sync, dgamma, dbeta, (bf16*)o,         \
                                       (bf16*)orr);                                                                \
                else                                                                                               \
                    hipLaunchKernelGGL((k_bn_bwd_cluster_nchw<8, 8, false>), gr, bl, 0, s, db, xb, yb, g, G,       \
                                       stats, partial, (int)act, (unsigned*)sync, dgamma, dbeta, (bf16*)o,         \
                                       (bf16*)orr);                                                                \
            } else if (G == 1 && LSS_BN_FUSED && fused_reg<T>(V, cnt)) {                                           \
                const bf16 *db = (const bf16*)d, *xb = (const bf16*)xx, *yb = (const bf16*)yy;                     \
                if (V == 8 && cnt <= 4 * kBlock)                                                                   \
                    hipLaunchKernelGGL((k_bn_bwd_fused_reg_nchw<8, 4>), gr, bl, 0, s, db, xb, yb, g, stats,       \
                                       (int)act, dgamma, dbeta, (bf16*)o, (bf16*)orr);                             \
                else if (V == 8 && cnt <= 5 * kBlock)                                                              \
                    hipLaunchKernelGGL((k_bn_bwd_fused_reg_nchw<8, 5>), gr, bl, 0, s, db, xb, yb, g, stats,       \
                                       (int)act, dgamma, dbeta, (bf16*)o, (bf16*)orr);                             \
                else if (V == 8)                                                                                   \
                    hipLaunchKernelGGL((k_bn_bwd_fused_reg_nchw<8, 8>), gr, bl, 0, s, db, xb, yb, g, stats,       \
                                       (int)act, dgamma, dbeta, (bf16*)o, (bf16*)orr);                             \
                else if (cnt <= 4 * kBlock)                                                                        \
                    hipLaunchKernelGGL((k_bn_bwd_fused_reg_nchw<4, 4>), gr, bl, 0, s, db, xb, yb, g, stats,       \
                                       (int)act, dgamma, dbeta, (bf16*)o, (bf16*)orr);                             \
                else                                                                                               \
                    hipLaunchKernelGGL((k_bn_bwd_fused_reg_nchw<4, 8>), gr, bl, 0, s, db, xb, yb, g, stats,       \
                                       (int)act, dgamma, dbeta, (bf16*)o, (bf16*)orr);                             \
            } else if (G == 1 && LSS_BN_FUSED) {                                                                   \
                if (V == 8)                                                                                        \
                    hipLaunchKernelGGL((k_bn_bwd_fused_nchw<8, T>), gr, bl, 0, s, d, xx, yy, g, stats, (int)act,  \
                                       dgamma, dbeta, o, orr);                                                     \
                else if (V == 4)                                                                                   \
                    hipLaunchKernelGGL((k_bn_bwd_fused_nchw<4, T>), gr, bl, 0, s, d, xx, yy, g, stats, (int)act,  \
                                       dgamma, dbeta, o, orr);                                                     \
                else                                                                                               \
                    hipLaunchKernelGGL((k_bn_bwd_fused_nchw<1, T>), gr, bl, 0, s, d, xx, yy, g, stats, (int)act,  \
                                       dgamma, dbeta, o, orr);                                                     \
            } else if (V == 8) {                                                                                   \
                hipLaunchKernelGGL((k_bn_bwd_stats_nchw<8, T>), gr, bl, 0, s, d, xx, yy, g, G, stats, (int)act,    \
                                   partial);                                                                       \
                hipLaunchKernelGGL((k_bn_bwd_apply_nchw<8, T>), gr, bl, 0, s, d, xx, yy, g, G, stats, partial,    \
                                   (int)act, dgamma, dbeta, o, orr);                                               \
            } else if (V == 4) {                                                                                   \
                hipLaunchKernelGGL((k_bn_bwd_stats_nchw<4, T>), gr, bl, 0, s, d, xx, yy, g, G, stats, (int)act,    \
                                   partial);                                                                       \
                hipLaunchKernelGGL((k_bn_bwd_apply_nchw<4, T>), gr, bl, 0, s, d, xx, yy, g, G, stats, partial,    \
                                   (int)act, dgamma, dbeta, o, orr);                                               \
            } else {                                                                                               \
                hipLaunchKernelGGL((k_bn_bwd_stats_nchw<1, T>), gr, bl, 0, s, d, xx, yy, g, G, stats, (int)act,    \
                                   partial);                                                                       \
                hipLaunchKernelGGL((k_bn_bwd_apply_nchw<1, T>), gr, bl, 0, s, d, xx, yy, g, G, stats, partial,    \
                                   (int)act, dgamma, dbeta, o, orr);                                               \
            }                                                                                                      \
        }                                                                                                          \
    } while (0)
    if (dtype == LSS_CONV_F32) LSS_BN_BWD(float);
    else if (dtype == LSS_CONV_BF16) LSS_BN_BWD(bf16);
    else return LSS_CONV_EINVAL;
#undef LSS_BN_BWD
    return launch_status();
}


int lss_bn_bwd_rank1(const void* g1, const float* w1, const void* x, int32_t N, int32_t C, int32_t HW,
                     const float* scale, const float* shift, const float* save_mean, const float* save_rstd,
                     int32_t act, int32_t ngroups, float* partial, float* coef, float* dgamma, float* dbeta, void* dx,
                     void* stream) {
    const BnGeo g{N, C, HW};
    if (!g1 || !w1 || !x || !scale || !shift || !save_mean || !save_rstd || !partial || !coef || !dx || ngroups <= 0 ||
        ngroups > kMaxGroupsNhwc || !bn_ok(g, LSS_CONV_NHWC))
        return LSS_CONV_EINVAL;
    if (save_rstd != save_mean + C || scale != save_mean + 2 * C || shift != save_mean + 3 * C) return LSS_CONV_EINVAL;
    if (act != LSS_ACT_NONE && act != LSS_ACT_RELU) return LSS_CONV_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    const int G = ngroups;
    const Rank1 r1{(const bf16*)g1, w1};
    const bf16* xx = (const bf16*)x;
    hipLaunchKernelGGL((k_bn_bwd_stats_nhwc<bf16, true>), dim3(G), dim3(kBlock), kNhwcStatsLds * C * sizeof(float), s,
                       (const bf16*)nullptr, xx, (const bf16*)nullptr, g, G, save_mean, (int)act, partial, r1);
    hipLaunchKernelGGL(k_bn_bwd_fold_nhwc, dim3((C + 3) / 4), dim3(kBlock), 0, s, partial, G, g, dgamma, dbeta, coef);
    hipLaunchKernelGGL((k_bn_bwd_apply_rows_nhwc<bf16, true>), dim3(apply_blocks(g)), dim3(kBlock), 0, s,
                       (const bf16*)nullptr, xx, (const bf16*)nullptr, g, save_mean, coef, (int)act, (bf16*)dx,
                       (bf16*)nullptr, r1);
    return launch_status();
}

}  // extern "C"

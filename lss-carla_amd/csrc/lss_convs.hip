// lss_convs.hip -- gfx950 kernels for the conv stack in front of the Lift-Splat hot path: the
// depthwise convolutions of CamEncode's EfficientNet-B0 trunk (src/models.py:43, 63-84; 16 MBConv
// blocks, 3x3 / 5x5, stride 1 / 2, TF "same" padding). MIOpen has no bf16 NCHW depthwise solver and
// falls back to naive kernels (≈5 ms of a 27 ms training step at config 3).
//
// NCHW planes, fp32 accumulation, activations fp32 or bf16, weights fp32 (the parameter itself: no
// per-step cast, and the weight gradient stays fp32).
//
// Forward / stride-1 backward-data: a thread owns a strip of TH output rows of one column; lanes run
// along the row, so every input-row load instruction of a wave is contiguous, and each input row
// loaded into registers feeds every output of the strip it overlaps. Index math is 32-bit (element
// counts are checked < 2^31); a wave whose lanes share one channel reads the weights with scalar
// loads. Stride-1 backward-data is the
// forward correlation with the kernel flipped and the padding mirrored. Stride-2 backward-data: a
// thread per 2 x 4 input elements with compile-time tap offsets. Backward-weight: a block per (channel, group
// of images) accumulates the K*K tap sums of its elements in registers, reduces them over the block
// in a fixed order and writes one partial per group; the caller sums the groups.

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <algorithm>
#include <type_traits>
#include <limits.h>
#include <stdint.h>

#include "lss_convs.h"

// The library is built with -ffp-contract=off for the geometry's reference op order (lss_hip.hip);
// the conv-stack kernels here have no bit-exact contract, so they keep FMA contraction.
#pragma clang fp contract(fast)

namespace {

using bf16 = __hip_bfloat16;
constexpr int kBlock = 256;
constexpr int kWave = 64;
// output tile per thread (rows x columns)
template <int S> struct Tile { static constexpr int TH = S == 1 ? 8 : 4, TW = S == 1 ? 4 : 2; };

__device__ __forceinline__ float ld(const float* p) { return *p; }
__device__ __forceinline__ float ld(const bf16* p) { return __bfloat162float(*p); }
__device__ __forceinline__ void st(float* p, float v) { *p = v; }
__device__ __forceinline__ void st(bf16* p, float v) { *p = __float2bfloat16(v); }

// 8 bf16 <-> fp32 (bf16 -> fp32 is exact; fp32 -> bf16 rounds to nearest even)
__device__ __forceinline__ void unpack8(const uint4& u, float* o) {
    const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        o[2 * i] = __uint_as_float(w[i] << 16);
        o[2 * i + 1] = __uint_as_float(w[i] & 0xFFFF0000u);
    }
}
__device__ __forceinline__ unsigned pack2(float a, float b) {
    const bf16 x = __float2bfloat16(a), y = __float2bfloat16(b);
    return (unsigned)*reinterpret_cast<const unsigned short*>(&x) |
           ((unsigned)*reinterpret_cast<const unsigned short*>(&y) << 16);
}

struct DwGeo {
    int C, Hi, Wi, Ho, Wo, pt, pl, nplanes;  // input (Hi, Wi) -> output (Ho, Wo); nplanes = N * C
};

// Weights of channel c for a wave: when every lane of the wave works on the same channel (planes
// of >= 64 outputs per row strip), the channel index is wave-uniform and the weights come in with
// scalar loads (SGPR operands of the FMAs); otherwise per lane.
template <int K, typename F>
__device__ __forceinline__ void with_weights(const float* __restrict__ w, int c, bool flip, F&& body) {
    const int cu = __builtin_amdgcn_readfirstlane(c);
    if (__ballot(c != cu) == 0) {
        const float* wc = w + (size_t)cu * K * K;
        float wk[K * K];
#pragma unroll
        for (int i = 0; i < K * K; ++i) wk[i] = wc[flip ? K * K - 1 - i : i];
        body(wk);
    } else {
        const float* wc = w + (size_t)c * K * K;
        float wk[K * K];
#pragma unroll
        for (int i = 0; i < K * K; ++i) wk[i] = wc[flip ? K * K - 1 - i : i];
        body(wk);
    }
}

// y[p][oh][ow] = sum_{kh, kw} x[p][oh*S - pt + kh][ow*S - pl + kw] * w[c][kh][kw] (zero outside x);
// flip: w[c][K-1-kh][K-1-kw] (stride-1 backward-data). Thread = (plane, TH x TW output tile): each
// input row segment it loads ((TW-1)*S + K values) feeds every output of the tile under it.
template <int K, int S, int TH, int TW, typename T>
__global__ __launch_bounds__(kBlock) void k_dw_fwd(const T* __restrict__ x, const float* __restrict__ w, DwGeo g,
                                                   int flip, T* __restrict__ y) {
    const int t = blockIdx.x * kBlock + threadIdx.x;
    const int ncol = (g.Wo + TW - 1) / TW, nrow = (g.Ho + TH - 1) / TH;
    const int per_plane = nrow * ncol;
    const bool live = t < g.nplanes * per_plane;
    const int plane = live ? t / per_plane : 0;
    const int rem = t - plane * per_plane;
    const int tr = rem / ncol, tc = rem - tr * ncol;
    const int c = plane % g.C;
    const int oh0 = tr * TH, ow0 = tc * TW;
    const int ih0 = oh0 * S - g.pt, iw0 = ow0 * S - g.pl;
    const T* xp = x + (size_t)plane * g.Hi * g.Wi;
    with_weights<K>(w, c, flip != 0, [&](const float* wk) {
        if (!live) return;
        float acc[TH][TW];
#pragma unroll
        for (int i = 0; i < TH; ++i)
#pragma unroll
            for (int j = 0; j < TW; ++j) acc[i][j] = 0.f;
        constexpr int R = (TH - 1) * S + K, CW = (TW - 1) * S + K;
#pragma unroll
        for (int rr = 0; rr < R; ++rr) {
            const int ih = ih0 + rr;
            const bool row_ok = ih >= 0 && ih < g.Hi;
            float v[CW];
#pragma unroll
            for (int q = 0; q < CW; ++q) {
                const int iw = iw0 + q;
                v[q] = (row_ok && iw >= 0 && iw < g.Wi) ? ld(xp + ih * g.Wi + iw) : 0.f;
            }
#pragma unroll
            for (int i = 0; i < TH; ++i) {
                const int kh = rr - i * S;
                if (kh >= 0 && kh < K) {
#pragma unroll
                    for (int j = 0; j < TW; ++j)
#pragma unroll
                        for (int kw = 0; kw < K; ++kw) acc[i][j] = fmaf(v[j * S + kw], wk[kh * K + kw], acc[i][j]);
                }
            }
        }
        T* yp = y + (size_t)plane * g.Ho * g.Wo;
#pragma unroll
        for (int i = 0; i < TH; ++i)
#pragma unroll
            for (int j = 0; j < TW; ++j)
                if (oh0 + i < g.Ho && ow0 + j < g.Wo) st(yp + (oh0 + i) * g.Wo + ow0 + j, acc[i][j]);
    });
}

// Stride-2 backward-data. Thread = 2 rows x 4 columns of dx: ih = 2m + a, iw = 4j + b. With
// pt = 2 PT2 + PT1, pl = 2 PL2 + PL1 (PT1, PL1 template parameters) the taps that reach dx[ih][iw]
// have kh = a + PT1 (mod 2), kw = b + PL1 (mod 2), at dy[m + PT2 + (a + PT1 - kh) / 2]
// [2j + PL2 + (b + PL1 - kw) / 2]: every offset is a compile-time constant, so the thread loads one
// small dy window and runs straight-line FMAs. g describes the forward conv.
template <int K, int PT1, int PL1, typename T>
__global__ __launch_bounds__(kBlock) void k_dw_bwd_data_s2(const T* __restrict__ dy, const float* __restrict__ w,
                                                           DwGeo g, T* __restrict__ dx) {
    constexpr int H0 = -(K - 1) / 2, H1 = 1;      // dy row offsets reached (relative to m + PT2)
    constexpr int W0 = -(K - 1) / 2, W1 = 2;      // dy column offsets reached (relative to 2j + PL2)
    const int t = blockIdx.x * kBlock + threadIdx.x;
    const int ncol = (g.Wi + 3) / 4, nrow = (g.Hi + 1) / 2;
    const int per_plane = nrow * ncol;
    const bool live = t < g.nplanes * per_plane;
    const int plane = live ? t / per_plane : 0;
    const int rem = t - plane * per_plane;
    const int m = rem / ncol, j = rem - m * ncol;
    const int c = plane % g.C;
    const int hb = m + (g.pt >> 1), wb = 2 * j + (g.pl >> 1);
    const T* dp = dy + (size_t)plane * g.Ho * g.Wo;
    with_weights<K>(w, c, false, [&](const float* wk) {
        if (!live) return;
        float win[H1 - H0 + 1][W1 - W0 + 1];
#pragma unroll
        for (int r = H0; r <= H1; ++r) {
            const int oh = hb + r;
#pragma unroll
            for (int q = W0; q <= W1; ++q) {
                const int ow = wb + q;
                win[r - H0][q - W0] = (oh >= 0 && oh < g.Ho && ow >= 0 && ow < g.Wo) ? ld(dp + oh * g.Wo + ow) : 0.f;
            }
        }
        T* xp = dx + (size_t)plane * g.Hi * g.Wi;
#pragma unroll
        for (int a = 0; a < 2; ++a) {
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                float acc = 0.f;
#pragma unroll
                for (int kh = (a + PT1) & 1; kh < K; kh += 2)
#pragma unroll
                    for (int kw = (b + PL1) & 1; kw < K; kw += 2)
                        acc = fmaf(win[(a + PT1 - kh) / 2 - H0][(b + PL1 - kw) / 2 - W0], wk[kh * K + kw], acc);
                const int ih = 2 * m + a, iw = 4 * j + b;
                if (ih < g.Hi && iw < g.Wi) st(xp + ih * g.Wi + iw, acc);
            }
        }
    });
}

// Weight-gradient fold (optional, DwFold.sync != NULL): the ngroups partials of a channel are summed by the
// LAST of its blocks to finish, in group order, into dw[c][tap] -- the separate fold launch (a torch sum,
// 5-8 us at c3) is gone. Hand-off as the batch-norm cluster kernels': the partials written through with
// agent-scope stores and retired (vmcnt counts stores) before the agent-scope counter add; the last block
// reads them with agent-scope loads and re-zeroes the counter. Nothing waits, so nothing can stall. The
// counter of channel c is word c * kDwSyncStride + 2 of the batch-norm sync workspace (lss_bn_sync_words:
// zero-filled, left zero-filled by every user; words 0 and 1 of a channel's line are the BN clusters').
struct DwFold {
    unsigned* sync;
    float* dw;
};
constexpr int kDwSyncStride = 32;
constexpr int kDwSyncMaxC = 4096;
template <int KK>
__device__ __forceinline__ void dw_finish(float* __restrict__ partial, int c, int q, int ngroups, float v,
                                          const DwFold& f) {
    const int t = threadIdx.x;
    const size_t base = (size_t)c * ngroups * KK;
    if (!f.sync) {
        if (t < KK) partial[base + (size_t)q * KK + t] = v;
        return;
    }
    if (ngroups == 1) {  // the block is the channel: no hand-off
        if (t < KK) f.dw[(size_t)c * KK + t] = v;
        return;
    }
    if (t >= kWave) return;  // wave 0 (KK <= 25 lanes hold the block's values)
    unsigned* pu = reinterpret_cast<unsigned*>(partial);
    if (t < KK) __hip_atomic_store(pu + base + (size_t)q * KK + t, __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's partial stores retired
    unsigned* ctr = f.sync + (size_t)c * kDwSyncStride + 2;
    int last = 0;
    if (t == 0) last = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)ngroups - 1u;
    last = __shfl(last, 0, kWave);
    if (!last) return;
    // lanes over groups (each lane's KK partials loaded together), then a butterfly per tap: fixed order
    float a[KK];
#pragma unroll
    for (int k = 0; k < KK; ++k) a[k] = 0.f;
    for (int qq = t; qq < ngroups; qq += kWave) {
        unsigned u[KK];
#pragma unroll
        for (int k = 0; k < KK; ++k)
            u[k] = __hip_atomic_load(pu + base + (size_t)qq * KK + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int k = 0; k < KK; ++k) a[k] += __uint_as_float(u[k]);
    }
    float mine = 0.f;
#pragma unroll
    for (int k = 0; k < KK; ++k) {
        float s = a[k];
#pragma unroll
        for (int o = kWave / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, kWave);
        if (t == k) mine = s;
    }
    if (t < KK) f.dw[(size_t)c * KK + t] = mine;
    if (t == 0) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Backward-weight partials: block (group q, channel c) sums, over images n in its group and every
// output element, dy[n][c][oh][ow] * x[n][c][oh*S - pt + kh][ow*S - pl + kw] for each tap; a thread
// takes TH x TW output tiles of the group's flat (image, tile) space.
// partial[(c * ngroups + q) * K*K + tap]; fixed reduction order (wave shuffles, then waves in order).
template <int K, int S, int TH, int TW, typename T>
__global__ __launch_bounds__(kBlock) void k_dw_bwd_weight(const T* __restrict__ x, const T* __restrict__ dy, DwGeo g,
                                                          int nimg, int ngroups, float* __restrict__ partial,
                                                          DwFold fold) {
    __shared__ float s_red[kBlock / kWave][K * K];
    const int c = blockIdx.x % g.C, q = blockIdx.x / g.C;
    const int n0 = (int)((long)nimg * q / ngroups), n1 = (int)((long)nimg * (q + 1) / ngroups);
    const int ncol = (g.Wo + TW - 1) / TW, nrow = (g.Ho + TH - 1) / TH;
    const int per_img = nrow * ncol;
    const int count = per_img * (n1 - n0);
    float acc[K * K];
#pragma unroll
    for (int i = 0; i < K * K; ++i) acc[i] = 0.f;
    constexpr int R = (TH - 1) * S + K, CW = (TW - 1) * S + K;
    for (int e = threadIdx.x; e < count; e += kBlock) {
        const int nl = e / per_img;
        const int rem = e - nl * per_img;
        const int tr = rem / ncol, tc = rem - tr * ncol;
        const int plane = (n0 + nl) * g.C + c;
        const T* xp = x + (size_t)plane * g.Hi * g.Wi;
        const T* dp = dy + (size_t)plane * g.Ho * g.Wo;
        const int oh0 = tr * TH, ow0 = tc * TW;
        float d[TH][TW];
#pragma unroll
        for (int i = 0; i < TH; ++i)
#pragma unroll
            for (int j = 0; j < TW; ++j)
                d[i][j] = (oh0 + i < g.Ho && ow0 + j < g.Wo) ? ld(dp + (oh0 + i) * g.Wo + ow0 + j) : 0.f;
        const int ih0 = oh0 * S - g.pt, iw0 = ow0 * S - g.pl;
#pragma unroll
        for (int rr = 0; rr < R; ++rr) {
            const int ih = ih0 + rr;
            const bool row_ok = ih >= 0 && ih < g.Hi;
            float v[CW];
#pragma unroll
            for (int qq = 0; qq < CW; ++qq) {
                const int iw = iw0 + qq;
                v[qq] = (row_ok && iw >= 0 && iw < g.Wi) ? ld(xp + ih * g.Wi + iw) : 0.f;
            }
#pragma unroll
            for (int i = 0; i < TH; ++i) {
                const int kh = rr - i * S;
                if (kh >= 0 && kh < K) {
#pragma unroll
                    for (int j = 0; j < TW; ++j)
#pragma unroll
                        for (int kw = 0; kw < K; ++kw)
                            acc[kh * K + kw] = fmaf(d[i][j], v[j * S + kw], acc[kh * K + kw]);
                }
            }
        }
    }
    const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
#pragma unroll
    for (int i = 0; i < K * K; ++i) {
        float v = acc[i];
#pragma unroll
        for (int o = kWave / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
        if (lane == 0) s_red[wave][i] = v;
    }
    __syncthreads();
    float s = 0.f;
    if (threadIdx.x < K * K) {
#pragma unroll
        for (int jw = 0; jw < kBlock / kWave; ++jw) s += s_red[jw][threadIdx.x];
    }
    dw_finish<K * K>(partial, c, q, ngroups, s, fold);
}

inline int blocks_for(long n) { return (int)((n + kBlock - 1) / kBlock); }

inline int launch_status() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

inline bool geo_ok(int N, int C, int Hi, int Wi, int K, int S, int Ho, int Wo) {
    return N > 0 && C > 0 && Hi > 0 && Wi > 0 && Ho > 0 && Wo > 0 && (K == 3 || K == 5) && (S == 1 || S == 2) &&
           (long)N * C * Hi * Wi < INT_MAX && (long)N * C * Ho * Wo < INT_MAX;
}

// ---- LDS-staged depthwise kernels (round 5). The kernels above read every input element about twice
// with 2-byte loads whose lanes stride by the thread tile (4 or 8 bytes apart): the load count, not
// the bytes, bounded them (10-20 % of HBM on the trunk's large planes). Here a block stages a band of
// rows of PB planes into LDS (fp32, zero-padded so the taps need no bounds checks), with 16-B loads
// when a row holds a multiple of 8 elements and coalesced 2-B / 4-B loads otherwise; each thread then
// computes row segments of SEG consecutive outputs (SEG | Wo: one vector store per segment) from LDS.
#ifndef LSS_DW_LDS
#define LSS_DW_LDS 1  // experiment switch: 0 = the register-tiled kernels above
#endif
constexpr int kDwLdsFloats = 8192;  // staged input per block (32 KB)

struct DwBand {
    int BHo, PB, LW, LHmax, nbands;  // output rows per band, planes per block, LDS row stride / rows
};

// "v if c else 0" without a branch (the mask laundered through an empty asm, so the compiler cannot
// sink the load that produced v into a conditional block: such blocks serialise loads that should all
// be in flight together)
__device__ __forceinline__ unsigned dw_keep_mask(bool c) {
    unsigned m = c ? 0xFFFFFFFFu : 0u;
    asm("" : "+v"(m));
    return m;
}
__device__ __forceinline__ uint4 dw_keep(bool c, uint4 v) {
    const unsigned m = dw_keep_mask(c);
    return make_uint4(v.x & m, v.y & m, v.z & m, v.w & m);
}

// LDS column of input column iw: iw + kDwCol (so the 8-element chunks of a row land 8-B aligned:
// vector LDS writes); the left padding columns sit just below kDwCol, zero-filled with the right ones.
constexpr int kDwCol = 4;
// staged 16-B input chunks per thread per round: every load of a round in flight together (the loop
// that loaded, converted and wrote one chunk per iteration waited a memory round trip per iteration)
constexpr int kDwStageU = 8;

// Stage np planes (global plane stride gps elements) x LH rows from input row ih0 into LDS planes of
// lps floats (row stride LW): LDS (pl, r, c) = x[plane pl][ih0 + r][c - kDwCol], zero outside x.
template <typename T>
__device__ __forceinline__ void dw_stage(const T* __restrict__ xp, size_t gps, int np, int Hi, int Wi, int ih0, int LH,
                                         int LW, int lps, float* __restrict__ dst) {
    if (Wi % 8 == 0) {  // 8-element row chunks: 16-B (bf16) / 2 x 16-B (fp32) loads, all of a round in flight
        const int cpr = Wi / 8, per = LH * cpr, n = np * per;
        constexpr int U = sizeof(T) == 2 ? kDwStageU : kDwStageU / 2;
        constexpr int NV = sizeof(T) == 2 ? 1 : 2;  // 16-B pieces per chunk
        for (int i0 = threadIdx.x; i0 < n; i0 += U * kBlock) {
            uint4 raw[U][NV];
            const int nu = (n - (i0 - (int)threadIdx.x) + kBlock - 1) / kBlock;  // loads this round (block-uniform)
#pragma unroll
            for (int u = 0; u < U; ++u) {  // clamped addresses, unconditional loads, masked values
                if (u >= nu) break;
                const int i = min(i0 + u * kBlock, n - 1);
                const int pl = i / per, rem = i - pl * per, r = rem / cpr, ch = rem - r * cpr;
                const int ih = ih0 + r;
                const bool ok = ih >= 0 && ih < Hi;
                const uint4* src = reinterpret_cast<const uint4*>(xp + pl * gps + (size_t)min(max(ih, 0), Hi - 1) * Wi + 8 * ch);
#pragma unroll
                for (int h = 0; h < NV; ++h) raw[u][h] = dw_keep(ok, src[h]);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {  // every load issued before the first LDS write (no sinking)
                if (u >= nu) break;
#pragma unroll
                for (int h = 0; h < NV; ++h) asm volatile("" : : "v"(raw[u][h].x), "v"(raw[u][h].y), "v"(raw[u][h].z), "v"(raw[u][h].w));
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {  // (a clamped chunk rewrites chunk n - 1 with its own values)
                if (u >= nu) break;
                const int i = min(i0 + u * kBlock, n - 1);
                const int pl = i / per, rem = i - pl * per, r = rem / cpr, ch = rem - r * cpr;
                float2* d = reinterpret_cast<float2*>(dst + pl * lps + r * LW + kDwCol + 8 * ch);  // 8-B aligned
                float v[8];
                if constexpr (sizeof(T) == 2) {
                    unpack8(raw[u][0], v);
                } else {
                    const float4 a = __builtin_bit_cast(float4, raw[u][0]), b = __builtin_bit_cast(float4, raw[u][1]);
                    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) d[k] = make_float2(v[2 * k], v[2 * k + 1]);
            }
        }
        const int npad = LW - Wi;  // columns [0, kDwCol) and [kDwCol + Wi, LW)
        for (int i = threadIdx.x; i < np * LH * npad; i += kBlock) {
            const int pr = i / npad, k = i - pr * npad;
            const int pl = pr / LH, r = pr - pl * LH;
            dst[pl * lps + r * LW + (k < kDwCol ? k : Wi + k)] = 0.f;
        }
    } else {
        for (int i = threadIdx.x; i < np * LH * LW; i += kBlock) {
            const int pr = i / LW, c = i - pr * LW;
            const int pl = pr / LH, r = pr - pl * LH;
            const int ih = ih0 + r, iw = c - kDwCol;
            dst[pl * lps + r * LW + c] =
                (ih >= 0 && ih < Hi && iw >= 0 && iw < Wi) ? ld(xp + pl * gps + (size_t)ih * Wi + iw) : 0.f;
        }
    }
}

template <int SEG, typename T>
__device__ __forceinline__ void store_seg(T* __restrict__ p, const float* v, int n) {
    if (n == SEG) {
        if constexpr (sizeof(T) == 2 && SEG == 8) {
            *reinterpret_cast<uint4*>(p) = make_uint4(pack2(v[0], v[1]), pack2(v[2], v[3]), pack2(v[4], v[5]), pack2(v[6], v[7]));
            return;
        } else if constexpr (sizeof(T) == 2 && SEG == 4) {
            *reinterpret_cast<uint2*>(p) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
            return;
        } else if constexpr (sizeof(T) == 2 && SEG == 2) {
            *reinterpret_cast<unsigned*>(p) = pack2(v[0], v[1]);
            return;
        } else if constexpr (sizeof(T) == 4 && SEG % 4 == 0) {
#pragma unroll
            for (int k = 0; k < SEG; k += 4) *reinterpret_cast<float4*>(p + k) = make_float4(v[k], v[k + 1], v[k + 2], v[k + 3]);
            return;
        }
    }
#pragma unroll
    for (int k = 0; k < SEG; ++k)
        if (k < n) st(p + k, v[k]);
}

template <int SEG, typename T>
__device__ __forceinline__ void load_seg(const T* __restrict__ p, float* v, int n) {
    if (n == SEG) {
        if constexpr (sizeof(T) == 2 && SEG == 8) {
            unpack8(*reinterpret_cast<const uint4*>(p), v);
            return;
        } else if constexpr (sizeof(T) == 2 && SEG == 4) {
            const uint2 r = *reinterpret_cast<const uint2*>(p);
            v[0] = __uint_as_float(r.x << 16); v[1] = __uint_as_float(r.x & 0xFFFF0000u);
            v[2] = __uint_as_float(r.y << 16); v[3] = __uint_as_float(r.y & 0xFFFF0000u);
            return;
        } else if constexpr (sizeof(T) == 4 && SEG % 4 == 0) {
#pragma unroll
            for (int k = 0; k < SEG; k += 4) {
                const float4 a = *reinterpret_cast<const float4*>(p + k);
                v[k] = a.x; v[k + 1] = a.y; v[k + 2] = a.z; v[k + 3] = a.w;
            }
            return;
        }
    }
#pragma unroll
    for (int k = 0; k < SEG; ++k) v[k] = k < n ? ld(p + k) : 0.f;
}

template <typename T>
__device__ __forceinline__ void dw_stage_seg(const T* __restrict__ xp, int Hi, int Wi, int ih0, int LH, int LW, int pl,
                                         bool vec8, float* __restrict__ dst) {
    // LDS rows r = input rows ih0 + r, columns c = input columns c - pl; zero outside the input
    if (vec8) {  // Wi % 8 == 0: 8-element row chunks, 16-B (bf16) loads; the pad columns separately
        const int cpr = Wi / 8;
        for (int i = threadIdx.x; i < LH * cpr; i += kBlock) {
            const int r = i / cpr, ch = i - r * cpr;
            const int ih = ih0 + r;
            float v[8];
            if (ih >= 0 && ih < Hi) {
                const T* src = xp + (size_t)ih * Wi + 8 * ch;
                if constexpr (sizeof(T) == 2) {
                    unpack8(*reinterpret_cast<const uint4*>(src), v);
                } else {
                    const float4 a = *reinterpret_cast<const float4*>(src), b = *reinterpret_cast<const float4*>(src + 4);
                    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
                }
            } else {
#pragma unroll
                for (int k = 0; k < 8; ++k) v[k] = 0.f;
            }
            float* d = dst + r * LW + pl + 8 * ch;
#pragma unroll
            for (int k = 0; k < 8; ++k) d[k] = v[k];
        }
        const int npad = LW - Wi;  // pl left + the rest right
        for (int i = threadIdx.x; i < LH * npad; i += kBlock) {
            const int r = i / npad, k = i - r * npad;
            dst[r * LW + (k < pl ? k : Wi + k)] = 0.f;
        }
    } else {
        for (int i = threadIdx.x; i < LH * LW; i += kBlock) {
            const int r = i / LW, c = i - r * LW;
            const int ih = ih0 + r, iw = c - pl;
            dst[i] = (ih >= 0 && ih < Hi && iw >= 0 && iw < Wi) ? ld(xp + (size_t)ih * Wi + iw) : 0.f;
        }
    }
}

// Round-5 segment kernel (the 5 x 5 and stride-2 forwards, where it measured faster than the tile
// mapping below): its own staging (column iw at iw + pl, row stride (Wo - 1) S + K) and SEG consecutive
// outputs of one row per thread. y (forward or stride-1 backward-data with flip): block = (PB
// consecutive planes, band of BHo output rows)
template <int K, int S, int SEG, typename T>
__global__ __launch_bounds__(kBlock) void k_dw_fwd_lds_seg(const T* __restrict__ x, const float* __restrict__ w, DwGeo g,
                                                       int flip, DwBand bd, T* __restrict__ y) {
    extern __shared__ float smem[];
    float* s_w = smem;                    // [PB][K*K]
    float* s_x = smem + bd.PB * K * K;    // [PB][LH][LW] (+ slack for the last segment's reads)
    const int band = blockIdx.x % bd.nbands, pg = blockIdx.x / bd.nbands;
    const int p0 = pg * bd.PB, np = min(bd.PB, g.nplanes - p0);
    const int oh0 = band * bd.BHo, nrow = min(bd.BHo, g.Ho - oh0);
    const int LH = (nrow - 1) * S + K;
    for (int i = threadIdx.x; i < np * K * K; i += kBlock) {
        const int pl = i / (K * K), t = i - pl * (K * K);
        s_w[i] = w[(size_t)((p0 + pl) % g.C) * K * K + (flip ? K * K - 1 - t : t)];
    }
    const bool vec8 = g.Wi % 8 == 0;
    for (int pl = 0; pl < np; ++pl)
        dw_stage_seg(x + (size_t)(p0 + pl) * g.Hi * g.Wi, g.Hi, g.Wi, oh0 * S - g.pt, LH, bd.LW, g.pl, vec8,
                 s_x + pl * bd.LHmax * bd.LW);
    __syncthreads();
    const int nseg = (g.Wo + SEG - 1) / SEG;
    const int items = np * nrow * nseg;
    constexpr int CW = (SEG - 1) * S + K;
    for (int it = threadIdx.x; it < items; it += kBlock) {
        const int pl = it / (nrow * nseg), rem = it - pl * (nrow * nseg);
        const int r = rem / nseg, sg = rem - r * nseg;
        const int ow0 = sg * SEG;
        const float* wk = s_w + pl * K * K;
        const float* xs = s_x + pl * bd.LHmax * bd.LW + (r * S) * bd.LW + ow0 * S;
        float acc[SEG];
#pragma unroll
        for (int j = 0; j < SEG; ++j) acc[j] = 0.f;
#pragma unroll
        for (int kh = 0; kh < K; ++kh) {
            float v[CW];
#pragma unroll
            for (int q = 0; q < CW; ++q) v[q] = xs[kh * bd.LW + q];
#pragma unroll
            for (int kw = 0; kw < K; ++kw) {
                const float wv = wk[kh * K + kw];
#pragma unroll
                for (int j = 0; j < SEG; ++j) acc[j] = fmaf(v[j * S + kw], wv, acc[j]);
            }
        }
        store_seg<SEG>(y + ((size_t)(p0 + pl) * g.Ho + oh0 + r) * g.Wo + ow0, acc, min(SEG, g.Wo - ow0));
    }
}

// Compute mapping of the LDS kernels: consecutive threads take consecutive output COLUMNS of a row
// group (TH output rows of one plane), so a wave's LDS reads of a tap are consecutive words (no bank
// conflicts; the round-5 mapping gave each thread SEG consecutive outputs, lanes 8 words apart: 8-way
// conflicts that made these kernels LDS-bound), and each staged input row a thread reads feeds every
// output row of its group it overlaps (vertical reuse: ((TH - 1) S + K) K reads for TH K^2 FMAs).
constexpr int kDwTH = 4;
// output columns per thread: TW consecutive outputs (one 4 * TW-byte store per row for bf16; the
// single-column form issued 8x the store instructions of the 16-B segment form and measured slower)
constexpr int kDwTW = 4;
// which LDS kernels take the TH x TW tile mapping (per-layer A/B, c3 step, profiles/r06/dw_tile_ab.txt):
// every weight gradient and the 3 x 3 stride-1 forward (27.9 vs 32.1 us at 64 x 176; weight gradients
// 33.6 vs 42.5, 46.3 vs 65.5); 5 x 5 and stride-2 forwards keep the segment mapping (57 vs 38 us: their
// threads' input columns 4 S words apart conflict in the LDS banks again)
__host__ __device__ constexpr bool dw_tile_map(int K, int S, bool fwd) { return !fwd || (K == 3 && S == 1); }

// y (forward or stride-1 backward-data with flip): block = (PB consecutive planes, band of BHo output rows)
template <int K, int S, int SEG, typename T>
__global__ __launch_bounds__(kBlock) void k_dw_fwd_lds(const T* __restrict__ x, const float* __restrict__ w, DwGeo g,
                                                       int flip, DwBand bd, T* __restrict__ y) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int TH = kDwTH, TR = (TH - 1) * S + K;  // output rows per thread, input rows they read
    const int band = blockIdx.x % bd.nbands, pg = blockIdx.x / bd.nbands;
    const int p0 = pg * bd.PB, np = min(bd.PB, g.nplanes - p0);
    const int oh0 = band * bd.BHo, nrow = min(bd.BHo, g.Ho - oh0);
    const int LH = (nrow - 1) * S + K;
    const int lps = bd.LHmax * bd.LW;
    float* s_x = smem;                    // [PB][LHmax][LW] (8-B aligned rows)
    float* s_w = smem + bd.PB * lps;      // [PB][K*K]
    dw_stage(x + (size_t)p0 * g.Hi * g.Wi, (size_t)g.Hi * g.Wi, np, g.Hi, g.Wi, oh0 * S - g.pt, LH, bd.LW, lps, s_x);
    for (int i = threadIdx.x; i < np * K * K; i += kBlock) {
        const int pl = i / (K * K), t = i - pl * (K * K);
        s_w[i] = w[(size_t)((p0 + pl) % g.C) * K * K + (flip ? K * K - 1 - t : t)];
    }
    __syncthreads();
    const int col0 = kDwCol - g.pl;
    constexpr int TW = kDwTW, CW = (TW - 1) * S + K;  // output columns per thread, input columns they read
    const int nrg = (nrow + TH - 1) / TH, ncg = g.Wo / TW;  // (Wo % TW == 0: dw_lds_ok)
    const int items = np * nrg * ncg;
    for (int it = threadIdx.x; it < items; it += kBlock) {
        const int pr = it / ncg, ow = (it - pr * ncg) * TW;
        const int pl = pr / nrg, rg = pr - pl * nrg;
        const float* wk = s_w + pl * K * K;
        const float* xs = s_x + pl * lps + (rg * TH * S) * bd.LW + ow * S + col0;
        float acc[TH][TW];
#pragma unroll
        for (int j = 0; j < TH; ++j)
#pragma unroll
            for (int c = 0; c < TW; ++c) acc[j][c] = 0.f;
#pragma unroll
        for (int t = 0; t < TR; ++t) {  // input row t of the group (rows past the band's end: never stored)
            float v[CW];
#pragma unroll
            for (int q = 0; q < CW; ++q) v[q] = xs[min(t, LH - 1 - rg * TH * S) * bd.LW + q];
#pragma unroll
            for (int j = 0; j < TH; ++j) {
                const int kh = t - j * S;
                if (kh >= 0 && kh < K)
#pragma unroll
                    for (int kw = 0; kw < K; ++kw) {
                        const float wv = wk[kh * K + kw];
#pragma unroll
                        for (int c = 0; c < TW; ++c) acc[j][c] = fmaf(v[c * S + kw], wv, acc[j][c]);
                    }
            }
        }
        T* yp = y + ((size_t)(p0 + pl) * g.Ho + oh0 + rg * TH) * g.Wo + ow;
#pragma unroll
        for (int j = 0; j < TH; ++j)
            if (rg * TH + j < nrow) store_seg<TW>(yp + (size_t)j * g.Wo, acc[j], TW);
    }
}

// weight-gradient partials: block (channel c, image group q), PB images of the group staged at a time
template <int K, int S, int SEG, typename T>
__global__ __launch_bounds__(kBlock) void k_dw_wgt_lds(const T* __restrict__ x, const T* __restrict__ dy, DwGeo g,
                                                       int nimg, int ngroups, DwBand bd, float* __restrict__ partial,
                                                       DwFold fold) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int TH = kDwTH, TR = (TH - 1) * S + K;
    float* s_x = smem;  // [PB][LHmax][LW]
    __shared__ float s_red[kBlock / kWave][K * K];
    const int c = blockIdx.x % g.C, q = blockIdx.x / g.C;
    const int n0 = (int)((long)nimg * q / ngroups), n1 = (int)((long)nimg * (q + 1) / ngroups);
    const int lps = bd.LHmax * bd.LW;
    const int col0 = kDwCol - g.pl;
    float acc[K * K];
#pragma unroll
    for (int i = 0; i < K * K; ++i) acc[i] = 0.f;
    for (int nb = n0; nb < n1; nb += bd.PB) {
        const int np = min(bd.PB, n1 - nb);
        for (int band = 0; band < bd.nbands; ++band) {
            const int oh0 = band * bd.BHo, nrow = min(bd.BHo, g.Ho - oh0);
            const int LH = (nrow - 1) * S + K;
            __syncthreads();  // the previous chunk's readers are done with s_x
            dw_stage(x + ((size_t)nb * g.C + c) * g.Hi * g.Wi, (size_t)g.C * g.Hi * g.Wi, np, g.Hi, g.Wi,
                     oh0 * S - g.pt, LH, bd.LW, lps, s_x);
            __syncthreads();
            constexpr int TW = kDwTW, CW = (TW - 1) * S + K;
            const int nrg = (nrow + TH - 1) / TH, ncg = g.Wo / TW;
            const int items = np * nrg * ncg;
            for (int it = threadIdx.x; it < items; it += kBlock) {
                const int pr = it / ncg, ow = (it - pr * ncg) * TW;
                const int pl = pr / nrg, rg = pr - pl * nrg;
                // the group's dy values (clamped rows, zeroed past the band: every load issued before the first use)
                const T* dp = dy + (((size_t)(nb + pl) * g.C + c) * g.Ho + oh0 + rg * TH) * g.Wo + ow;
                float d[TH][TW];
#pragma unroll
                for (int j = 0; j < TH; ++j) load_seg<TW>(dp + (size_t)min(j, nrow - 1 - rg * TH) * g.Wo, d[j], TW);
#pragma unroll
                for (int j = 0; j < TH; ++j)
                    if (rg * TH + j >= nrow)
#pragma unroll
                        for (int cc = 0; cc < TW; ++cc) d[j][cc] = 0.f;
                const float* xs = s_x + pl * lps + (rg * TH * S) * bd.LW + ow * S + col0;
#pragma unroll
                for (int t = 0; t < TR; ++t) {
                    float v[CW];
#pragma unroll
                    for (int qq = 0; qq < CW; ++qq) v[qq] = xs[min(t, LH - 1 - rg * TH * S) * bd.LW + qq];
#pragma unroll
                    for (int j = 0; j < TH; ++j) {
                        const int kh = t - j * S;
                        if (kh >= 0 && kh < K)
#pragma unroll
                            for (int kw = 0; kw < K; ++kw)
#pragma unroll
                                for (int cc = 0; cc < TW; ++cc)
                                    acc[kh * K + kw] = fmaf(d[j][cc], v[cc * S + kw], acc[kh * K + kw]);
                    }
                }
            }
        }
    }
    const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
#pragma unroll
    for (int i = 0; i < K * K; ++i) {
        float v = acc[i];
#pragma unroll
        for (int o = kWave / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
        if (lane == 0) s_red[wave][i] = v;
    }
    __syncthreads();
    float t = 0.f;
    if (threadIdx.x < K * K) {
#pragma unroll
        for (int jw = 0; jw < kBlock / kWave; ++jw) t += s_red[jw][threadIdx.x];
    }
    dw_finish<K * K>(partial, c, q, ngroups, t, fold);
}

// bands and planes per block for the LDS kernels: the whole plane when it fits, several planes per
// block while the block has fewer than ~2 output segments per thread
template <int K, int S>
inline DwBand dw_band(const DwGeo& g, int seg, int max_planes, bool tile) {
    DwBand b;
    // row stride: the data at kDwCol, every compute read of the last (possibly partial) segment inside
    // the row; LW = 2 (mod 4): rows 8-B aligned for the staging writes, and consecutive rows start 2
    // banks apart (a stride of 0 mod 8 lined every row's segments up on the same banks: 32 -> 49 us at
    // block 0's 64 x 176 planes)
    (void)seg;
    b.LW = ((kDwCol - g.pl + (g.Wo - 1) * S + K + 1) & ~3) + 2;
    const int full = (g.Ho - 1) * S + K;
    if (full * b.LW <= kDwLdsFloats) {
        b.BHo = g.Ho;
        const int per_plane = tile ? ((g.Ho + kDwTH - 1) / kDwTH) * (g.Wo / kDwTW) : g.Ho * (g.Wo / seg);  // items
        int pb = std::max(1, kDwLdsFloats / (full * b.LW));
        pb = std::min(pb, std::max(1, (2 * kBlock + per_plane - 1) / per_plane));
        b.PB = std::max(1, std::min(pb, max_planes));
    } else {
        b.BHo = std::max(1, (kDwLdsFloats / b.LW - K) / S + 1);
        b.PB = 1;
    }
    b.LHmax = (b.BHo - 1) * S + K;
    b.nbands = (g.Ho + b.BHo - 1) / b.BHo;
    return b;
}

// the LDS kernels' vector accesses need 16-B aligned tensors; the staged row holds the whole input row
// (the right padding is not negative); and they run only where an output row splits into segments of
// 4 or 8 (Wo % 4 == 0): on the trunk's narrow planes (Wo = 22, 11) the register-tiled kernels are
// faster (c3 step, per layer: 15-55 vs 21-98 us), on the wide ones the LDS kernels (23-74 vs 50-181 us)
template <int K, int S>
inline bool dw_lds_ok(const DwGeo& g, const void* a, const void* b) {
    return ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b)) & 15) == 0 && g.Wo % 4 == 0 &&
           (g.Wo - 1) * S + K >= g.pl + g.Wi && (g.Ho - 1) * S + K >= g.pt + g.Hi;
}

inline int dw_seg(int Wo) { return Wo % 8 == 0 ? 8 : Wo % 4 == 0 ? 4 : Wo % 2 == 0 ? 2 : 1; }

// the round-5 band for the segment kernel: LDS rows of exactly (Wo - 1) S + K floats
template <int K, int S>
inline DwBand dw_band_seg(const DwGeo& g, int seg, int max_planes) {
    DwBand b;
    b.LW = (g.Wo - 1) * S + K;
    const int full = (g.Ho - 1) * S + K;
    if (full * b.LW <= kDwLdsFloats) {
        b.BHo = g.Ho;
        const int per_plane = g.Ho * ((g.Wo + seg - 1) / seg);
        int pb = std::max(1, kDwLdsFloats / (full * b.LW));
        pb = std::min(pb, std::max(1, (2 * kBlock + per_plane - 1) / per_plane));
        b.PB = std::max(1, std::min(pb, max_planes));
    } else {
        b.BHo = std::max(1, (kDwLdsFloats / b.LW - K) / S + 1);
        b.PB = 1;
    }
    b.LHmax = (b.BHo - 1) * S + K;
    b.nbands = (g.Ho + b.BHo - 1) / b.BHo;
    return b;
}

template <int K, int S, typename T>
int dw_fwd_lds(const void* x, const float* w, DwGeo g, int flip, void* y, hipStream_t s) {
    const int seg = dw_seg(g.Wo);
    if constexpr (!dw_tile_map(K, S, true)) {
        const DwBand b = dw_band_seg<K, S>(g, seg, g.nplanes);
        const long blocks = (long)b.nbands * ((g.nplanes + b.PB - 1) / b.PB);
        // slack past the staged rows: the last segment of a row reads up to (SEG - 1) * S columns past Wo
        const size_t lds = sizeof(float) * ((size_t)b.PB * K * K + (size_t)b.PB * b.LHmax * b.LW + 8 * S + K);
        if (blocks > INT_MAX) return LSS_CONV_EINVAL;
#define LSS_DW_FWD_SEG(SG) hipLaunchKernelGGL((k_dw_fwd_lds_seg<K, S, SG, T>), dim3((unsigned)blocks), dim3(kBlock), lds, \
                                              s, (const T*)x, w, g, flip, b, (T*)y)
        switch (seg) {
            case 8: LSS_DW_FWD_SEG(8); break;
            case 4: LSS_DW_FWD_SEG(4); break;
            case 2: LSS_DW_FWD_SEG(2); break;
            default: LSS_DW_FWD_SEG(1); break;
        }
#undef LSS_DW_FWD_SEG
        return launch_status();
    }
    const DwBand b = dw_band<K, S>(g, seg, g.nplanes, dw_tile_map(K, S, true));
    const long blocks = (long)b.nbands * ((g.nplanes + b.PB - 1) / b.PB);
    const size_t lds = sizeof(float) * ((size_t)b.PB * b.LHmax * b.LW + (size_t)b.PB * K * K);
    if (blocks > INT_MAX) return LSS_CONV_EINVAL;
#define LSS_DW_FWD(SG) hipLaunchKernelGGL((k_dw_fwd_lds<K, S, SG, T>), dim3((unsigned)blocks), dim3(kBlock), lds, s, \
                                          (const T*)x, w, g, flip, b, (T*)y)
    switch (seg) {
        case 8: LSS_DW_FWD(8); break;
        case 4: LSS_DW_FWD(4); break;
        case 2: LSS_DW_FWD(2); break;
        default: LSS_DW_FWD(1); break;
    }
#undef LSS_DW_FWD
    return launch_status();
}

template <int K, int S, typename T>
int dw_wgt_lds(const void* x, const void* dy, DwGeo g, int nimg, int ngroups, float* partial, DwFold fold,
               hipStream_t s) {
    const int seg = dw_seg(g.Wo);
    const DwBand b = dw_band<K, S>(g, seg, (nimg + ngroups - 1) / ngroups, dw_tile_map(K, S, false));
    const size_t lds = sizeof(float) * ((size_t)b.PB * b.LHmax * b.LW);
#define LSS_DW_WGT(SG) hipLaunchKernelGGL((k_dw_wgt_lds<K, S, SG, T>), dim3(g.C * ngroups), dim3(kBlock), lds, s, \
                                          (const T*)x, (const T*)dy, g, nimg, ngroups, b, partial, fold)
    switch (seg) {
        case 8: LSS_DW_WGT(8); break;
        case 4: LSS_DW_WGT(4); break;
        case 2: LSS_DW_WGT(2); break;
        default: LSS_DW_WGT(1); break;
    }
#undef LSS_DW_WGT
    return launch_status();
}

// ---- narrow planes (the trunk's 8 x 22 and 4 x 11 maps: Wo in {22, 11}), whole planes per block. The
// register-tiled kernels above issue ~100 two-byte loads per thread on these (lanes 8 B apart; 0.6-1.4
// TB/s, profiles/r06/step_roofline.json), and their rows of 22 / 11 elements are not 16-B aligned,
// which kept them off the LDS kernels' vector staging. But a block's consecutive planes are ONE
// contiguous run of memory: staged here with flat 16-B loads into zero-padded fp32 LDS planes; a
// thread computes one output row (WO outputs; every staged value it reads feeds all the taps that
// reach it); the outputs go back through LDS as one contiguous run of 16-B stores.
template <typename T>
__device__ __forceinline__ void ldv16(const T* p, float* o);  // 16 B -> 16 / sizeof(T) floats
template <> __device__ __forceinline__ void ldv16<bf16>(const bf16* p, float* o) { unpack8(*reinterpret_cast<const uint4*>(p), o); }
template <> __device__ __forceinline__ void ldv16<float>(const float* p, float* o) {
    const float4 a = *reinterpret_cast<const float4*>(p);
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w;
}

// f(i, v) for the n elements of the run at src: 16-B loads when the run allows them (src 16-B aligned,
// n a multiple of the vector), else one element per load
template <typename T, typename F>
__device__ __forceinline__ void for_run(const T* __restrict__ src, int n, F&& f) {
    constexpr int V = 16 / sizeof(T);
    if ((reinterpret_cast<uintptr_t>(src) & 15) == 0 && n % V == 0) {
        for (int i = threadIdx.x; i < n / V; i += kBlock) {
            float v[V];
            ldv16<T>(src + (size_t)i * V, v);
#pragma unroll
            for (int j = 0; j < V; ++j) f(i * V + j, v[j]);
        }
    } else {
        for (int i = threadIdx.x; i < n; i += kBlock) f(i, ld(src + i));
    }
}

// VW consecutive elements -> fp32, in loads of up to 16 B (the caller guarantees the alignment)
template <int VW, typename T>
__device__ __forceinline__ void ld_vec(const T* __restrict__ p, float* o) {
    constexpr int B = VW * (int)sizeof(T);
    if constexpr (B >= 16) {
        constexpr int E = 16 / (int)sizeof(T);
#pragma unroll
        for (int k = 0; k < VW; k += E) ldv16<T>(p + k, o + k);
    } else if constexpr (B == 8 && sizeof(T) == 2) {
        const uint2 u = *reinterpret_cast<const uint2*>(p);
        o[0] = __uint_as_float(u.x << 16); o[1] = __uint_as_float(u.x & 0xFFFF0000u);
        o[2] = __uint_as_float(u.y << 16); o[3] = __uint_as_float(u.y & 0xFFFF0000u);
    } else if constexpr (B == 8) {
        const float2 a = *reinterpret_cast<const float2*>(p);
        o[0] = a.x; o[1] = a.y;
    } else if constexpr (B == 4 && sizeof(T) == 2) {
        const unsigned u = *reinterpret_cast<const unsigned*>(p);
        o[0] = __uint_as_float(u << 16); o[1] = __uint_as_float(u & 0xFFFF0000u);
    } else {
#pragma unroll
        for (int k = 0; k < VW; ++k) o[k] = ld(p + k);
    }
}

// f(pl, e, v) for element e of plane pl, over np planes of n elements each at x + (first + pl * step) * n:
// one flat loop over every plane's VW-element vectors, so all their loads are in flight together
template <int VW, typename T, typename F>
__device__ __forceinline__ void for_planes_v(const T* __restrict__ x, size_t first, size_t step, int np, int n, F&& f) {
    const int nv = n / VW;
    for (int i = threadIdx.x; i < np * nv; i += kBlock) {
        const int pl = i / nv, v = i - pl * nv;
        float vals[VW];
        ld_vec<VW, T>(x + (first + (size_t)pl * step) * n + (size_t)v * VW, vals);
#pragma unroll
        for (int j = 0; j < VW; ++j) f(pl, v * VW + j, vals[j]);
    }
}
template <typename T, typename F>
__device__ __forceinline__ void for_planes(const T* __restrict__ x, size_t first, size_t step, int np, int n, F&& f) {
    // (plane bases are n elements apart: n % VW == 0 keeps every vector aligned on an aligned tensor)
    if (n % 8 == 0) for_planes_v<8, T>(x, first, step, np, n, f);
    else if (n % 4 == 0) for_planes_v<4, T>(x, first, step, np, n, f);
    else if (n % 2 == 0) for_planes_v<2, T>(x, first, step, np, n, f);
    else for_planes_v<1, T>(x, first, step, np, n, f);
}

// the run [0, n) of s (T in LDS) to dst: 16-B stores when aligned
template <typename T>
__device__ __forceinline__ void store_run(T* __restrict__ dst, const T* __restrict__ s, int n) {
    constexpr int V = 16 / sizeof(T);
    if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0 && n % V == 0) {
        for (int i = threadIdx.x; i < n / V; i += kBlock)
            *reinterpret_cast<uint4*>(dst + (size_t)i * V) = *reinterpret_cast<const uint4*>(s + (size_t)i * V);
    } else {
        for (int i = threadIdx.x; i < n; i += kBlock) dst[i] = s[i];
    }
}

__device__ __forceinline__ void to_t(float* p, float v) { *p = v; }
__device__ __forceinline__ void to_t(bf16* p, float v) { *p = __float2bfloat16(v); }

// one input plane element (r, c) into its padded LDS slot (never read if it lies past the reach)
__device__ __forceinline__ void put_padded(float* __restrict__ plane, int r, int c, int pt, int pl, int LH, int LW,
                                          float v) {
    const int rr = r + pt, cc = c + pl;
    if (rr < LH && cc < LW) plane[rr * LW + cc] = v;
}

template <int K, int S, int WO>
struct PlaneGeo {
    static constexpr int LW = (WO - 1) * S + K;
    __host__ __device__ static int LH(int Ho) { return (Ho - 1) * S + K; }
};

// forward (and stride-1 backward-data with flip): block = PB consecutive planes
template <int K, int S, int WO, typename T>
__global__ __launch_bounds__(kBlock) void k_dw_fwd_planes(const T* __restrict__ x, const float* __restrict__ w,
                                                          DwGeo g, int flip, int PB, T* __restrict__ y) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    using PG = PlaneGeo<K, S, WO>;
    constexpr int LW = PG::LW;
    const int LH = PG::LH(g.Ho), plane_f = LH * LW;
    const int p0 = blockIdx.x * PB, np = min(PB, g.nplanes - p0);
    const int HiWi = g.Hi * g.Wi, HoWo = g.Ho * WO;
    float* s_w = smem;                                   // [PB][K*K]
    float* s_x = s_w + ((PB * K * K + 3) & ~3);          // [PB][LH][LW]
    T* s_y = reinterpret_cast<T*>(s_x + ((PB * plane_f + 3) & ~3));  // [PB][Ho][WO], 16-B aligned
    for (int i = threadIdx.x; i < np * plane_f; i += kBlock) s_x[i] = 0.f;
    for (int i = threadIdx.x; i < np * K * K; i += kBlock) {
        const int pl = i / (K * K), t = i - pl * (K * K);
        s_w[i] = w[(size_t)((p0 + pl) % g.C) * K * K + (flip ? K * K - 1 - t : t)];
    }
    __syncthreads();
    for_run(x + (size_t)p0 * HiWi, np * HiWi, [&](int f, float v) {
        const int pl = f / HiWi, rem = f - pl * HiWi;
        const int r = rem / g.Wi;
        put_padded(s_x + pl * plane_f, r, rem - r * g.Wi, g.pt, g.pl, LH, LW, v);
    });
    __syncthreads();
    for (int it = threadIdx.x; it < np * g.Ho; it += kBlock) {
        const int pl = it / g.Ho, oh = it - pl * g.Ho;
        const float* xs = s_x + pl * plane_f + oh * S * LW;
        const float* wk = s_w + pl * K * K;
        float acc[WO];
#pragma unroll
        for (int j = 0; j < WO; ++j) acc[j] = 0.f;
#pragma unroll
        for (int kh = 0; kh < K; ++kh) {
            float v[LW];
#pragma unroll
            for (int q = 0; q < LW; ++q) v[q] = xs[kh * LW + q];
#pragma unroll
            for (int kw = 0; kw < K; ++kw) {
                const float wv = wk[kh * K + kw];
#pragma unroll
                for (int j = 0; j < WO; ++j) acc[j] = fmaf(v[j * S + kw], wv, acc[j]);
            }
        }
        T* o = s_y + pl * HoWo + oh * WO;
#pragma unroll
        for (int j = 0; j < WO; ++j) to_t(o + j, acc[j]);
    }
    __syncthreads();
    store_run(y + (size_t)p0 * HoWo, s_y, np * HoWo);
}

// weight-gradient partials: block (channel c, image group q); PB images' planes of x and dy staged at
// a time; a thread takes output rows; fixed reduction order (the thread's rows in order, then wave
// shuffles, then waves in order)
template <int K, int S, int WO, typename T>
__global__ __launch_bounds__(kBlock) void k_dw_wgt_planes(const T* __restrict__ x, const T* __restrict__ dy, DwGeo g,
                                                          int nimg, int ngroups, int PB, float* __restrict__ partial,
                                                          DwFold fold) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    __shared__ float s_red[kBlock / kWave][K * K];
    using PG = PlaneGeo<K, S, WO>;
    constexpr int LW = PG::LW;
    const int LH = PG::LH(g.Ho), plane_f = LH * LW;
    const int c = blockIdx.x % g.C, q = blockIdx.x / g.C;
    const int n0 = (int)((long)nimg * q / ngroups), n1 = (int)((long)nimg * (q + 1) / ngroups);
    const int HiWi = g.Hi * g.Wi, HoWo = g.Ho * WO;
    float* s_x = smem;                                   // [PB][LH][LW]
    float* s_d = s_x + PB * plane_f;                     // [PB][Ho][WO]
    float acc[K * K];
#pragma unroll
    for (int i = 0; i < K * K; ++i) acc[i] = 0.f;
    for (int nb = n0; nb < n1; nb += PB) {
        const int np = min(PB, n1 - nb);
        __syncthreads();  // the previous chunk's readers are done
        for (int i = threadIdx.x; i < np * plane_f; i += kBlock) s_x[i] = 0.f;
        __syncthreads();
        const size_t first = (size_t)nb * g.C + c;  // plane (image nb, channel c); images g.C planes apart
        for_planes(x, first, (size_t)g.C, np, HiWi, [&](int pl, int f, float v) {
            const int r = f / g.Wi;
            put_padded(s_x + pl * plane_f, r, f - r * g.Wi, g.pt, g.pl, LH, LW, v);
        });
        for_planes(dy, first, (size_t)g.C, np, HoWo, [&](int pl, int f, float v) { s_d[pl * HoWo + f] = v; });
        __syncthreads();
        for (int it = threadIdx.x; it < np * g.Ho; it += kBlock) {
            const int pl = it / g.Ho, oh = it - pl * g.Ho;
            const float* xs = s_x + pl * plane_f + oh * S * LW;
            const float* ds = s_d + pl * HoWo + oh * WO;
            float d[WO];
#pragma unroll
            for (int j = 0; j < WO; ++j) d[j] = ds[j];
#pragma unroll
            for (int kh = 0; kh < K; ++kh) {
                float v[LW];
#pragma unroll
                for (int qq = 0; qq < LW; ++qq) v[qq] = xs[kh * LW + qq];
#pragma unroll
                for (int kw = 0; kw < K; ++kw) {
                    float a = acc[kh * K + kw];
#pragma unroll
                    for (int j = 0; j < WO; ++j) a = fmaf(d[j], v[j * S + kw], a);
                    acc[kh * K + kw] = a;
                }
            }
        }
    }
    const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
#pragma unroll
    for (int i = 0; i < K * K; ++i) {
        float v = acc[i];
#pragma unroll
        for (int o = kWave / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
        if (lane == 0) s_red[wave][i] = v;
    }
    __syncthreads();
    float t = 0.f;
    if (threadIdx.x < K * K) {
#pragma unroll
        for (int jw = 0; jw < kBlock / kWave; ++jw) t += s_red[jw][threadIdx.x];
    }
    dw_finish<K * K>(partial, c, q, ngroups, t, fold);
}

#ifndef LSS_DW_PLANES
#define LSS_DW_PLANES 1  // experiment switch: 0 = the register-tiled kernels on the narrow planes
#endif
constexpr int kDwPlanesLdsMax = 48 * 1024;  // bytes of LDS a planes block may use

// the planes kernels take Wo in {22, 11} (the trunk's narrow maps), a staged plane holding every input
// element a tap reaches; PB = planes per block: one output row per thread, within the LDS budget
template <int K, int S, int WO>
inline int dw_planes_pb(const DwGeo& g, int extra_floats_per_plane, int elt) {
    if (!LSS_DW_PLANES || g.Wo != WO) return 0;
    using PG = PlaneGeo<K, S, WO>;
    const int plane_bytes = 4 * (PG::LH(g.Ho) * PG::LW + extra_floats_per_plane) + elt * g.Ho * WO;
    int pb = std::max(1, kBlock / g.Ho);
    while (pb > 1 && pb * plane_bytes + 4 * pb * K * K + 64 > kDwPlanesLdsMax) --pb;
    return pb * plane_bytes + 4 * pb * K * K + 64 <= kDwPlanesLdsMax ? pb : 0;
}

template <int K, int S, typename T>
int dw_fwd_planes(const void* x, const float* w, DwGeo g, int flip, void* y, hipStream_t s) {
    // (stride 2: slower than the register-tiled kernel, 21.9 / 21.0 vs 15.3 / 19.1 us in the c3 step)
    if (S != 1) return 1;
    auto go = [&](auto wo_tag) -> int {
        constexpr int WO = decltype(wo_tag)::value;
        const int pb = dw_planes_pb<K, S, WO>(g, 0, (int)sizeof(T));
        if (pb == 0) return 1;
        using PG = PlaneGeo<K, S, WO>;
        const size_t lds = 4 * ((((size_t)pb * K * K + 3) & ~(size_t)3) +
                                (((size_t)pb * PG::LH(g.Ho) * PG::LW + 3) & ~(size_t)3)) +
                           sizeof(T) * (size_t)pb * g.Ho * WO;
        const long blocks = ((long)g.nplanes + pb - 1) / pb;
        if (blocks > INT_MAX) return 1;
        hipLaunchKernelGGL((k_dw_fwd_planes<K, S, WO, T>), dim3((unsigned)blocks), dim3(kBlock), lds, s, (const T*)x,
                           w, g, flip, pb, (T*)y);
        return 0;
    };
    if (g.Wo == 22) return go(std::integral_constant<int, 22>{});
    if (g.Wo == 11) return go(std::integral_constant<int, 11>{});
    return 1;
}

template <int K, int S, typename T>
int dw_wgt_planes(const void* x, const void* dy, DwGeo g, int nimg, int ngroups, float* partial, DwFold fold,
                  hipStream_t s) {
    auto go = [&](auto wo_tag) -> int {
        constexpr int WO = decltype(wo_tag)::value;
        const int pb = dw_planes_pb<K, S, WO>(g, g.Ho * WO, 0);
        if (pb == 0) return 1;
        using PG = PlaneGeo<K, S, WO>;
        const size_t lds = 4 * (size_t)pb * (PG::LH(g.Ho) * PG::LW + g.Ho * WO);
        hipLaunchKernelGGL((k_dw_wgt_planes<K, S, WO, T>), dim3(g.C * ngroups), dim3(kBlock), lds, s, (const T*)x,
                           (const T*)dy, g, nimg, ngroups, pb, partial, fold);
        return 0;
    };
    if (g.Wo == 22) return go(std::integral_constant<int, 22>{});
    if (g.Wo == 11) return go(std::integral_constant<int, 11>{});
    return 1;
}

// dispatch over (K, S, T)
template <template <int, int, typename> class F, typename... A>
int dispatch_kst(int K, int S, int dtype, A... a) {
    if (dtype == LSS_CONV_F32) {
        if (K == 3 && S == 1) return F<3, 1, float>::run(a...);
        if (K == 3 && S == 2) return F<3, 2, float>::run(a...);
        if (K == 5 && S == 1) return F<5, 1, float>::run(a...);
        if (K == 5 && S == 2) return F<5, 2, float>::run(a...);
    } else if (dtype == LSS_CONV_BF16) {
        if (K == 3 && S == 1) return F<3, 1, bf16>::run(a...);
        if (K == 3 && S == 2) return F<3, 2, bf16>::run(a...);
        if (K == 5 && S == 1) return F<5, 1, bf16>::run(a...);
        if (K == 5 && S == 2) return F<5, 2, bf16>::run(a...);
    }
    return LSS_CONV_EINVAL;
}

template <int K, int S, typename T>
struct Fwd {
    static int run(const void* x, const float* w, DwGeo g, int flip, void* y, hipStream_t s) {
        if (LSS_DW_LDS && dw_lds_ok<K, S>(g, x, y)) return dw_fwd_lds<K, S, T>(x, w, g, flip, y, s);
        if (dw_fwd_planes<K, S, T>(x, w, g, flip, y, s) == 0) return launch_status();
        constexpr int TH = Tile<S>::TH, TW = Tile<S>::TW;
        const long n = (long)g.nplanes * ((g.Ho + TH - 1) / TH) * ((g.Wo + TW - 1) / TW);
        hipLaunchKernelGGL((k_dw_fwd<K, S, TH, TW, T>), dim3(blocks_for(n)), dim3(kBlock), 0, s, (const T*)x, w, g,
                           flip, (T*)y);
        return launch_status();
    }
};

template <int K, int S, typename T>
struct BwdData {
    static int run(const void* dy, const float* w, DwGeo g, void* dx, hipStream_t s) {
        if (S == 1) {  // the forward correlation with the kernel flipped, padding mirrored
            DwGeo t{g.C, g.Ho, g.Wo, g.Hi, g.Wi, K - 1 - g.pt, K - 1 - g.pl, g.nplanes};
            return Fwd<K, 1, T>::run(dy, w, t, 1, dx, s);
        }
        const dim3 gr(blocks_for((long)g.nplanes * ((g.Hi + 1) / 2) * ((g.Wi + 3) / 4))), bl(kBlock);
        const int par = ((g.pt & 1) << 1) | (g.pl & 1);
        if (par == 0) hipLaunchKernelGGL((k_dw_bwd_data_s2<K, 0, 0, T>), gr, bl, 0, s, (const T*)dy, w, g, (T*)dx);
        else if (par == 1) hipLaunchKernelGGL((k_dw_bwd_data_s2<K, 0, 1, T>), gr, bl, 0, s, (const T*)dy, w, g, (T*)dx);
        else if (par == 2) hipLaunchKernelGGL((k_dw_bwd_data_s2<K, 1, 0, T>), gr, bl, 0, s, (const T*)dy, w, g, (T*)dx);
        else hipLaunchKernelGGL((k_dw_bwd_data_s2<K, 1, 1, T>), gr, bl, 0, s, (const T*)dy, w, g, (T*)dx);
        return launch_status();
    }
};

template <int K, int S, typename T>
struct BwdWeight {
    static int run(const void* x, const void* dy, DwGeo g, int nimg, int ngroups, float* partial, DwFold fold,
                   hipStream_t s) {
        if (LSS_DW_LDS && dw_lds_ok<K, S>(g, x, dy))
            return dw_wgt_lds<K, S, T>(x, dy, g, nimg, ngroups, partial, fold, s);
        if (dw_wgt_planes<K, S, T>(x, dy, g, nimg, ngroups, partial, fold, s) == 0) return launch_status();
        hipLaunchKernelGGL((k_dw_bwd_weight<K, S, 4, S == 1 ? 4 : 2, T>), dim3(g.C * ngroups), dim3(kBlock), 0, s,
                           (const T*)x, (const T*)dy, g, nimg, ngroups, partial, fold);
        return launch_status();
    }
};

// ---- 1x1 convolution to ONE output channel over channels-last rows (BevEncode's last conv, up2.4:
// 128 -> outC = 1, src/models.py:115). As a GEMM it is a GEMV: its weight gradient is a K = B*X*Y
// reduction that hipBLASLt ran on 8 workgroups (MT16x16x512, ~210 us of a c3 step). Here a wave
// reads 4 rows per instruction (16 lanes x 16 B = one 128-channel row), fp32 accumulation.
constexpr int kHeadRows = 256;  // rows per block (64 per wave)

// BN mode (bnst = a batch norm's saved (4, C) statistics, NHWC): the input row is the batch norm's INPUT and
// each value goes through the apply pass's arithmetic first -- bf16(relu(fmaf(x, scale, shift))), what
// lss_bn_fwd's ReLU apply would have stored -- so the normalised map is never materialised.
__device__ __forceinline__ void head_bn8(const float* __restrict__ bnst, int C, int c0, float* sc, float* sh) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        sc[i] = bnst ? bnst[2 * C + c0 + i] : 1.f;
        sh[i] = bnst ? bnst[3 * C + c0 + i] : 0.f;
    }
}
__device__ __forceinline__ float head_in(float v, bool bn, float sc, float sh) {
    return bn ? __bfloat162float(__float2bfloat16(fmaxf(fmaf(v, sc, sh), 0.f))) : v;
}

template <int LPR>  // lanes per row: C / 8
__global__ __launch_bounds__(kBlock) void k_head1_fwd(const uint4* __restrict__ x, const float* __restrict__ w,
                                                      const float* __restrict__ bias, int P, bf16* __restrict__ y,
                                                      const float* __restrict__ bnst) {
    constexpr int RPI = kWave / LPR;  // rows per wave instruction
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int col = lane % LPR, sub = lane / LPR;
    float wv[8], sc[8], sh[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) wv[i] = w[col * 8 + i];
    const bool bn = bnst != nullptr;
    head_bn8(bnst, LPR * 8, col * 8, sc, sh);
    const float b = bias ? *bias : 0.f;  // (a device value: a captured graph replays with the current bias)
    const int r0 = blockIdx.x * kHeadRows + wave * (kHeadRows / 4);
#pragma unroll 4
    for (int it = 0; it < kHeadRows / 4 / RPI; ++it) {
        const int r = r0 + it * RPI + sub;
        float acc = 0.f;
        if (r < P) {
            const uint4 v = x[(size_t)r * LPR + col];
            const unsigned u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                acc = fmaf(head_in(__uint_as_float(u[i] << 16), bn, sc[2 * i], sh[2 * i]), wv[2 * i], acc);
                acc = fmaf(head_in(__uint_as_float(u[i] & 0xFFFF0000u), bn, sc[2 * i + 1], sh[2 * i + 1]), wv[2 * i + 1],
                           acc);
            }
        }
#pragma unroll
        for (int o = LPR / 2; o > 0; o >>= 1) acc += __shfl_xor(acc, o, kWave);
        if (col == 0 && r < P) y[r] = __float2bfloat16(acc + b);
    }
}

// dx[r, c] = dy[r] * w[c] (bf16); partial[block][c] = sum over the block's rows of dy[r] * x[r, c],
// partial[block][C] = sum of dy[r] (fixed reduction order: deterministic).
// (BN mode as k_head1_fwd's; dx == NULL: no input gradient written -- the batch norm's backward takes it
// as the rank-1 product bf16(dy[r] w[c]) itself, lss_bn_bwd_rank1)
template <int LPR>
__global__ __launch_bounds__(kBlock) void k_head1_bwd(const uint4* __restrict__ x, const bf16* __restrict__ dy,
                                                      const float* __restrict__ w, int P, uint4* __restrict__ dx,
                                                      float* __restrict__ partial, const float* __restrict__ bnst) {
    constexpr int RPI = kWave / LPR;
    constexpr int C = LPR * 8;
    __shared__ float s_part[4][C + 1];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int col = lane % LPR, sub = lane / LPR;
    float wv[8], acc[8] = {}, sc[8], sh[8];
    float dsum = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) wv[i] = w[col * 8 + i];
    const bool bn = bnst != nullptr;
    head_bn8(bnst, C, col * 8, sc, sh);
    const int r0 = blockIdx.x * kHeadRows + wave * (kHeadRows / 4);
#pragma unroll 4
    for (int it = 0; it < kHeadRows / 4 / RPI; ++it) {
        const int r = r0 + it * RPI + sub;
        if (r < P) {
            const float g = __bfloat162float(dy[r]);
            const uint4 v = x[(size_t)r * LPR + col];
            const unsigned u[4] = {v.x, v.y, v.z, v.w};
            unsigned o[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float lo = head_in(__uint_as_float(u[i] << 16), bn, sc[2 * i], sh[2 * i]);
                const float hi = head_in(__uint_as_float(u[i] & 0xFFFF0000u), bn, sc[2 * i + 1], sh[2 * i + 1]);
                acc[2 * i] = fmaf(g, lo, acc[2 * i]);
                acc[2 * i + 1] = fmaf(g, hi, acc[2 * i + 1]);
                const bf16 a = __float2bfloat16(g * wv[2 * i]), c = __float2bfloat16(g * wv[2 * i + 1]);
                o[i] = (unsigned)*reinterpret_cast<const unsigned short*>(&a) |
                       ((unsigned)*reinterpret_cast<const unsigned short*>(&c) << 16);
            }
            if (dx) dx[(size_t)r * LPR + col] = make_uint4(o[0], o[1], o[2], o[3]);
            if (col == 0) dsum += g;
        }
    }
    // lanes of one column slice: reduce over the wave's row groups, then over the waves via LDS
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int off = LPR; off < kWave; off <<= 1) acc[i] += __shfl_xor(acc[i], off, kWave);
#pragma unroll
    for (int off = LPR; off < kWave; off <<= 1) dsum += __shfl_xor(dsum, off, kWave);
    if (sub == 0) {
#pragma unroll
        for (int i = 0; i < 8; ++i) s_part[wave][col * 8 + i] = acc[i];
        if (col == 0) s_part[wave][C] = dsum;
    }
    __syncthreads();
    for (int c = threadIdx.x; c <= C; c += kBlock)
        partial[(size_t)blockIdx.x * (C + 1) + c] = ((s_part[0][c] + s_part[1][c]) + s_part[2][c]) + s_part[3][c];
}

// ----------------------------------------------------------------------------- per-sample scale (+ add)
// y = bf16(x * scale[n] (+ r)) over sample-major bf16 tensors, scale[n] from the sample's draw, 8 elements (16 B) per thread: the
// MBConv residual with stochastic depth (efficientnet_pytorch drop_connect, x / keep * mask +
// inputs) in one pass instead of three; with r == nullptr, its backward dx = bf16(dy * scale[n]).

// the sample's scale from its uniform draw u (bf16): mask = floor(bf16(keep + u)) as torch computes
// floor(keep + rand(..., dtype=bf16)), scale = mask / keep
__device__ __forceinline__ float drop_scale(const bf16* u, long long n, float keep) {
    const float t = __bfloat162float(__float2bfloat16(keep + __bfloat162float(u[n])));
    return floorf(t) / keep;
}

__global__ __launch_bounds__(kBlock) void k_scale_add(const uint4* __restrict__ x, const bf16* __restrict__ u,
                                                      float keep, const uint4* __restrict__ r, long long per8,
                                                      long long n8, uint4* __restrict__ y) {
    const long long i = (long long)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n8) return;
    const float sc = drop_scale(u, i / per8, keep);
    float v[8], w[8];
    unpack8(x[i], v);
    if (r) {
        unpack8(r[i], w);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = fmaf(v[k], sc, w[k]);
    } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] *= sc;
    }
    y[i] = make_uint4(pack2(v[0], v[1]), pack2(v[2], v[3]), pack2(v[4], v[5]), pack2(v[6], v[7]));
}


// ---- dropout (CamEncode.dropout, src/models.py:44, 53) on a counter-based RNG, laid out for the next kernel
// Philox4x32-10 (Salmon et al., SC'11): 10 rounds of the two multiplies and key bumps; a pure function of
// (key, counter), so the backward regenerates the forward's mask from the same seed.
__device__ __forceinline__ uint4 philox4x32(uint2 key, uint4 c) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const unsigned lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
        const unsigned lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
        c = make_uint4(hi1 ^ c.y ^ key.x, lo1, hi0 ^ c.w ^ key.y, lo0);
        key.x += 0x9E3779B9u;
        key.y += 0xBB67AE85u;
    }
    return c;
}

// Elements of 16-B vector v (8 bf16 or 4 fp32) kept: bit j = element j; uniform u = top 24 bits / 2^24,
// kept when u < keep (P = keep). Counter (v, 0, 0, 0): 4 draws, a second block (v, 0, 1, 0) for bf16.
template <int EPV>
__device__ __forceinline__ unsigned keep_bits(uint2 key, long long v, unsigned thresh) {
    unsigned bits = 0;
#pragma unroll
    for (int h = 0; h < EPV / 4; ++h) {
        const uint4 r = philox4x32(key, make_uint4((unsigned)v, (unsigned)(v >> 32), (unsigned)h, 0u));
        bits |= ((r.x >> 8) < thresh ? 1u : 0u) << (4 * h);
        bits |= ((r.y >> 8) < thresh ? 1u : 0u) << (4 * h + 1);
        bits |= ((r.z >> 8) < thresh ? 1u : 0u) << (4 * h + 2);
        bits |= ((r.w >> 8) < thresh ? 1u : 0u) << (4 * h + 3);
    }
    return bits;
}

constexpr int kDropVpt = 2;  // 16-B vectors per thread
// XCD x (blockIdx & 7) writes one contiguous eighth of the tensor, the eighth the fused lift's blocks on
// that XCD read (k_depthnet_lift3: pixel tiles in XCD-contiguous runs), so the lift finds its features
// in its own L2 instead of another XCD's; the blocks also touch `pf` (the lift's packed weights), one
// slice per block of each XCD, so every XCD's L2 holds them before the lift starts.
template <typename T>
__global__ __launch_bounds__(kBlock) void k_dropout(const uint4* __restrict__ x, long long nv,
                                                    const unsigned long long* __restrict__ seed, unsigned thresh,
                                                    float scale, uint4* __restrict__ y, const uint4* __restrict__ pf,
                                                    long long pf16) {
    constexpr int EPV = 16 / (int)sizeof(T);
    const int bpx = gridDim.x >> 3;                                         // blocks per XCD
    const long long lb = (long long)(blockIdx.x & 7) * bpx + (blockIdx.x >> 3);  // XCD-contiguous
    uint4 warm = make_uint4(0u, 0u, 0u, 0u);
    if (pf) {
        const long long per = (pf16 + bpx - 1) / bpx;  // 16-B pieces per block
        const long long i = (long long)(blockIdx.x >> 3) * per + threadIdx.x;
        if (threadIdx.x < per && i < pf16) warm = pf[i];
    }
    const unsigned long long sd = *seed;
    const uint2 key = make_uint2((unsigned)sd, (unsigned)(sd >> 32));
    uint4 in[kDropVpt];
    long long vi[kDropVpt];
#pragma unroll
    for (int k = 0; k < kDropVpt; ++k) {
        vi[k] = (lb * kDropVpt + k) * kBlock + threadIdx.x;
        in[k] = vi[k] < nv ? x[vi[k]] : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int k = 0; k < kDropVpt; ++k) {
        if (vi[k] >= nv) continue;
        const unsigned bits = keep_bits<EPV>(key, vi[k], thresh);
        uint4 o;
        if constexpr (EPV == 8) {
            float v[8];
            unpack8(in[k], v);
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = ((bits >> j) & 1u) ? v[j] * scale : 0.f;
            o = make_uint4(pack2(v[0], v[1]), pack2(v[2], v[3]), pack2(v[4], v[5]), pack2(v[6], v[7]));
        } else {
            const float v[4] = {__uint_as_float(in[k].x), __uint_as_float(in[k].y), __uint_as_float(in[k].z),
                                __uint_as_float(in[k].w)};
            o = make_uint4(__float_as_uint((bits & 1u) ? v[0] * scale : 0.f),
                           __float_as_uint((bits & 2u) ? v[1] * scale : 0.f),
                           __float_as_uint((bits & 4u) ? v[2] * scale : 0.f),
                           __float_as_uint((bits & 8u) ? v[3] * scale : 0.f));
        }
        y[vi[k]] = o;
    }
    asm volatile("" : : "v"(warm.x), "v"(warm.y), "v"(warm.z), "v"(warm.w));  // (the prefetch must land)
}


// ---- 1x1 convolution weight gradient over NCHW activations (the MBConv expand / project convs of
// the trunk, src/models.py:43 via efficientnet_pytorch): dW[co][ci] = sum over images n and pixels q
// of dy[n][co][q] * x[n][ci][q]. A GEMM whose K index (n, q) runs along q in BOTH operands, so the
// v_mfma_f32_16x16x32_bf16 fragments (8 consecutive k per lane) load straight from global memory --
// no LDS staging, no transposes, no fp32 workspace to zero and cast (MIOpen's atomic NHWC solver
// needs both, plus NCHW <-> NHWC transposes). Block = 64 x 64 dW tile x one K range (a split); its
// 4 waves take the range's 32-wide K steps in turn, double-buffered (the next step's 8 fragment loads
// in flight behind the current step's 16 MFMAs), and are summed in LDS in a fixed order; the splits'
// partials are summed by k_pw_wrw_reduce in split order (deterministic).
constexpr int kPwWaves = 4;
constexpr int kPwThreads = kPwWaves * kWave;

using pw_bf16x8 = __attribute__((ext_vector_type(8))) short;
using pw_f32x4 = __attribute__((ext_vector_type(4))) float;

// A lane's fragment of one K step: KS consecutive k (8 or 16) of one row, as KS / 8 MFMA operands. Any
// assignment of k to MFMA slots is a valid GEMM as long as A and B use the same one, so with KS = 16
// a lane's 32 contiguous bytes feed two MFMAs and a row's 4 lanes read one whole 128-B line.
template <int VEC, int KS>  // VEC 8: 16-B loads (HW % 8 == 0); VEC 4: 8-B loads (HW % 4 == 0)
struct PwFrag {
    pw_bf16x8 v[KS / 8];
};

template <int VEC, int KS>
__device__ __forceinline__ PwFrag<VEC, KS> pw_frag(const bf16* __restrict__ p, int q, int HW, bool live) {
    PwFrag<VEC, KS> f;
#pragma unroll
    for (int h = 0; h < KS / 8; ++h) {
        if constexpr (VEC == 8) {
            const bool ok = live && q + 8 * h < HW;
            const uint4 v = ok ? *reinterpret_cast<const uint4*>(p + 8 * h) : make_uint4(0u, 0u, 0u, 0u);
            f.v[h] = __builtin_bit_cast(pw_bf16x8, v);
        } else {
            const bool ok0 = live && q + 8 * h < HW, ok1 = live && q + 8 * h + 4 < HW;
            const uint2 lo = ok0 ? *reinterpret_cast<const uint2*>(p + 8 * h) : make_uint2(0u, 0u);
            const uint2 hi = ok1 ? *reinterpret_cast<const uint2*>(p + 8 * h + 4) : make_uint2(0u, 0u);
            f.v[h] = __builtin_bit_cast(pw_bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
        }
    }
    return f;
}

template <int VEC, int KS>
__global__ __launch_bounds__(kPwThreads) void k_pw_wrw(const bf16* __restrict__ x, const bf16* __restrict__ dy,
                                                      int Cin, int Cout, int HW, int spi, int nsteps, int tiles_n,
                                                      int ntiles, int nsplit, float* __restrict__ partial) {
    constexpr int SW = 4 * KS;                // k per step: 4 lane groups x KS
    __shared__ pw_f32x4 s_red[2][16][kWave];  // two waves' 64 x 64 tiles (16 fragments x 64 lanes)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // XCD-contiguous logical block: consecutive tiles of one split (one K range, whose activation rows
    // the tiles share) run on one XCD and meet in its L2
    const int bpx = gridDim.x >> 3;
    const int lb = (blockIdx.x & 7) * bpx + (blockIdx.x >> 3);
    const int split = lb / ntiles, tile = lb - split * ntiles;
    if (split >= nsplit) return;  // block-uniform (grid padded to a multiple of 8)
    const int m0 = (tile / tiles_n) * 64, n0 = (tile % tiles_n) * 64;
    const int fm = min(4, (Cout - m0 + 15) >> 4), fn = min(4, (Cin - n0 + 15) >> 4);  // live 16-row fragments
    const int t0 = (int)((long long)nsteps * split / nsplit), t1 = (int)((long long)nsteps * (split + 1) / nsplit);
    const int r16 = lane & 15, kq = KS * (lane >> 4);
    int arow[4], brow[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        arow[i] = min(m0 + 16 * i + r16, Cout - 1);  // clamped rows feed only discarded outputs
        brow[i] = min(n0 + 16 * i + r16, Cin - 1);
    }
    pw_f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = pw_f32x4{0.f, 0.f, 0.f, 0.f};
    PwFrag<VEC, KS> a[2][4], b[2][4];
    auto load = [&](int t, PwFrag<VEC, KS>* av, PwFrag<VEC, KS>* bv) {
        const bool live = t < t1;
        t = min(t, nsteps - 1);
        const int n = t / spi;
        const int q = (t - n * spi) * SW + kq;
        const int qq = q < HW ? q : 0;  // (masked halves read nothing; the address stays in the tensor)
        const bf16* ap = dy + (size_t)n * Cout * HW + qq;
        const bf16* bp = x + (size_t)n * Cin * HW + qq;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (i < fm) av[i] = pw_frag<VEC, KS>(ap + (size_t)arow[i] * HW, q, HW, live);
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (j < fn) bv[j] = pw_frag<VEC, KS>(bp + (size_t)brow[j] * HW, q, HW, live);
    };
    auto mma = [&](const PwFrag<VEC, KS>* av, const PwFrag<VEC, KS>* bv) {
#pragma unroll
        for (int h = 0; h < KS / 8; ++h)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (i < fm && j < fn)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i].v[h], bv[j].v[h], acc[i][j], 0, 0, 0);
    };
    int t = t0 + wave;
    if (t < t1) load(t, a[0], b[0]);
    for (; t < t1; t += 2 * kPwWaves) {
        load(t + kPwWaves, a[1], b[1]);  // (past t1: zeros)
        mma(a[0], b[0]);
        if (t + kPwWaves >= t1) break;
        load(t + 2 * kPwWaves, a[0], b[0]);
        mma(a[1], b[1]);
    }
    // waves (0 + 2) and (1 + 3) in LDS, then every wave sums the two for its 16-row block
    if (wave >= 2) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) s_red[wave - 2][4 * i + j][lane] = acc[i][j];
    }
    __syncthreads();
    if (wave < 2) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) s_red[wave][4 * i + j][lane] += acc[i][j];
    }
    __syncthreads();
    const int i = wave;  // this wave writes rows m0 + 16 i + 4 (lane >> 4) + r
    if (i >= fm) return;
    float* out = partial + (size_t)split * Cout * Cin;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int ci = n0 + 16 * j + r16;
        if (j >= fn || ci >= Cin) continue;
        const pw_f32x4 v = s_red[0][4 * i + j][lane] + s_red[1][4 * i + j][lane];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int co = m0 + 16 * i + 4 * (lane >> 4) + r;
            if (co < Cout) out[(size_t)co * Cin + ci] = v[r];
        }
    }
}

// ---- 1x1 convolution forward / backward-data over NCHW bf16 activations (the trunk's MBConv expand /
// project convs): Y[n][m][p] = sum_k A[m][k] X[n][k][p], A = W (forward, [m][k]) or W^T (backward-data,
// W given as [k][m]). MIOpen runs these as batched GEMMs of one image each (15-50 us per layer at c3).
// Here the MFMA rows are PIXELS: D[px][m] = sum_k X^T[px][k] A^T[k][m], so a lane's 4 accumulators are 4
// consecutive pixels of one channel (one 8-B store). Block = 64 pixels (flattened over images) x 64
// channels, 4 waves of 16 channels; the X tile (KC k x 64 px) is staged in LDS as it lies in memory and
// read transposed by ds_read_tr16_b64 (8 consecutive k of one pixel per lane); A comes straight from
// global ([m][k] rows, forward) or through a second LDS tile ([k][m] rows, backward-data). The next
// stage's global loads are in flight while the current stage's MFMAs run.
constexpr int kPgPx = 64, kPgM = 64;
constexpr int kPgRow = kPgPx * 2 + 8;  // LDS bytes per staged k row (+8: spread the banks)

template <int VEC, bool WT, int KC>  // VEC: pixels per X load (8: P % 8 == 0, else 4); WT: A given as [k][m]
__global__ __launch_bounds__(256) void k_pw_gemm(const bf16* __restrict__ X, const bf16* __restrict__ A, int M, int K,
                                                 int P, int ncols, int mtiles, bf16* __restrict__ Y) {
    using v4s = __attribute__((ext_vector_type(4))) short;
    constexpr int XL = KC * (kPgPx / VEC) / 256;            // X loads per thread per stage
    constexpr int WL = WT ? KC * (kPgM / 8) / 256 : KC / 32;  // A loads per thread (WT) / per lane (forward)
    static_assert(XL >= 1 && WL >= 1, "whole loads per thread");
    __shared__ __attribute__((aligned(16))) unsigned char s_x[KC * kPgRow];
    __shared__ __attribute__((aligned(16))) unsigned char s_w[WT ? KC * kPgRow : 16];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int c16 = lane & 15, g = lane >> 4, tq = c16 >> 2, tp = c16 & 3;
    // XCD-contiguous logical block, m-tiles fastest: the m-tiles of one pixel tile (same X rows) share an L2
    const int bpx = gridDim.x >> 3;
    const int lb = (blockIdx.x & 7) * bpx + (blockIdx.x >> 3);
    const int mt = lb % mtiles, jt = lb / mtiles;
    const int j0 = jt * kPgPx, m0 = mt * kPgM;
    if (j0 >= ncols) return;  // block-uniform (grid padded to a multiple of 8)
    // this thread's X chunks: (row, pixel chunk) -> global address (pixels of a chunk never straddle images)
    const uint2 z2 = make_uint2(0u, 0u);
    uint4 xr[XL];
    uint2 xr2[XL];
    uint4 wr[WL], wcur[WT ? 1 : WL];
    auto gload = [&](int kb) {
#pragma unroll
        for (int i = 0; i < XL; ++i) {
            const int c = threadIdx.x + 256 * i;
            const int row = c / (kPgPx / VEC), ch = c - row * (kPgPx / VEC);
            const int col = j0 + ch * VEC, k = kb + row;
            const bool ok = col < ncols && k < K;
            const int n = ok ? col / P : 0, pp = ok ? col - n * P : 0;
            const bf16* src = X + ((size_t)n * K + (ok ? k : 0)) * P + pp;
            if constexpr (VEC == 8) xr[i] = ok ? *reinterpret_cast<const uint4*>(src) : make_uint4(0u, 0u, 0u, 0u);
            else xr2[i] = ok ? *reinterpret_cast<const uint2*>(src) : z2;
        }
        if constexpr (WT) {  // A^T tile rows k, 64 channels each: A[k][m0 .. m0 + 63], 8 per load (M % 8 == 0)
#pragma unroll
            for (int i = 0; i < WL; ++i) {
                const int c = threadIdx.x + 256 * i;
                const int row = c >> 3, ch = c & 7;
                const int k = kb + row, m = m0 + 8 * ch;
                wr[i] = (k < K && m < M) ? *reinterpret_cast<const uint4*>(A + (size_t)k * M + m) : make_uint4(0u, 0u, 0u, 0u);
            }
        } else {  // forward: this lane's B fragments straight from A's rows (K % 8 == 0)
            const int m = m0 + 16 * wave + c16;
#pragma unroll
            for (int i = 0; i < WL; ++i) {
                const int k = kb + 32 * i + 8 * g;
                wr[i] = (m < M && k < K) ? *reinterpret_cast<const uint4*>(A + (size_t)m * K + k) : make_uint4(0u, 0u, 0u, 0u);
            }
        }
    };
    auto lstore = [&]() {
#pragma unroll
        for (int i = 0; i < XL; ++i) {
            const int c = threadIdx.x + 256 * i;
            const int row = c / (kPgPx / VEC), ch = c - row * (kPgPx / VEC);
            if constexpr (VEC == 8) *reinterpret_cast<uint4*>(s_x + row * kPgRow + ch * 16) = xr[i];
            else *reinterpret_cast<uint2*>(s_x + row * kPgRow + ch * 8) = xr2[i];
        }
        if constexpr (WT) {
#pragma unroll
            for (int i = 0; i < WL; ++i) {
                const int c = threadIdx.x + 256 * i;
                *reinterpret_cast<uint4*>(s_w + (c >> 3) * kPgRow + (c & 7) * 16) = wr[i];
            }
        } else {
#pragma unroll
            for (int i = 0; i < WL; ++i) wcur[i] = wr[i];
        }
    };
    auto tr8 = [&](const unsigned char* s, int step, int col0) {  // 8 consecutive k (step) of column col0 + c16
        const unsigned char* base = s + (32 * step + 8 * g + tq) * kPgRow + (col0 + 4 * tp) * 2;
        const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(base));
        const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(base + 4 * kPgRow));
        return pw_bf16x8{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    };
    pw_f32x4 acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = pw_f32x4{0.f, 0.f, 0.f, 0.f};
    gload(0);
    for (int kb = 0; kb < K; kb += KC) {
        __syncthreads();  // the previous stage's reads of s_x / s_w are done
        lstore();
        __syncthreads();
        if (kb + KC < K) gload(kb + KC);  // in flight behind this stage's MFMAs
#pragma unroll
        for (int st = 0; st < KC / 32; ++st) {
            if (kb + 32 * st >= K) break;
            pw_bf16x8 b;
            if constexpr (WT) b = tr8(s_w, st, 16 * wave);
            else b = __builtin_bit_cast(pw_bf16x8, wcur[st]);
#pragma unroll
            for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tr8(s_x, st, 16 * t), b, acc[t], 0, 0, 0);
        }
    }
    // D[px][m]: this lane holds channel m0 + 16 wave + c16, pixels 16 t + 4 g + 0..3
    const int m = m0 + 16 * wave + c16;
    if (m >= M) return;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int col = j0 + 16 * t + 4 * g;
        if (col >= ncols) continue;
        const int n = col / P, pp = col - n * P;
        *reinterpret_cast<uint2*>(Y + ((size_t)n * M + m) * P + pp) =
            make_uint2(pack2(acc[t][0], acc[t][1]), pack2(acc[t][2], acc[t][3]));
    }
}

// dw[e] = sum over splits s (in order) of partial[s][e], nsplit <= kPwMaxSplit. Four consecutive
// elements per lane (16-B loads); the splits of a lane's elements are shared by G waves of the block
// (G = 1 for nsplit <= 16, else 16), each summing its run of <= 16 consecutive splits with every
// load in flight at once, then the G sums in order.
constexpr int kPwMaxSplit = 256;
template <typename T, int G>
__global__ __launch_bounds__(G == 1 ? 256 : 1024) void k_pw_wrw_reduce(const float* __restrict__ partial, int nsplit,
                                                                       int E, T* __restrict__ dw) {
    constexpr int kThreads = G == 1 ? 256 : 1024;
    __shared__ float4 s_sum[G][kWave];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int chunk = G == 1 ? blockIdx.x * (kThreads / kWave) + wave : blockIdx.x;  // 64 lanes x 4 elements
    const int e = (chunk * kWave + lane) * 4;
    const int gw = G == 1 ? 0 : wave;
    const int per = (nsplit + G - 1) / G, s0 = gw * per, s1 = min(s0 + per, nsplit);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (e < E) {
        float4 p[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            if (s0 + k < s1) {
                const float* src = partial + (size_t)(s0 + k) * E + e;
                p[k] = (E & 3) == 0 ? *reinterpret_cast<const float4*>(src)  // (16-B aligned rows)
                                    : make_float4(src[0], e + 1 < E ? src[1] : 0.f, e + 2 < E ? src[2] : 0.f,
                                                  e + 3 < E ? src[3] : 0.f);
            } else {
                p[k] = make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            v.x += p[k].x;
            v.y += p[k].y;
            v.z += p[k].z;
            v.w += p[k].w;
        }
    }
    if constexpr (G > 1) {
        s_sum[wave][lane] = v;
        __syncthreads();
        if (wave != 0) return;
        v = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int w = 0; w < G; ++w) {
            const float4 t = s_sum[w][lane];
            v.x += t.x;
            v.y += t.y;
            v.z += t.z;
            v.w += t.w;
        }
    }
    if (e >= E) return;
    const float o[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (e + k < E) st(dw + e + k, o[k]);
}


__device__ __forceinline__ void ldv8(const float* p, float* o) {
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}
__device__ __forceinline__ void ldv8(const bf16* p, float* o) {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        o[2 * i] = __uint_as_float(w[i] << 16);
        o[2 * i + 1] = __uint_as_float(w[i] & 0xFFFF0000u);
    }
}
__device__ __forceinline__ void stv8(float* p, const float* v) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}
__device__ __forceinline__ void stv8(bf16* p, const float* v) {
    bf16 b[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) b[i] = __float2bfloat16(v[i]);
    *reinterpret_cast<uint4*>(p) = *reinterpret_cast<const uint4*>(b);
}
__device__ __forceinline__ void st1(float* p, float v) { *p = v; }
__device__ __forceinline__ void st1(bf16* p, float v) { *p = __float2bfloat16(v); }

// ---- SimpleLoss (src/tools.py:222-230): BCEWithLogitsLoss(pos_weight), mean over the n elements,
// with its input gradient computed in the same pass. Per element (torch's formula for pos_weight):
//   lw = 1 + (pw - 1) t,  l = (1 - t) x + lw (log1p(exp(-|x|)) + max(-x, 0)),
//   dl/dx = lw sigmoid(x) - pw t = (1 - t) sigmoid(x) - pw t sigmoid(-x)
// Thread = 8 consecutive elements; block sums in a fixed order (wave butterflies, then the 4 waves
// in order) into partial[block]; k_bce_total folds the partials in block order. fp32 arithmetic for
// fp32 and bf16 logits (a bf16 input is the same as its exact fp32 cast); the gradient (times 1 / n)
// is written in the logits' type.
constexpr int kBceVpt = 8;
template <typename T>
__global__ __launch_bounds__(kBlock) void k_bce_fwd(const T* __restrict__ x, const float* __restrict__ t, long long n,
                                                    float pw, float inv_n, float* __restrict__ partial,
                                                    T* __restrict__ grad) {
    __shared__ float s_w[kBlock / kWave];
    const long long i0 = ((long long)blockIdx.x * kBlock + threadIdx.x) * kBceVpt;
    float xv[kBceVpt], tv[kBceVpt], gv[kBceVpt];
    const bool full = i0 + kBceVpt <= n;
    if (full) {
        ldv8(x + i0, xv);
        const float4 a = *reinterpret_cast<const float4*>(t + i0), b = *reinterpret_cast<const float4*>(t + i0 + 4);
        tv[0] = a.x; tv[1] = a.y; tv[2] = a.z; tv[3] = a.w; tv[4] = b.x; tv[5] = b.y; tv[6] = b.z; tv[7] = b.w;
    } else {
#pragma unroll
        for (int j = 0; j < kBceVpt; ++j) {
            xv[j] = i0 + j < n ? ld(x + i0 + j) : 0.f;
            tv[j] = i0 + j < n ? t[i0 + j] : 0.f;
        }
    }
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < kBceVpt; ++j) {
        const float xx = xv[j], tt = tv[j];
        const float lw = fmaf(pw - 1.f, tt, 1.f);
        const float e = expf(-fabsf(xx));
        const float l = (1.f - tt) * xx + lw * (log1pf(e) + fmaxf(-xx, 0.f));
        // lw sigmoid(x) - pw t = (1 - t) sigmoid(x) - pw t sigmoid(-x): no cancellation for saturated x
        const float sp = 1.f / (1.f + e), sn = e / (1.f + e);  // sigmoid(|x|), sigmoid(-|x|)
        const float sx = xx >= 0.f ? sp : sn, smx = xx >= 0.f ? sn : sp;
        gv[j] = ((1.f - tt) * sx - pw * tt * smx) * inv_n;
        if (i0 + j < n) s += l;
    }
    if (full) stv8(grad + i0, gv);
    else {
#pragma unroll
        for (int j = 0; j < kBceVpt; ++j)
            if (i0 + j < n) st1(grad + i0 + j, gv[j]);
    }
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, kWave);
    if ((threadIdx.x & (kWave - 1)) == 0) s_w[threadIdx.x / kWave] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        float b = 0.f;
#pragma unroll
        for (int w = 0; w < kBlock / kWave; ++w) b += s_w[w];
        partial[blockIdx.x] = b;
    }
}

// dx = grad * gout[0] (the incoming gradient of the loss, read on the device), rounded once to T
template <typename T>
__global__ __launch_bounds__(kBlock) void k_bce_bwd(const T* __restrict__ grad, long long n, const float* __restrict__ gout,
                                                    T* __restrict__ dx) {
    const long long i0 = ((long long)blockIdx.x * kBlock + threadIdx.x) * kBceVpt;
    const float gs = gout[0];
    float v[kBceVpt];
    if (i0 + kBceVpt <= n) {
        ldv8(grad + i0, v);
#pragma unroll
        for (int j = 0; j < kBceVpt; ++j) v[j] *= gs;
        stv8(dx + i0, v);
    } else {
        for (long long i = i0; i < n; ++i) st1(dx + i, ld(grad + i) * gs);
    }
}

// Per-channel sums of an NCHW tensor (the depthnet bias gradient from d(logits), src/models.py:47):
// block = channel, the (image, pixel) elements strided over the threads, 4 loads in flight per thread,
// then a fixed-order block reduction (deterministic).
template <typename T>
__global__ __launch_bounds__(kBlock) void k_channel_sums(const T* __restrict__ x, int N, int C, int HW,
                                                         float* __restrict__ out) {
    __shared__ float s_w[kBlock / kWave];
    const int c = blockIdx.x;
    const int total = N * HW;
    float s = 0.f;
    int e = threadIdx.x;
    for (; e + 3 * kBlock < total; e += 4 * kBlock) {
        float v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = e + u * kBlock, n = i / HW, p = i - n * HW;
            v[u] = ld(x + ((size_t)n * C + c) * HW + p);
        }
        s += (v[0] + v[1]) + (v[2] + v[3]);
    }
    for (; e < total; e += kBlock) {
        const int n = e / HW, p = e - n * HW;
        s += ld(x + ((size_t)n * C + c) * HW + p);
    }
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, kWave);
    if ((threadIdx.x & (kWave - 1)) == 0) s_w[threadIdx.x / kWave] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        float b = 0.f;
#pragma unroll
        for (int w = 0; w < kBlock / kWave; ++w) b += s_w[w];
        out[c] = b;
    }
}

// loss = (sum of the block partials, lanes strided over blocks then a fixed butterfly) / n
__global__ __launch_bounds__(kWave) void k_bce_total(const float* __restrict__ partial, int nb, float inv_n,
                                                     float* __restrict__ loss) {
    float s = 0.f;
    for (int b = threadIdx.x; b < nb; b += kWave) s += partial[b];
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, kWave);
    if (threadIdx.x == 0) loss[0] = s * inv_n;
}
}  // namespace

extern "C" {

int lss_head1_blocks(int32_t P) { return P > 0 ? (P + kHeadRows - 1) / kHeadRows : 0; }

int lss_head1_fwd(const void* x, const float* w, const float* bias, int32_t P, int32_t C, void* y, void* stream) {
    return lss_head1_fwd2(x, w, bias, P, C, nullptr, y, stream);
}
int lss_head1_fwd2(const void* x, const float* w, const float* bias, int32_t P, int32_t C, const float* bn_stats,
                   void* y, void* stream) {
    if (!x || !w || !y || P <= 0 || C <= 0 || C % 8 != 0 || 64 % (C / 8) != 0) return LSS_CONV_EINVAL;
    const dim3 gr(lss_head1_blocks(P)), bl(kBlock);
    hipStream_t s = (hipStream_t)stream;
#define LSS_HEAD1_FWD(L) \
    hipLaunchKernelGGL((k_head1_fwd<L>), gr, bl, 0, s, (const uint4*)x, w, bias, P, (bf16*)y, bn_stats)
    switch (C / 8) {
        case 16: LSS_HEAD1_FWD(16); break;
        case 8: LSS_HEAD1_FWD(8); break;
        case 32: LSS_HEAD1_FWD(32); break;
        case 64: LSS_HEAD1_FWD(64); break;
        case 4: LSS_HEAD1_FWD(4); break;
        case 2: LSS_HEAD1_FWD(2); break;
        case 1: LSS_HEAD1_FWD(1); break;
        default: return LSS_CONV_EINVAL;
    }
#undef LSS_HEAD1_FWD
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}
int lss_head1_bwd(const void* x, const void* dy, const float* w, int32_t P, int32_t C, void* dx, float* partial,
                  void* stream) {
    if (!dx) return LSS_CONV_EINVAL;
    return lss_head1_bwd2(x, dy, w, P, C, nullptr, dx, partial, stream);
}
int lss_head1_bwd2(const void* x, const void* dy, const float* w, int32_t P, int32_t C, const float* bn_stats, void* dx,
                   float* partial, void* stream) {
    if (!x || !dy || !w || (!dx && !bn_stats) || !partial || P <= 0 || C <= 0 || C % 8 != 0 || 64 % (C / 8) != 0)
        return LSS_CONV_EINVAL;
    const dim3 gr(lss_head1_blocks(P)), bl(kBlock);
    hipStream_t s = (hipStream_t)stream;
#define LSS_HEAD1_BWD(L)                                                                                          \
    hipLaunchKernelGGL((k_head1_bwd<L>), gr, bl, 0, s, (const uint4*)x, (const bf16*)dy, w, P, (uint4*)dx, partial, \
                       bn_stats)
    switch (C / 8) {
        case 16: LSS_HEAD1_BWD(16); break;
        case 8: LSS_HEAD1_BWD(8); break;
        case 32: LSS_HEAD1_BWD(32); break;
        case 64: LSS_HEAD1_BWD(64); break;
        case 4: LSS_HEAD1_BWD(4); break;
        case 2: LSS_HEAD1_BWD(2); break;
        case 1: LSS_HEAD1_BWD(1); break;
        default: return LSS_CONV_EINVAL;
    }
#undef LSS_HEAD1_BWD
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

// split count of lss_pw_wrw: about 512 blocks (2 per CU) and >= 2 K steps per wave, at most
// kPwMaxSplit, and the fp32 partials at most half the activation bytes (or one split)
static void pw_plan(int N, int Cin, int Cout, int HW, int* spi, int* nsteps, int* tiles_n, int* ntiles, int* nsplit) {
    *spi = (HW + 63) / 64;
    *nsteps = N * *spi;
    *tiles_n = (Cin + 63) / 64;
    *ntiles = ((Cout + 63) / 64) * *tiles_n;
    long s = (512 + *ntiles - 1) / *ntiles;
    s = std::min(s, (long)std::max(1, *nsteps / (2 * kPwWaves)));
    const long in_bytes = 2L * N * HW * (Cin + Cout), per_split = 4L * Cin * Cout;
    s = std::min(s, std::max(1L, in_bytes / (2 * per_split)));
    *nsplit = (int)std::max(1L, std::min(s, (long)kPwMaxSplit));
}

int64_t lss_pw_wrw_workspace_bytes(int32_t N, int32_t Cin, int32_t Cout, int32_t HW) {
    if (N <= 0 || Cin <= 0 || Cout <= 0 || HW <= 0) return 0;
    int spi, nsteps, tiles_n, ntiles, nsplit;
    pw_plan(N, Cin, Cout, HW, &spi, &nsteps, &tiles_n, &ntiles, &nsplit);
    return (int64_t)nsplit * Cout * Cin * (int64_t)sizeof(float);
}

int lss_pw_wrw(const void* x, const void* dy, int32_t N, int32_t Cin, int32_t Cout, int32_t HW, void* dw,
               int32_t dw_dtype, void* workspace, int64_t workspace_bytes, void* stream) {
    if (!x || !dy || !dw || !workspace || N <= 0 || Cin <= 0 || Cout <= 0 || HW <= 0 || HW % 4 != 0 ||
        (dw_dtype != LSS_CONV_F32 && dw_dtype != LSS_CONV_BF16) || (long)N * ((HW + 31) / 32) >= INT_MAX ||
        (long)N * std::max(Cin, Cout) * HW >= INT_MAX ||
        ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(dy)) & 7) ||
        workspace_bytes < lss_pw_wrw_workspace_bytes(N, Cin, Cout, HW))
        return LSS_CONV_EINVAL;
    int spi, nsteps, tiles_n, ntiles, nsplit;
    pw_plan(N, Cin, Cout, HW, &spi, &nsteps, &tiles_n, &ntiles, &nsplit);
    const long blocks = 8L * (((long)ntiles * nsplit + 7) / 8);
    hipStream_t s = (hipStream_t)stream;
    float* part = (float*)workspace;
    const bool v8 = HW % 8 == 0 && ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(dy)) & 15) == 0;
    if (v8)
        hipLaunchKernelGGL((k_pw_wrw<8, 16>), dim3((unsigned)blocks), dim3(kPwThreads), 0, s, (const bf16*)x,
                           (const bf16*)dy, Cin, Cout, HW, spi, nsteps, tiles_n, ntiles, nsplit, part);
    else
        hipLaunchKernelGGL((k_pw_wrw<4, 16>), dim3((unsigned)blocks), dim3(kPwThreads), 0, s, (const bf16*)x,
                           (const bf16*)dy, Cin, Cout, HW, spi, nsteps, tiles_n, ntiles, nsplit, part);
    const int E = Cout * Cin;
    const int chunks = (E + 4 * kWave - 1) / (4 * kWave);  // 64 lanes x 4 elements
#define LSS_PW_REDUCE(T)                                                                                          \
    if (nsplit <= 16)                                                                                             \
        hipLaunchKernelGGL((k_pw_wrw_reduce<T, 1>), dim3((chunks + 3) / 4), dim3(256), 0, s, (const float*)part,  \
                           nsplit, E, (T*)dw);                                                                    \
    else                                                                                                          \
        hipLaunchKernelGGL((k_pw_wrw_reduce<T, 16>), dim3(chunks), dim3(1024), 0, s, (const float*)part, nsplit, E, \
                           (T*)dw)
    if (dw_dtype == LSS_CONV_BF16) {
        LSS_PW_REDUCE(bf16);
    } else {
        LSS_PW_REDUCE(float);
    }
#undef LSS_PW_REDUCE
    return launch_status();
}

int lss_pw_conv(const void* x, const void* a, int32_t a_layout, int32_t N, int32_t K, int32_t M, int32_t HW, void* y,
                void* stream) {
    if (!x || !a || !y || N <= 0 || K <= 0 || M <= 0 || HW <= 0 || HW % 4 != 0 || K % 8 != 0 || M % 8 != 0 ||
        (a_layout != LSS_PW_MK && a_layout != LSS_PW_KM) || (long)N * HW >= INT_MAX ||
        (long)N * std::max(K, M) * HW >= INT_MAX ||
        ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y) | reinterpret_cast<uintptr_t>(a)) & 15))
        return LSS_CONV_EINVAL;
    const int ncols = N * HW, mtiles = (M + kPgM - 1) / kPgM;
    const long tiles = (long)mtiles * ((ncols + kPgPx - 1) / kPgPx);
    const long blocks = 8L * ((tiles + 7) / 8);
    if (blocks > INT_MAX) return LSS_CONV_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    const bool v8 = HW % 8 == 0, wt = a_layout == LSS_PW_KM, small = K <= 64;
#define LSS_PW_GEMM(V, W, KC)                                                                                      \
    hipLaunchKernelGGL((k_pw_gemm<V, W, KC>), dim3((unsigned)blocks), dim3(256), 0, s, (const bf16*)x, (const bf16*)a, \
                       M, K, HW, ncols, mtiles, (bf16*)y)
    if (v8) {
        if (wt) { if (small) LSS_PW_GEMM(8, true, 32); else LSS_PW_GEMM(8, true, 128); }
        else { if (small) LSS_PW_GEMM(8, false, 32); else LSS_PW_GEMM(8, false, 128); }
    } else {
        if (wt) { if (small) LSS_PW_GEMM(4, true, 32); else LSS_PW_GEMM(4, true, 128); }
        else { if (small) LSS_PW_GEMM(4, false, 32); else LSS_PW_GEMM(4, false, 128); }
    }
#undef LSS_PW_GEMM
    return launch_status();
}

int lss_dwconv_fwd(const void* x, int32_t dtype, const float* w, int32_t N, int32_t C, int32_t Hi, int32_t Wi,
                   int32_t K, int32_t stride, int32_t pad_top, int32_t pad_left, int32_t Ho, int32_t Wo, void* y,
                   void* stream) {
    if (!x || !w || !y || !geo_ok(N, C, Hi, Wi, K, stride, Ho, Wo)) return LSS_CONV_EINVAL;
    const DwGeo g{C, Hi, Wi, Ho, Wo, pad_top, pad_left, N * C};
    return dispatch_kst<Fwd>(K, stride, dtype, x, w, g, 0, y, (hipStream_t)stream);
}

int lss_dwconv_bwd_data(const void* dy, int32_t dtype, const float* w, int32_t N, int32_t C, int32_t Hi, int32_t Wi,
                        int32_t K, int32_t stride, int32_t pad_top, int32_t pad_left, int32_t Ho, int32_t Wo, void* dx,
                        void* stream) {
    if (!dy || !w || !dx || !geo_ok(N, C, Hi, Wi, K, stride, Ho, Wo)) return LSS_CONV_EINVAL;
    const DwGeo g{C, Hi, Wi, Ho, Wo, pad_top, pad_left, N * C};
    return dispatch_kst<BwdData>(K, stride, dtype, dy, w, g, dx, (hipStream_t)stream);
}

int lss_dwconv_bwd_weight(const void* x, const void* dy, int32_t dtype, int32_t N, int32_t C, int32_t Hi, int32_t Wi,
                          int32_t K, int32_t stride, int32_t pad_top, int32_t pad_left, int32_t Ho, int32_t Wo,
                          int32_t ngroups, float* partial, void* stream) {
    if (!x || !dy || !partial || ngroups <= 0 || ngroups > N || !geo_ok(N, C, Hi, Wi, K, stride, Ho, Wo))
        return LSS_CONV_EINVAL;
    const DwGeo g{C, Hi, Wi, Ho, Wo, pad_top, pad_left, N * C};
    return dispatch_kst<BwdWeight>(K, stride, dtype, x, dy, g, (int)N, (int)ngroups, partial, DwFold{nullptr, nullptr},
                                   (hipStream_t)stream);
}

int lss_dwconv_bwd_weight2(const void* x, const void* dy, int32_t dtype, int32_t N, int32_t C, int32_t Hi, int32_t Wi,
                           int32_t K, int32_t stride, int32_t pad_top, int32_t pad_left, int32_t Ho, int32_t Wo,
                           int32_t ngroups, float* partial, uint32_t* sync, float* dw, void* stream) {
    if (!x || !dy || !partial || !sync || !dw || ngroups <= 0 || ngroups > N || C > kDwSyncMaxC ||
        !geo_ok(N, C, Hi, Wi, K, stride, Ho, Wo))
        return LSS_CONV_EINVAL;
    const DwGeo g{C, Hi, Wi, Ho, Wo, pad_top, pad_left, N * C};
    return dispatch_kst<BwdWeight>(K, stride, dtype, x, dy, g, (int)N, (int)ngroups, partial, DwFold{sync, dw},
                                   (hipStream_t)stream);
}

int lss_scale_add(const void* x, const void* u, float keep, const void* res, int64_t N, int64_t per, void* y,
                  void* stream) {
    if (!x || !u || !y || !(keep > 0.f && keep <= 1.f) || N <= 0 || per <= 0 || per % 8 != 0 ||
        ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(res) | reinterpret_cast<uintptr_t>(y)) & 15))
        return LSS_CONV_EINVAL;
    const long long n8 = (long long)N * per / 8;
    const long long nb = (n8 + kBlock - 1) / kBlock;
    if (nb > INT_MAX) return LSS_CONV_EINVAL;
    hipLaunchKernelGGL(k_scale_add, dim3((unsigned)nb), dim3(kBlock), 0, (hipStream_t)stream, (const uint4*)x, (const bf16*)u,
                       keep, (const uint4*)res, (long long)(per / 8), n8, (uint4*)y);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}


}  // extern "C"

namespace {
// wt[i][o][a][b] = w[o][i][K-1-a][K-1-b], written channels-last ([i][a][b][o] in memory): the weight of a
// stride-1 transposed convolution as a forward one (models._Conv3x3's backward-data). One thread per
// output element, consecutive threads along o (coalesced writes; the reads are a 1.2 MB weight, in L2).
template <typename T>
__global__ __launch_bounds__(kBlock) void k_conv_flip_weight(const T* __restrict__ w, int O, int I, int K, int cl_in,
                                                             T* __restrict__ wt) {
    const long e = (long)blockIdx.x * kBlock + threadIdx.x;
    const long n = (long)O * I * K * K;
    if (e >= n) return;
    const int o = (int)(e % O);
    long r = e / O;
    const int b = (int)(r % K);
    r /= K;
    const int a = (int)(r % K);
    const int i = (int)(r / K);
    const int ka = K - 1 - a, kb = K - 1 - b;
    const long src = cl_in ? (((long)o * K + ka) * K + kb) * I + i : (((long)o * I + i) * K + ka) * K + kb;
    wt[e] = w[src];
}

// The tiled form: per tap, a 64 x 64 (o, i) tile read along i (coalesced for channels-last weights,
// whose innermost index is i; 9-element strides for contiguous ones) and written along o (wt's innermost)
// through an LDS transpose (odd row stride); each thread's 16 loads are issued together (a loop that
// loaded and stored one element per iteration took 11 us per weight: 16 dependent round trips).
template <typename T>
__global__ __launch_bounds__(kBlock) void k_conv_flip_weight_cl(const T* __restrict__ w, int O, int I, int K, int cl,
                                                                T* __restrict__ wt) {
    __shared__ T tile[64][65];
    const int ti = (I + 63) / 64, to = (O + 63) / 64;
    int b = blockIdx.x;
    const int it = b % ti;
    b /= ti;
    const int ot = b % to;
    const int tap = b / to;  // output tap (a, b) = (tap / K, tap % K); source tap K*K - 1 - tap
    const int i0 = it * 64, o0 = ot * 64, src_tap = K * K - 1 - tap;
    const long so = (long)K * K * I, si = cl ? 1 : K * K, st = cl ? I : 1;
    const int c = threadIdx.x & 63, r0 = threadIdx.x >> 6;
    constexpr int R = 64 / (kBlock / 64);
    T v[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {  // rows o, columns i (clamped addresses, all loads in flight)
        const int o = min(o0 + r0 + k * (kBlock / 64), O - 1), i = min(i0 + c, I - 1);
        v[k] = w[o * so + src_tap * st + i * si];
    }
#pragma unroll
    for (int k = 0; k < R; ++k) tile[r0 + k * (kBlock / 64)][c] = v[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < R; ++k) {  // rows i, columns o
        const int i = i0 + r0 + k * (kBlock / 64), o = o0 + c;
        if (o < O && i < I) wt[((long)i * K * K + tap) * O + o] = tile[c][r0 + k * (kBlock / 64)];
    }
}
}  // namespace

extern "C" {

int lss_conv_flip_weight(const void* w, int32_t dtype, int32_t O, int32_t I, int32_t K, int32_t w_layout, void* wt,
                         void* stream) {
    if (!w || !wt || O <= 0 || I <= 0 || K <= 0 || (dtype != LSS_CONV_BF16 && dtype != LSS_CONV_F32) ||
        (w_layout != LSS_CONV_NCHW && w_layout != LSS_CONV_NHWC))
        return LSS_CONV_EINVAL;
    const long n = (long)O * I * K * K;
    if (n >= INT_MAX) return LSS_CONV_EINVAL;
    const int cl = w_layout == LSS_CONV_NHWC;
    const unsigned grid = (unsigned)((n + kBlock - 1) / kBlock);
    hipStream_t s = (hipStream_t)stream;
    if (O >= 64 && I >= 64) {
        const unsigned gcl = (unsigned)(((I + 63) / 64) * ((O + 63) / 64) * K * K);
        if (dtype == LSS_CONV_BF16)
            hipLaunchKernelGGL(k_conv_flip_weight_cl<bf16>, dim3(gcl), dim3(kBlock), 0, s, (const bf16*)w, O, I, K, cl,
                               (bf16*)wt);
        else
            hipLaunchKernelGGL(k_conv_flip_weight_cl<float>, dim3(gcl), dim3(kBlock), 0, s, (const float*)w, O, I, K,
                               cl, (float*)wt);
    } else if (dtype == LSS_CONV_BF16)
        hipLaunchKernelGGL(k_conv_flip_weight<bf16>, dim3(grid), dim3(kBlock), 0, s, (const bf16*)w, O, I, K, cl, (bf16*)wt);
    else
        hipLaunchKernelGGL(k_conv_flip_weight<float>, dim3(grid), dim3(kBlock), 0, s, (const float*)w, O, I, K, cl,
                           (float*)wt);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

int lss_dropout(const void* x, int32_t dtype, int64_t n, const uint64_t* seed, float keep, void* y, const void* prefetch,
                int64_t prefetch_bytes, void* stream) {
    const int esz = dtype == LSS_CONV_BF16 ? 2 : dtype == LSS_CONV_F32 ? 4 : 0;
    if (!x || !y || !seed || !esz || n <= 0 || (n * esz) % 16 != 0 || !(keep > 0.f && keep <= 1.f) ||
        prefetch_bytes < 0 || (prefetch && prefetch_bytes % 16 != 0) ||
        ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y) | reinterpret_cast<uintptr_t>(prefetch)) & 15))
        return LSS_CONV_EINVAL;
    const long long nv = n * esz / 16;
    const long long nb = (nv + (long long)kBlock * kDropVpt - 1) / ((long long)kBlock * kDropVpt);
    const long long grid = 8 * ((nb + 7) / 8);  // logical blocks past nb write nothing
    if (grid > INT_MAX) return LSS_CONV_EINVAL;
    // keep when (24 random bits) < keep * 2^24; the kept elements are scaled by 1 / keep (torch's dropout)
    const unsigned thresh = (unsigned)fminf(keep * 16777216.0f, 16777216.0f);
    const float scale = 1.0f / keep;
    hipStream_t s = (hipStream_t)stream;
    const uint4* pf = prefetch_bytes > 0 ? (const uint4*)prefetch : nullptr;
    if (esz == 2)
        hipLaunchKernelGGL(k_dropout<bf16>, dim3((unsigned)grid), dim3(kBlock), 0, s, (const uint4*)x, nv,
                           (const unsigned long long*)seed, thresh, scale, (uint4*)y, pf, prefetch_bytes / 16);
    else
        hipLaunchKernelGGL(k_dropout<float>, dim3((unsigned)grid), dim3(kBlock), 0, s, (const uint4*)x, nv,
                           (const unsigned long long*)seed, thresh, scale, (uint4*)y, pf, prefetch_bytes / 16);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

int lss_bce_logits(const void* x, int32_t dtype, const float* target, int64_t n, float pos_weight, float* partial,
                   float* loss, void* grad, void* stream) {
    const int esz = dtype == LSS_CONV_BF16 ? 2 : dtype == LSS_CONV_F32 ? 4 : 0;
    if (!x || !target || !partial || !loss || !grad || !esz || n <= 0 ||
        ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(grad)) & 15) ||
        (reinterpret_cast<uintptr_t>(target) & 15))
        return LSS_CONV_EINVAL;
    const long long nb = (n + (long long)kBlock * kBceVpt - 1) / ((long long)kBlock * kBceVpt);
    if (nb > INT_MAX) return LSS_CONV_EINVAL;
    const float inv_n = 1.0f / (float)n;
    hipStream_t s = (hipStream_t)stream;
    if (esz == 2)
        hipLaunchKernelGGL(k_bce_fwd<bf16>, dim3((unsigned)nb), dim3(kBlock), 0, s, (const bf16*)x, target, (long long)n,
                           pos_weight, inv_n, partial, (bf16*)grad);
    else
        hipLaunchKernelGGL(k_bce_fwd<float>, dim3((unsigned)nb), dim3(kBlock), 0, s, (const float*)x, target,
                           (long long)n, pos_weight, inv_n, partial, (float*)grad);
    hipLaunchKernelGGL(k_bce_total, dim3(1), dim3(kWave), 0, s, partial, (int)nb, inv_n, loss);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

int lss_bce_logits_bwd(const void* grad, int32_t dtype, int64_t n, const float* grad_loss, void* dx, void* stream) {
    const int esz = dtype == LSS_CONV_BF16 ? 2 : dtype == LSS_CONV_F32 ? 4 : 0;
    if (!grad || !grad_loss || !dx || !esz || n <= 0 ||
        ((reinterpret_cast<uintptr_t>(grad) | reinterpret_cast<uintptr_t>(dx)) & 15))
        return LSS_CONV_EINVAL;
    const long long nb = (n + (long long)kBlock * kBceVpt - 1) / ((long long)kBlock * kBceVpt);
    if (nb > INT_MAX) return LSS_CONV_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    if (esz == 2)
        hipLaunchKernelGGL(k_bce_bwd<bf16>, dim3((unsigned)nb), dim3(kBlock), 0, s, (const bf16*)grad, (long long)n,
                           grad_loss, (bf16*)dx);
    else
        hipLaunchKernelGGL(k_bce_bwd<float>, dim3((unsigned)nb), dim3(kBlock), 0, s, (const float*)grad, (long long)n,
                           grad_loss, (float*)dx);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

int lss_channel_sums(const void* x, int32_t dtype, int32_t N, int32_t C, int32_t HW, float* out, void* stream) {
    if (!x || !out || N <= 0 || C <= 0 || HW <= 0 || (long long)N * C * HW >= INT_MAX ||
        (dtype != LSS_CONV_BF16 && dtype != LSS_CONV_F32))
        return LSS_CONV_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    if (dtype == LSS_CONV_BF16)
        hipLaunchKernelGGL(k_channel_sums<bf16>, dim3(C), dim3(kBlock), 0, s, (const bf16*)x, N, C, HW, out);
    else
        hipLaunchKernelGGL(k_channel_sums<float>, dim3(C), dim3(kBlock), 0, s, (const float*)x, N, C, HW, out);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

int64_t lss_bce_partials(int64_t n) { return (n + (int64_t)kBlock * kBceVpt - 1) / ((int64_t)kBlock * kBceVpt); }

}  // extern "C"

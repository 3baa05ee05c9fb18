// lss_hip.hip -- gfx950 (MI355X / CDNA4) kernels of the Lift-Splat hot path + C ABI.
//
// Compiled with -ffp-contract=off: the geometry must reproduce the reference's
// un-fused fp32 arithmetic bit for bit. Kernels that may
// fuse say so explicitly.
//
// Pipeline (forward, one training step):
//   lss_camera_inverse      48 cameras, fp64 adjugate
//   lss_geometry_cells      1 thread / point: frustum -> ego xyz -> cell id, atomic count
//   lss_csr_build           counting sort: block reduce -> scan -> scatter of (cell, point) keys ->
//                           canonical order (point id inside a cell) + context-row index per entry
//   lss_lift_prep           1 block / 64 pixels: depth softmax + context -> pixel-major rows
//   lss_splat_fwd           channels-last: 1 wave / 64-entry CSR chunk (ordered per-cell sums, rows stored
//                           directly) + 1 wave / 64 cells zero-filling empty rows  <- the HBM-bound kernel
//                           NCHW: 1 block (8 waves) / BEV row tile, LDS accumulator, transposed write
// Backward:
//   lss_bev_rows            NCHW dbev -> compact per-cell rows (occupied cells only)
//   lss_splat_bwd           1 wave / pixel: 16-B gathers of D rows to LDS, d_ctx, d_depth, softmax bwd

#include <hip/hip_runtime.h>
#include <atomic>
#include <hip/hip_bf16.h>
#include <hip/hip_ext.h>
#include <algorithm>
#include <limits.h>
#include <stdint.h>
#include <type_traits>

#include "lss_hip.h"

namespace {

constexpr int kC = 64;       // camC (src/models.py:148)
constexpr int kWave = 64;
constexpr int kBlock = 256;
constexpr int kScanItems = 4096;  // cells per scan block (1024 threads x 4)

using bf16 = __hip_bfloat16;
using u32x4 = __attribute__((ext_vector_type(4))) unsigned;
using u32x2 = __attribute__((ext_vector_type(2))) unsigned;

__device__ __forceinline__ float to_f32(float v) { return v; }
__device__ __forceinline__ float to_f32(bf16 v) { return __bfloat162float(v); }

template <typename T> __device__ __forceinline__ T from_f32(float v);
template <> __device__ __forceinline__ float from_f32<float>(float v) { return v; }
template <> __device__ __forceinline__ bf16 from_f32<bf16>(float v) { return __float2bfloat16(v); }

// 4 consecutive elements, 16 B (fp32) or 8 B (bf16) store.
__device__ __forceinline__ void store4(float* dst, float a, float b, float c, float d) {
    *reinterpret_cast<float4*>(dst) = make_float4(a, b, c, d);
}
__device__ __forceinline__ void store4(bf16* dst, float a, float b, float c, float d) {
    bf16 v[4] = {__float2bfloat16(a), __float2bfloat16(b), __float2bfloat16(c), __float2bfloat16(d)};
    *reinterpret_cast<uint2*>(dst) = *reinterpret_cast<const uint2*>(v);
}

__device__ __forceinline__ int uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }
// The lane id recomputed from the exec mask (v_mbcnt) in place: an asm the compiler can neither hoist
// nor merge with an earlier lane id, so no register has to hold one across a long stretch of code (a
// value kept live there can be spilled to scratch, one more memory round trip to reload it).
__device__ __forceinline__ int fresh_lane() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}
__device__ __forceinline__ float readlane_f(float v, int lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

// "v if c else 0" without a branch: the mask goes through an empty asm, so the compiler cannot turn
// the AND back into a select and then into a branch around the load that produced v (it sinks such
// loads into conditional blocks, and the blocks serialise loads that should all be in flight).
__device__ __forceinline__ unsigned keep_mask(bool c) {
    unsigned m = c ? 0xFFFFFFFFu : 0u;
    asm("" : "+v"(m));
    return m;
}
__device__ __forceinline__ uint4 keep_if(bool c, uint4 v) {
    const unsigned m = keep_mask(c);
    return make_uint4(v.x & m, v.y & m, v.z & m, v.w & m);
}
__device__ __forceinline__ float keep_if(bool c, float v) { return __uint_as_float(__float_as_uint(v) & keep_mask(c)); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}
__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}
__device__ __forceinline__ int wave_min(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, kWave));
    return v;
}

// Cross-lane sums without the LDS crossbar (each __shfl_xor is a ds_bpermute: ~50 per pixel made the
// splat backward's reductions its longest phase): DPP quad / row permutes and gfx950's permlane16 /
// permlane32 swaps. Level O adds the same two operands as the xor butterfly's level O (v_l +
// v_{l^O}; fp32 addition commutes), so results are bit-identical to the butterfly -- in every lane for
// O = 1, 2, 8, 16, 32, and for O = 4 (row_shl:4: lane l reads l + 4 of its row) in the lanes with
// (l & 7) < 4 (scripts/probes/dpp_check.hip checks each primitive against the butterfly, lane by lane).
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
template <int O>
__device__ __forceinline__ float xsum(float v) {
    if constexpr (O == 1) {
        return v + dpp_f<0xB1>(v);  // quad_perm [1,0,3,2]
    } else if constexpr (O == 2) {
        return v + dpp_f<0x4E>(v);  // quad_perm [2,3,0,1]
    } else if constexpr (O == 4) {
        return v + dpp_f<0x104>(v);  // row_shl:4
    } else if constexpr (O == 8) {
        return v + dpp_f<0x128>(v);  // row_ror:8 (= l ^ 8 inside a row of 16)
    } else if constexpr (O == 16) {
        const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
        return __uint_as_float(p[0]) + __uint_as_float(p[1]);
    } else {
        static_assert(O == 32, "butterfly level");
        const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
        return __uint_as_float(p[0]) + __uint_as_float(p[1]);
    }
}
// sum over the lanes l ^ o, o = LO, 2 LO, ..., HI (exact as above)
template <int LO, int HI>
__device__ __forceinline__ float xsum_range(float v) {
    if constexpr (LO <= HI) return xsum_range<LO * 2, HI>(xsum<LO>(v));
    else return v;
}
// wave_sum's value (its butterfly levels in its order, 32 down to 1), exact in lane 0, broadcast
__device__ __forceinline__ float wave_sum_dpp(float v) {
    v = xsum<1>(xsum<2>(xsum<4>(xsum<8>(xsum<16>(xsum<32>(v))))));
    return readlane_f(v, 0);
}

#ifndef LSS_TRACE
#define LSS_TRACE 0  // diagnostics build: per-wave s_memrealtime stamps of the channels-last splat
#endif
#if LSS_TRACE
// [wave slot][0: start, 1: after round trip 1, 2: after the first gather batch, 3: end, 4: kind | hw id]
__device__ unsigned long long g_lss_trace[16384][5];
#define LSS_STAMP(slot, i)                                                                                     \
    do {                                                                                                       \
        const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                                        \
        if ((threadIdx.x & 63) == 0 && (slot) < 16384) g_lss_trace[(slot)][(i)] = t_;                          \
    } while (0)
#else
#define LSS_STAMP(slot, i) do { } while (0)
#endif

// Blocks are dealt round-robin over the 8 XCDs (observed placement: speed only, never correctness).
// xcd_block gives each XCD one contiguous run of ceil(nb / 8) logical blocks, so kernels that follow
// each other with the same mapping hand data over through the same XCD's L2: the lift writes a
// sample's context rows / depth weights, the CSR build its keys, the scan its cell starts, from the
// XCD whose splat blocks read them. The grid must be xcd_grid(nb) blocks; logical ids >= nb idle.
__device__ __forceinline__ int xcd_block() {
    return (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
}
inline int xcd_grid(long nb) { return (int)(8 * ((nb + 7) / 8)); }

// ---- LSS_DEBUG builds (liblss_hip_debug.so): every global index that comes from data (cell ids, CSR
// positions, point ids, context rows) is checked before it is used. A failed check records
// {count, code, value, bound} of the first failure in g_lss_dbg (read by lss_debug_status) and the
// index is replaced by 0, so the kernel reports instead of faulting. Release builds compile the checks
// away (dchk(i, n, code) is i).
#ifndef LSS_DEBUG
#define LSS_DEBUG 0
#endif
__device__ int g_lss_dbg[4];  // [failures, first code, first value, first bound]
__device__ __attribute__((noinline)) void lss_dbg_fail(int code, long long v, long long hi) {
    if (atomicAdd(&g_lss_dbg[0], 1) == 0) {
        g_lss_dbg[1] = code;
        g_lss_dbg[2] = (int)v;
        g_lss_dbg[3] = (int)hi;
    }
}
// i if 0 <= i < n; else record the failure and return 0
__device__ __forceinline__ int dchk(int i, long long n, int code) {
    if (LSS_DEBUG && (i < 0 || (long long)i >= n)) {
        lss_dbg_fail(code, i, n);
        return 0;
    }
    return i;
}
// a condition that must hold (records only)
__device__ __forceinline__ void dassert(bool ok, int code, long long v, long long hi) {
    if (LSS_DEBUG && !ok) lss_dbg_fail(code, v, hi);
}
// Check codes (lss_debug_status reports the first failure's code).
enum : int {
    kDbgScatterPos = 1,    // counting-sort scatter position outside [cell_start[cell], cell_start[cell + 1])
    kDbgCsrTotal = 2,      // cell_start[ncells] > nprime
    kDbgCsrMonotone = 3,   // cell_start decreasing
    kDbgCanonPos = 4,      // k_csr_canon write position outside [0, total)
    kDbgSplatPoint = 5,    // splat: point id outside [0, nprime)
    kDbgSplatRow = 6,      // splat: context row outside [0, rows)
    kDbgSplatCell = 7,     // splat: cell outside the tile / grid
    kDbgBwdRow = 8,        // backward: gradient row outside [0, rows)
    kDbgCell = 9,          // a cell id outside [-1, ncells)
    kDbgSegRun = 10,       // QuickCumsum operator: run index outside [0, nseg)
};

// acc = 0; for k: acc = acc + m[k] * v[k]   -- fp32, each op rounded (CPU torch.matmul order).
__device__ __forceinline__ float dot3_seq(float m0, float m1, float m2, float v0, float v1, float v2) {
    float acc = __fmul_rn(m0, v0);
    acc = __fadd_rn(acc, __fmul_rn(m1, v1));
    return __fadd_rn(acc, __fmul_rn(m2, v2));
}

// ----------------------------------------------------------------------------- geometry -> cells
__device__ __forceinline__ int quantize_cell(float ex, float ey, float ez, const lss_grid_t& g, int b) {
    // ((geom - (bx - dx/2)) / dx).long() + bounds filter (src/models.py:212-223).
    // trunc(v) in [0, n)  <=>  v > -1 && v < n   (NaN fails both).
    const float vx = __fdiv_rn(__fsub_rn(ex, g.lo[0]), g.dx[0]);
    const float vy = __fdiv_rn(__fsub_rn(ey, g.lo[1]), g.dx[1]);
    const float vz = __fdiv_rn(__fsub_rn(ez, g.lo[2]), g.dx[2]);
    const bool ok = vx > -1.0f && vx < (float)g.nx[0] && vy > -1.0f && vy < (float)g.nx[1] &&
                    vz > -1.0f && vz < (float)g.nx[2];
    if (!ok) return -1;
    const int ix = (int)vx, iy = (int)vy, iz = (int)vz;  // truncation toward zero
    return ((b * g.nx[2] + iz) * g.nx[0] + ix) * g.nx[1] + iy;
}

constexpr int kGeoBlock = 256;  // threads (points) per block of the geometry / cell kernels
constexpr int kGeoHashBits = kGeoBlock <= 256 ? 9 : kGeoBlock <= 512 ? 10 : 11;
constexpr int kGeoHash = 1 << kGeoHashBits;  // >= 2 entries per point of the block: short probe chains
static_assert(kGeoHash >= 2 * kGeoBlock, "hash table at most half full");

// The block's distinct cells: open-addressing table in LDS (key -1 = free; cnt = points, then base).
struct GeoHash {
    int key[kGeoHash];
    int cnt[kGeoHash];
};

// Slots grouped per block. Every kept point inserts its cell into the block's LDS table
// (multiplicative hash, linear probing) and takes a rank among the block's points of that cell from an
// LDS atomic; then ONE returning device atomic per distinct cell of the block adds the group's size to
// the count, and a point's slot is that old count plus its rank (arrival order; k_csr_canon fixes the
// order later). At c3 a block of 256 points holds 67 k distinct (block, cell) pairs in all against
// 141 k (wave, cell) pairs; at c5 171 k against 535 k -- and the device atomics, executed at the memory
// side, are what the kernel waits on (per-wave groups: 11.8 vs 7.3 us at c3, profiles/r02).
// Must be called by every thread of the block (cell = -1 for dropped / out-of-range points).
__device__ __forceinline__ void emit_cell_block(int p, int cell, int32_t* cell_of, int32_t* cell_count,
                                                int32_t* slot_of, bool live, GeoHash& h) {
    if (live) cell_of[p] = cell;
    if (cell_count == nullptr) return;  // block-uniform
    for (int i = threadIdx.x; i < kGeoHash; i += kGeoBlock) {
        h.key[i] = -1;
        h.cnt[i] = 0;
    }
    __syncthreads();
    const bool kept = live && cell >= 0;
    int at = 0, rank = 0;
    if (kept) {
        at = (int)(((unsigned)cell * 2654435761u) >> (32 - kGeoHashBits));
        for (;;) {
            const int prev = atomicCAS(&h.key[at], -1, cell);
            if (prev == -1 || prev == cell) break;
            at = (at + 1) & (kGeoHash - 1);
        }
        rank = atomicAdd(&h.cnt[at], 1);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kGeoHash; i += kGeoBlock) {
        const int c = h.key[i];
        if (c >= 0) h.cnt[i] = atomicAdd(cell_count + c, h.cnt[i]);
    }
    __syncthreads();
    if (live) slot_of[p] = kept ? h.cnt[at] + rank : -1;
}

// One frustum point through one camera (src/models.py:172-190), fp32, each op rounded in the
// reference's order.
__device__ __forceinline__ void geometry_point(const float* __restrict__ frustum, const float* __restrict__ rots,
                                               const float* __restrict__ trans, const float* __restrict__ kinv,
                                               const float* __restrict__ pinv, const float* __restrict__ post_trans,
                                               int cam, int f, float e[3]) {
    const float* P = pinv + 9 * cam;
    const float* K = kinv + 9 * cam;
    const float* R = rots + 9 * cam;
    // points = frustum - post_trans                         (src/models.py:179)
    const float x0 = __fsub_rn(frustum[3 * f + 0], post_trans[3 * cam + 0]);
    const float x1 = __fsub_rn(frustum[3 * f + 1], post_trans[3 * cam + 1]);
    const float x2 = __fsub_rn(frustum[3 * f + 2], post_trans[3 * cam + 2]);
    // points = inv(post_rots) @ points                      (src/models.py:180)
    const float q0 = dot3_seq(P[0], P[1], P[2], x0, x1, x2);
    const float q1 = dot3_seq(P[3], P[4], P[5], x0, x1, x2);
    const float q2 = dot3_seq(P[6], P[7], P[8], x0, x1, x2);
    // (x*z, y*z, z)                                         (src/models.py:183-185)
    const float r0 = __fmul_rn(q0, q2), r1 = __fmul_rn(q1, q2), r2 = q2;
    // combine = rots @ inv(intrins); points = combine @ points + trans   (src/models.py:186-188)
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float c0 = dot3_seq(R[3 * i + 0], R[3 * i + 1], R[3 * i + 2], K[0], K[3], K[6]);
        const float c1 = dot3_seq(R[3 * i + 0], R[3 * i + 1], R[3 * i + 2], K[1], K[4], K[7]);
        const float c2 = dot3_seq(R[3 * i + 0], R[3 * i + 1], R[3 * i + 2], K[2], K[5], K[8]);
        e[i] = __fadd_rn(dot3_seq(c0, c1, c2, r0, r1, r2), trans[3 * cam + i]);
    }
}

__global__ __launch_bounds__(kGeoBlock) void k_geometry_cells(
    const float* __restrict__ frustum, const float* __restrict__ rots, const float* __restrict__ trans,
    const float* __restrict__ kinv, const float* __restrict__ pinv, const float* __restrict__ post_trans,
    int N, int DHW, int nprime, lss_grid_t g, float* __restrict__ out_geom,
    int32_t* __restrict__ cell_of, int32_t* __restrict__ cell_count, int32_t* __restrict__ slot_of) {
    const int p0 = blockIdx.x * kGeoBlock + threadIdx.x;
    const bool live = p0 < nprime;
    const int p = live ? p0 : nprime - 1;  // dead lanes recompute the last point, then write nothing
    const int cam = p / DHW;
    const int f = p - cam * DHW;
    const int b = cam / N;
    float e[3];
    geometry_point(frustum, rots, trans, kinv, pinv, post_trans, cam, f, e);
    if (out_geom != nullptr && live) {
        out_geom[3 * (size_t)p + 0] = e[0];
        out_geom[3 * (size_t)p + 1] = e[1];
        out_geom[3 * (size_t)p + 2] = e[2];
    }
    const int cell = live ? quantize_cell(e[0], e[1], e[2], g, b) : -1;
    __shared__ GeoHash hash;
    emit_cell_block(p, cell, cell_of, cell_count, slot_of, live, hash);
}

__global__ __launch_bounds__(kGeoBlock) void k_cells_from_geom(const float* __restrict__ geom, int nprime, int ppb,
                                                               lss_grid_t g, int32_t* __restrict__ cell_of,
                                                               int32_t* __restrict__ cell_count,
                                                               int32_t* __restrict__ slot_of) {
    const int p0 = blockIdx.x * kGeoBlock + threadIdx.x;
    const bool live = p0 < nprime;
    const int p = live ? p0 : nprime - 1;  // dead lanes stay for the block barriers, write nothing
    const int cell =
        live ? quantize_cell(geom[3 * (size_t)p], geom[3 * (size_t)p + 1], geom[3 * (size_t)p + 2], g, p / ppb) : -1;
    __shared__ GeoHash hash;
    emit_cell_block(p, cell, cell_of, cell_count, slot_of, live, hash);
}

// ---- ordered plan (lss_geometry_cells_ordered + lss_csr_build_ordered, ABI 22): every kept point's
// position in the canonical CSR (ascending cell, then ascending point id) follows from the counts
// alone, so no sort pass (k_csr_canon) is needed after the scatter.
//   in the block: a point's rank among the block's points of its cell is the number of LOWER threads
//     with that cell -- one bit per thread in a 256-bit mask per hash slot (LDS), popcounts below;
//   across blocks: the one returning device atomic per distinct (block, cell) adds
//     (1 << kOrdCountBits) | n to the cell's word, and the entry index it returns (the high bits)
//     places the record (logical block, n) in the cell's list of kOrdList records (or, past them,
//     in an overflow area through a counter in the workspace header: never at c1-c5, at most 8
//     blocks share a cell at c5). The scatter then sums the counts of the cell's records from lower
//     blocks: that is the number of the cell's points with a lower point id in other blocks.
// Points of logical block lb are [256 lb, 256 lb + 256) (XCD-contiguous blocks, xcd_block), so block
// order is point order. Cell words: points in the low kOrdCountBits bits, records in the high bits.
constexpr int kOrdCountBits = 20;
constexpr int kOrdCountMask = (1 << kOrdCountBits) - 1;
constexpr int kOrdList = 8;                 // records per cell held in the cell's list
constexpr int kGeoWaves = kGeoBlock / kWave;
static_assert(kGeoBlock == 256, "records pack n (<= 256) into 9 bits");

struct GeoHashOrd {
    int key[kGeoHash];
    unsigned long long mask[kGeoHash][kGeoWaves];  // bit l of word w: thread 64 w + l holds this cell
};

__device__ __forceinline__ void emit_cell_block_ordered(int lb, int p, int cell, int32_t* __restrict__ cell_of,
                                                        int32_t* __restrict__ cell_word, int32_t* __restrict__ rank_of,
                                                        int32_t* __restrict__ list, int2* __restrict__ ovf,
                                                        unsigned* __restrict__ ovf_count, bool live,
                                                        GeoHashOrd& h) {
    if (live) cell_of[p] = cell;
    for (int i = threadIdx.x; i < kGeoHash; i += kGeoBlock) h.key[i] = -1;
    unsigned long long* m = &h.mask[0][0];
    for (int i = threadIdx.x; i < kGeoHash * kGeoWaves; i += kGeoBlock) m[i] = 0ull;
    __syncthreads();
    const bool kept = live && cell >= 0;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int at = 0;
    if (kept) {
        at = (int)(((unsigned)cell * 2654435761u) >> (32 - kGeoHashBits));
        for (;;) {
            const int prev = atomicCAS(&h.key[at], -1, cell);
            if (prev == -1 || prev == cell) break;
            at = (at + 1) & (kGeoHash - 1);
        }
        atomicOr(&h.mask[at][wave], 1ull << lane);
    }
    __syncthreads();
    int rank = 0;
    if (kept) {
#pragma unroll
        for (int w = 0; w < kGeoWaves; ++w) {
            const unsigned long long mw = h.mask[at][w];
            rank += w < wave ? __popcll(mw) : (w == wave ? __popcll(mw & ((1ull << lane) - 1ull)) : 0);
        }
    }
    for (int i = threadIdx.x; i < kGeoHash; i += kGeoBlock) {
        const int c = h.key[i];
        if (c >= 0) {
            int n = 0;
#pragma unroll
            for (int w = 0; w < kGeoWaves; ++w) n += __popcll(h.mask[i][w]);
            const int old = atomicAdd(cell_word + c, (1 << kOrdCountBits) | n);
            const int idx = (int)((unsigned)old >> kOrdCountBits);
            const int rec = (lb << 9) | n;
            if (idx < kOrdList) {
                list[(size_t)c * kOrdList + idx] = rec;
            } else {
                const unsigned o = atomicAdd(ovf_count, 1u);
                ovf[o] = make_int2(c, rec);
            }
        }
    }
    if (live) rank_of[p] = kept ? rank : -1;
}

__global__ __launch_bounds__(kGeoBlock) void k_geometry_cells_ord(
    const float* __restrict__ frustum, const float* __restrict__ rots, const float* __restrict__ trans,
    const float* __restrict__ kinv, const float* __restrict__ pinv, const float* __restrict__ post_trans,
    int N, int DHW, int nprime, lss_grid_t g, float* __restrict__ out_geom, int32_t* __restrict__ cell_of,
    int32_t* __restrict__ cell_word, int32_t* __restrict__ rank_of, int32_t* __restrict__ list,
    int2* __restrict__ ovf, unsigned* __restrict__ ovf_count) {
    const int lb = xcd_block();
    if (lb * kGeoBlock >= nprime) return;  // block-uniform (padding blocks of the XCD-contiguous grid)
    const int p0 = lb * kGeoBlock + threadIdx.x;
    const bool live = p0 < nprime;
    const int p = live ? p0 : nprime - 1;  // dead lanes recompute the last point, then write nothing
    const int cam = p / DHW;
    const int f = p - cam * DHW;
    const int b = cam / N;
    float e[3];
    geometry_point(frustum, rots, trans, kinv, pinv, post_trans, cam, f, e);
    if (out_geom != nullptr && live) {
        out_geom[3 * (size_t)p + 0] = e[0];
        out_geom[3 * (size_t)p + 1] = e[1];
        out_geom[3 * (size_t)p + 2] = e[2];
    }
    const int cell = live ? quantize_cell(e[0], e[1], e[2], g, b) : -1;
    __shared__ GeoHashOrd hash;
    emit_cell_block_ordered(lb, p, cell, cell_of, cell_word, rank_of, list, ovf, ovf_count, live, hash);
}

__global__ __launch_bounds__(kGeoBlock) void k_cells_from_geom_ord(const float* __restrict__ geom, int nprime, int ppb,
                                                                   lss_grid_t g, int32_t* __restrict__ cell_of,
                                                                   int32_t* __restrict__ cell_word,
                                                                   int32_t* __restrict__ rank_of,
                                                                   int32_t* __restrict__ list, int2* __restrict__ ovf,
                                                                   unsigned* __restrict__ ovf_count) {
    const int lb = xcd_block();
    if (lb * kGeoBlock >= nprime) return;
    const int p0 = lb * kGeoBlock + threadIdx.x;
    const bool live = p0 < nprime;
    const int p = live ? p0 : nprime - 1;
    const int cell =
        live ? quantize_cell(geom[3 * (size_t)p], geom[3 * (size_t)p + 1], geom[3 * (size_t)p + 2], g, p / ppb) : -1;
    __shared__ GeoHashOrd hash;
    emit_cell_block_ordered(lb, p, cell, cell_of, cell_word, rank_of, list, ovf, ovf_count, live, hash);
}

// ----------------------------------------------------------------------------- CSR (counting sort)
// Exclusive scan of 1024 thread totals inside a block; returns the thread's exclusive prefix.
// Inclusive scan over the 64 lanes on DPP (integer adds: exact in any order): the sum of the 4 lanes up
// to l in each row (row_shr 1, 2, 3), of 8 and 16 (row_shr 4 / 8 into the upper banks), then the
// rows' totals carried over by row_bcast 15 / 31 -- VALU only, where the __shfl_up form was six
// dependent ds_bpermute round trips through the LDS crossbar.
__device__ __forceinline__ int wave_incl_scan(int v) {
    int t = v + __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);  // row_shr:1
    t += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);         // row_shr:2
    t += __builtin_amdgcn_update_dpp(0, v, 0x113, 0xf, 0xf, false);         // row_shr:3
    t += __builtin_amdgcn_update_dpp(0, t, 0x114, 0xf, 0xe, false);         // row_shr:4, banks 1-3
    t += __builtin_amdgcn_update_dpp(0, t, 0x118, 0xf, 0xc, false);         // row_shr:8, banks 2-3
    t += __builtin_amdgcn_update_dpp(0, t, 0x142, 0xa, 0xf, false);         // row_bcast:15 into rows 1, 3
    t += __builtin_amdgcn_update_dpp(0, t, 0x143, 0xc, 0xf, false);         // row_bcast:31 into rows 2, 3
    return t;
}

__device__ int block_exclusive_scan_1024(int v, int* s_wave, int* total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int incl = wave_incl_scan(v);
    if (lane == 63) s_wave[wave] = incl;
    __syncthreads();
    if (wave == 0) {
        int w = lane < 16 ? s_wave[lane] : 0;
        const int wi = wave_incl_scan(w);  // (lanes 16.. add zeros)
        if (lane < 16) s_wave[16 + lane] = wi - w;
        if (lane == 15) *total = wi;
    }
    __syncthreads();
    return s_wave[16 + wave] + incl - v;
}

__global__ __launch_bounds__(1024) void k_scan_partials(const int32_t* __restrict__ cnt, int ncells,
                                                        int32_t* __restrict__ partial) {
    __shared__ int s_wave[32];
    __shared__ int s_total;
    const int base = blockIdx.x * kScanItems + threadIdx.x * 4;
    int v = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) v += (base + i < ncells) ? cnt[base + i] : 0;
    block_exclusive_scan_1024(v, s_wave, &s_total);
    if (threadIdx.x == 0) partial[blockIdx.x] = s_total;
}

__global__ __launch_bounds__(1024) void k_scan_apply(const int32_t* __restrict__ cnt, int ncells,
                                                     const int32_t* __restrict__ partial,
                                                     int32_t* __restrict__ cell_start) {
    __shared__ int s_wave[32];
    __shared__ int s_total;
    __shared__ int s_red[16];
    const int lb = xcd_block();
    const int nb = (ncells + kScanItems - 1) / kScanItems;
    if (lb >= nb) return;  // block-uniform
    // prefix = sum of the preceding blocks' totals
    int pre = 0;
    for (int i = threadIdx.x; i < lb; i += 1024) pre += partial[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) pre += __shfl_xor(pre, o, kWave);
    if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = pre;
    __syncthreads();
    int prefix = 0;
#pragma unroll
    for (int w = 0; w < 16; ++w) prefix += s_red[w];
    const int base = lb * kScanItems + threadIdx.x * 4;
    int c[4];
    int v = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        c[i] = (base + i < ncells) ? cnt[base + i] : 0;
        v += c[i];
    }
    int run = prefix + block_exclusive_scan_1024(v, s_wave, &s_total);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (base + i < ncells) cell_start[base + i] = run;
        run += c[i];
    }
    if (lb == nb - 1 && threadIdx.x == 0) cell_start[ncells] = prefix + s_total;
}

// Position of a kept point's key in the counting sort: cell_start[cell] + slot (checked in LSS_DEBUG
// builds: inside the cell's range, and that range inside the nprime-entry buffer).
__device__ __forceinline__ int scatter_pos(int cell, int slot, const int32_t* __restrict__ cell_start, int nprime) {
    const int a = cell_start[cell];
    if (LSS_DEBUG) {
        const int b = cell_start[cell + 1];
        dassert(a <= b && b <= nprime, kDbgCsrTotal, b, nprime);
        dassert(slot >= 0 && a + slot < b, kDbgScatterPos, slot, b - a);
        return dchk(a + slot, nprime, kDbgScatterPos);
    }
    return a + slot;
}

// Counting-sort scatter: point p lands at cell_start[cell] + slot as the key (cell << 32) | p
// (slot order inside a cell is the atomics' arrival order; k_csr_canon fixes it).
__global__ __launch_bounds__(kBlock) void k_scatter(const int32_t* __restrict__ cell_of,
                                                    const int32_t* __restrict__ slot_of, int nprime,
                                                    const int32_t* __restrict__ cell_start,
                                                    long long* __restrict__ key_out) {
    const int p = blockIdx.x * kBlock + threadIdx.x;
    if (p >= nprime) return;
    const int cell = cell_of[p];
    if (cell >= 0) key_out[scatter_pos(cell, slot_of[p], cell_start, nprime)] = ((long long)cell << 32) | (unsigned)p;
}

// ---- single-pass scan (lss_csr_build_ws): one launch in place of k_scan_partials + k_scan_apply.
// Block k (blockIdx; workgroups are dispatched in index order, so it only waits for blocks already
// dispatched -- no residency assumption) publishes its aggregate, then wave 0 looks back over its
// predecessors' 8-byte {status, value} granules, 128 at a time,
// up to the nearest inclusive prefix, and publishes its own inclusive prefix. Granules are written
// with agent-scope (sc1, write-through) atomic stores and polled with agent-scope atomic loads --
// the cross-XCD hand-off form of the R2 recipe (cdna_hip_programming.md, Guideline 16). Spins are
// bounded: after kScanSpinLimit polls a block stops waiting and computes the aggregate of every
// predecessor that has not published yet straight from its cell counts (intact until the scatter
// after the scan re-zeroes them), then keeps looking back -- the prefix is exact either way, a
// timeout only costs time; the sticky timeout word counts them. The scatter re-zeroes the ticket and
// the granules after the scan, so every call starts from zeros.
constexpr unsigned kScanSpinLimit = 1u << 22;
struct ScanWs {  // lss_csr_workspace_bytes: [ovf_count, timeouts, spin_limit_override, pad][granule x nb]
    unsigned ovf_count;  // ordered plans: records past a cell's list (reset by k_scatter_ord)
    unsigned timeouts;
    unsigned spin_override;  // 0: kScanSpinLimit polls; s > 0: s - 1 polls (tests of the timeout path)
    unsigned pad;
};


// Look-back granules still 0 (their block has not published): replaced by the block's aggregate
// {status 1, sum of its kScanItems counts}, summed by the whole wave from `cnt`. jb = the block each
// lane polled (>= 0 wherever x == 0).
__device__ unsigned long long scan_fill_missing(unsigned long long x, int jb, const int32_t* __restrict__ cnt,
                                                int ncells, int lane, int cmask) {
    unsigned long long miss = __ballot(x == 0ull);
    while (miss) {
        const int l = __builtin_ctzll(miss);
        miss &= miss - 1;
        const int blk = __builtin_amdgcn_readlane(jb, l);
        const int lo = blk * kScanItems, hi = min(lo + kScanItems, ncells);
        int s = 0;
        for (int i = lo + lane; i < hi; i += kWave) s += cnt[i] & cmask;
        s = wave_sum_i(s);
        if (lane == l) x = (1ull << 32) | (unsigned)s;
    }
    return x;
}
__device__ __forceinline__ unsigned long long ld_agent(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(unsigned long long* p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// cmask: the count bits of a cell word (-1: plain counts; kOrdCountMask: ordered-plan words)
__global__ __launch_bounds__(1024) void k_scan_lookback(const int32_t* __restrict__ cnt, int ncells,
                                                        ScanWs* __restrict__ ws, int32_t* __restrict__ cell_start,
                                                        int cmask) {
    __shared__ int s_wave[32];
    __shared__ int s_total;
    __shared__ int s_prefix;
    unsigned long long* gran = reinterpret_cast<unsigned long long*>(ws + 1);
    // Logical index = blockIdx: workgroups of a launch are dispatched in index order, so block k only
    // waits for blocks that were dispatched before it (at worst delayed while another kernel holds
    // their XCD's CUs).
    const int lb = blockIdx.x;
    const int nb = (ncells + kScanItems - 1) / kScanItems;
    const int base = lb * kScanItems + threadIdx.x * 4;
    // 16-byte count loads / cell_start stores when both arrays allow it (uniform over the launch)
    const bool vec = ((reinterpret_cast<uintptr_t>(cnt) | reinterpret_cast<uintptr_t>(cell_start)) & 15) == 0;
    int4 c4 = make_int4(0, 0, 0, 0);
    if (vec && base + 4 <= ncells) {
        c4 = *reinterpret_cast<const int4*>(cnt + base);
    } else if (base < ncells) {
        c4.x = cnt[base];
        if (base + 1 < ncells) c4.y = cnt[base + 1];
        if (base + 2 < ncells) c4.z = cnt[base + 2];
        if (base + 3 < ncells) c4.w = cnt[base + 3];
    }
    c4.x &= cmask;
    c4.y &= cmask;
    c4.z &= cmask;
    c4.w &= cmask;
    const int excl = block_exclusive_scan_1024(c4.x + c4.y + c4.z + c4.w, s_wave, &s_total);
    if (threadIdx.x < kWave) {
        const int lane = threadIdx.x;
        const int agg = s_total;
        int prefix = 0;
        if (lb == 0) {
            if (lane == 0) st_agent(&gran[0], (2ull << 32) | (unsigned)agg);
        } else {
            if (lane == 0) st_agent(&gran[lb], (1ull << 32) | (unsigned)agg);
            const unsigned so = ws->spin_override;
            const unsigned limit = so ? so - 1u : kScanSpinLimit;
            bool gave_up = false;
            // 128 predecessors per poll (two granules a lane: distances lane + 1 and lane + 65)
            for (int j = lb - 1;; j -= 2 * kWave) {
                const int j0 = j - lane, j1 = j0 - kWave;  // past block 0: an inclusive prefix of 0
                unsigned long long x0 = 2ull << 32, x1 = 2ull << 32;
                for (unsigned spins = 0;; ++spins) {
                    x0 = j0 >= 0 ? ld_agent(&gran[j0]) : (2ull << 32);
                    x1 = j1 >= 0 ? ld_agent(&gran[j1]) : (2ull << 32);
                    if (__all(x0 != 0ull && x1 != 0ull)) break;
                    if (gave_up || spins >= limit) {
                        // stop waiting: the unpublished predecessors' aggregates from their counts
                        if (!gave_up && lane == 0) atomicAdd(&ws->timeouts, 1u);
                        gave_up = true;
                        x0 = scan_fill_missing(x0, j0, cnt, ncells, lane, cmask);
                        x1 = scan_fill_missing(x1, j1, cnt, ncells, lane, cmask);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                const unsigned long long pm0 = __ballot((x0 >> 32) == 2ull);
                const unsigned long long pm1 = __ballot((x1 >> 32) == 2ull);
                // nearest inclusive prefix: in the first 64, else in the second 64, else keep going
                const int upto0 = pm0 ? __builtin_ctzll(pm0) : kWave - 1;
                const int upto1 = pm0 ? -1 : (pm1 ? __builtin_ctzll(pm1) : kWave - 1);
                int val = (lane <= upto0 ? (int)(unsigned)x0 : 0) + (lane <= upto1 ? (int)(unsigned)x1 : 0);
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) val += __shfl_xor(val, o, kWave);
                prefix += val;
                if (pm0 | pm1) break;
            }
            if (lane == 0) st_agent(&gran[lb], (2ull << 32) | (unsigned)(prefix + agg));
        }
        if (lane == 0) s_prefix = prefix;
    }
    __syncthreads();
    const int r0 = s_prefix + excl;
    const int4 o4 = make_int4(r0, r0 + c4.x, r0 + c4.x + c4.y, r0 + c4.x + c4.y + c4.z);
    if (vec && base + 4 <= ncells) {
        *reinterpret_cast<int4*>(cell_start + base) = o4;
    } else if (base < ncells) {
        cell_start[base] = o4.x;
        if (base + 1 < ncells) cell_start[base + 1] = o4.y;
        if (base + 2 < ncells) cell_start[base + 2] = o4.z;
        if (base + 3 < ncells) cell_start[base + 3] = o4.w;
    }
    if (lb == nb - 1 && threadIdx.x == 0) cell_start[ncells] = s_prefix + s_total;
}

// k_scatter plus the reset for the next call: the scan's granules and the cell counts (nothing reads
// them after the scan). The grid covers max(nprime, ncells) threads.
__global__ __launch_bounds__(kBlock) void k_scatter_ws(const int32_t* __restrict__ cell_of,
                                                       const int32_t* __restrict__ slot_of, int nprime,
                                                       const int32_t* __restrict__ cell_start,
                                                       long long* __restrict__ key_out, int32_t* __restrict__ cnt,
                                                       int ncells, ScanWs* __restrict__ ws) {
    const int t = blockIdx.x * kBlock + threadIdx.x;
    if (t < nprime) {
        const int cell = cell_of[t];
        if (cell >= 0) key_out[scatter_pos(cell, slot_of[t], cell_start, nprime)] = ((long long)cell << 32) | (unsigned)t;
    }
    if (t < ncells) cnt[t] = 0;
    const int nb = (ncells + kScanItems - 1) / kScanItems;
    if (t < nb) reinterpret_cast<unsigned long long*>(ws + 1)[t] = 0ull;
}

__device__ __forceinline__ int point_row(int p, int DHW, int HW) {
    const int cam = p / DHW;
    return cam * HW + (p - cam * DHW) % HW;  // pixel of point p = its context row
}

// Ordered scatter (lss_csr_build_ordered): point p of cell c goes straight to its canonical position
// cell_start[c] + (the cell's points in lower blocks, summed from the cell's records) + (its rank in
// its block), with its key and context row; entries [total, nprime) get the sentinel key. Then the
// reset for the next plan: the cell words, the scan's granules and the overflow counter (nothing in
// this launch reads them). Points are taken in XCD-contiguous blocks (xcd_block), as the geometry and
// the splat's chunk waves take them, so each sample's CSR entries are written from the XCD that reads
// them. The grid covers max(nprime, ncells) threads.
__device__ __forceinline__ void ord_rec(int rec, int n_c, int myblk, int& seen, int& before) {
    if (seen < n_c) {
        const int n = rec & 511;
        seen += n;
        before += (rec >> 9) < myblk ? n : 0;
    }
}

__global__ __launch_bounds__(kBlock) void k_scatter_ord(const int32_t* __restrict__ cell_of,
                                                        const int32_t* __restrict__ rank_of, int nprime,
                                                        const int32_t* __restrict__ cell_start,
                                                        const int32_t* __restrict__ list,
                                                        const int2* __restrict__ ovf, int DHW, int HW,
                                                        long long* __restrict__ key_out, int32_t* __restrict__ row_out,
                                                        int32_t* __restrict__ cell_word, int ncells,
                                                        ScanWs* __restrict__ ws) {
    static_assert(kBlock == kGeoBlock, "one scatter block = one geometry block of points");
    const int t = xcd_block() * kBlock + threadIdx.x;
    if (t < nprime) {
        const int total = min(cell_start[ncells], nprime);
        const int cell = cell_of[t];
        const int r = rank_of[t];
        if (cell >= 0) {
            const int c = dchk(cell, ncells, kDbgCell);
            const int a = cell_start[c], z = cell_start[c + 1];
            const int4 l0 = *reinterpret_cast<const int4*>(list + (size_t)c * kOrdList);
            const int n_c = z - a;
            const int myblk = t / kGeoBlock;
            int seen = 0, before = 0;
            ord_rec(l0.x, n_c, myblk, seen, before);
            ord_rec(l0.y, n_c, myblk, seen, before);
            ord_rec(l0.z, n_c, myblk, seen, before);
            ord_rec(l0.w, n_c, myblk, seen, before);
            if (seen < n_c) {  // more than 4 blocks share the cell (none at c1-c4, ~1 % of c5's occupied cells)
                const int4 l1 = *reinterpret_cast<const int4*>(list + (size_t)c * kOrdList + 4);
                ord_rec(l1.x, n_c, myblk, seen, before);
                ord_rec(l1.y, n_c, myblk, seen, before);
                ord_rec(l1.z, n_c, myblk, seen, before);
                ord_rec(l1.w, n_c, myblk, seen, before);
            }
            // more than kOrdList blocks share the cell: its other records, in the overflow area's valid
            // prefix (the counter restarts at 0 every plan; the records of this cell end before the
            // cell's points are all accounted for, so nothing past that prefix is read)
            for (int o = 0; seen < n_c && o < nprime; ++o) {
                const int2 v = ovf[o];
                if (v.x == c) ord_rec(v.y, n_c, myblk, seen, before);
            }
            dassert(seen == n_c, kDbgScatterPos, seen, n_c);
            const int at = dchk(a + before + r, total, kDbgScatterPos);
            dassert(before + r < n_c, kDbgScatterPos, before + r, n_c);
            key_out[at] = ((long long)cell << 32) | (unsigned)t;
            row_out[at] = point_row(t, DHW, HW);
        }
        if (t >= total) key_out[t] = -1ll;  // sentinel tail
    }
    const int g = blockIdx.x * kBlock + threadIdx.x;  // the reset, in launch order
    if (g < ncells) cell_word[g] = 0;
    const int nb = (ncells + kScanItems - 1) / kScanItems;
    if (g < nb) reinterpret_cast<unsigned long long*>(ws + 1)[g] = 0ull;
    if (g == 0) ws->ovf_count = 0u;
}

// The sorted list is cut into 64-entry chunks; the wave of chunk w owns the cells that START
// in [64w, 64w + 64). It reads entries [64w - 1, 64w + 128): the owned cells (<= 64 entries each;
// a longer last cell is flagged `big`) and the entry before the chunk (a cell that started earlier).
struct ChunkCells {
    int s, end;           // owned entries [s, end) held in the two registers (end <= base + 128)
    int big_start;        // start of an owned cell that runs past base + 127, or -1
};

__device__ __forceinline__ ChunkCells chunk_cells(int base, int total, int c0, int c1, int prevcell, int lane,
                                                  int ch = kWave) {
    // ch <= 64: the chunk is [base, base + ch) (cells of <= 64 entries starting there end below base + 128)
    ChunkCells r{0, 0, -1};
    const int up = __shfl(c0, (lane + 63) & 63, kWave);
    const int before = lane == 0 ? prevcell : up;
    const unsigned long long sm = __ballot(lane < ch && base + lane < total && c0 != before);
    if (!sm) {
        r.s = r.end = base;
        return r;
    }
    const int first = __builtin_ctzll(sm), last = 63 - __builtin_clzll(sm);
    const int lastcell = __builtin_amdgcn_readlane(c0, last);
    r.s = base + first;
    const unsigned long long m0 = __ballot(lane > last && c0 != lastcell);  // c = -1 past the total
    if (m0) {
        r.end = base + __builtin_ctzll(m0);
        return r;
    }
    const unsigned long long m1 = __ballot(c1 != lastcell);
    if (m1) {
        r.end = base + 64 + __builtin_ctzll(m1);
        return r;
    }
    r.end = base + last;  // the last owned cell has more than 64 entries
    r.big_start = base + last;
    return r;
}

__device__ __forceinline__ int pick(int r0, int r1, int idx) {  // idx uniform, 0..127
    return idx < kWave ? __builtin_amdgcn_readlane(r0, idx) : __builtin_amdgcn_readlane(r1, idx - kWave);
}


// Canonical CSR order: inside every cell the entries are sorted by point id (so every later
// reduction over a cell is deterministic without sorting again), and each entry's context-row
// index (its pixel) is stored beside it. One wave per 64-entry chunk, cells owned as above.
__global__ __launch_bounds__(kBlock) void k_csr_canon(const long long* __restrict__ key_in,
                                                      const int32_t* __restrict__ total_ptr, int nchunks, int nprime,
                                                      int DHW,
                                                      int HW, long long* __restrict__ key_out,
                                                      int32_t* __restrict__ row_out) {
    const int lane = threadIdx.x & 63;
    const int w = xcd_block() * (kBlock / kWave) + uniform(threadIdx.x >> 6);
    if (w >= nchunks) return;
    const int base = w * kWave;
    const int e0 = base + lane, e1 = base + kWave + lane;
    // the entry count and the window's keys in ONE round trip: the keys are read unconditionally
    // (clamped into the nprime-entry buffer) and masked with the count afterwards
    const int total_in = *total_ptr;
    if (LSS_DEBUG && w == 0 && lane == 0) dassert(total_in >= 0 && total_in <= nprime, kDbgCsrTotal, total_in, nprime);
    const int total = min(total_in, nprime);  // (== total_in for any consistent count)
    const long long k0r = key_in[min(e0, nprime - 1)];
    const long long k1r = key_in[min(e1, nprime - 1)];
    int prev_at = max(base - 1, 0);
    asm("" : "+v"(prev_at));  // a vector load issued with the others, not a scalar one sunk past the stores
    const long long kpr = key_in[prev_at];
    // sentinel tail: entries [total, nprime) hold key -1 (cell -1), so a reader needs no entry count
    if (e0 >= total && e0 < nprime) key_out[e0] = -1ll;
    if (base >= total) return;
    const long long k0 = e0 < total ? k0r : -1ll;
    const long long k1 = e1 < total ? k1r : -1ll;
    const int prevcell = base > 0 ? (int)(kpr >> 32) : -2;
    const int c0 = (int)(k0 >> 32), c1 = (int)(k1 >> 32);
    const int p0 = (int)(k0 & 0xFFFFFFFF), p1 = (int)(k1 & 0xFFFFFFFF);
    const ChunkCells cc = chunk_cells(base, total, c0, c1, prevcell, lane);
    // start (global entry index) of the cell of each held entry
    // (cross-lane reads hoisted out of the lane-0 select: a permute from a lane that is switched
    // off returns 0)
    const int up0 = __shfl(c0, (lane + 63) & 63, kWave), up1 = __shfl(c1, (lane + 63) & 63, kWave);
    const int c0_last = __builtin_amdgcn_readlane(c0, 63);
    const unsigned long long st0 = __ballot(c0 != (lane == 0 ? prevcell : up0));
    const unsigned long long st1 = __ballot(c1 != (lane == 0 ? c0_last : up1));
    const unsigned long long le = ~0ull >> (63 - lane);
    const int cs0 = base + 63 - __builtin_clzll((st0 & le) | 1ull);  // bit 0 guard: owned entries have a start
    const int cs1 = (st1 & le) ? base + kWave + 63 - __builtin_clzll(st1 & le)
                               : base + 63 - __builtin_clzll(st0 | 1ull);
    // rank inside the cell from the window's point ids staged in LDS: each lane scans only its own
    // cell's run [cell start, next start) -- at most 64 entries, 8.5 on average at c3
    int r0 = 0, r1 = 0;
    __shared__ int s_pid[kBlock / kWave][2 * kWave];
    int* sp = s_pid[threadIdx.x >> 6];
    sp[lane] = p0;
    sp[kWave + lane] = p1;
    __builtin_amdgcn_wave_barrier();
    const int lim = cc.end - base;
    const unsigned long long after = lane == 63 ? 0ull : (~0ull << (lane + 1));
    const unsigned long long n0 = st0 & after, n1 = st1 & after;
    const int ce0 = min(n0 ? (int)__builtin_ctzll(n0) : (st1 ? kWave + (int)__builtin_ctzll(st1) : 2 * kWave), lim);
    const int ce1 = min(n1 ? kWave + (int)__builtin_ctzll(n1) : 2 * kWave, lim);
    if (e0 >= cc.s && e0 < cc.end)
        for (int j = cs0 - base; j < ce0; ++j) r0 += sp[j] < p0 ? 1 : 0;
    if (e1 >= cc.s && e1 < cc.end)
        for (int j = cs1 - base; j < ce1; ++j) r1 += sp[j] < p1 ? 1 : 0;
    if (e0 >= cc.s && e0 < cc.end) {
        const int at = dchk(cs0 + r0, total, kDbgCanonPos);
        key_out[at] = k0;
        row_out[at] = point_row(dchk(p0, nprime, kDbgSplatPoint), DHW, HW);
    }
    if (e1 >= cc.s && e1 < cc.end) {
        const int at = dchk(cs1 + r1, total, kDbgCanonPos);
        key_out[at] = k1;
        row_out[at] = point_row(dchk(p1, nprime, kDbgSplatPoint), DHW, HW);
    }
    if (cc.big_start >= 0) {
        // one cell with more than 64 entries: ordered selection straight from memory (rare)
        const int cell = (int)(key_in[cc.big_start] >> 32);
        int n = 0;
        while (cc.big_start + n < total && (int)(key_in[cc.big_start + n] >> 32) == cell) ++n;
        int last = -1;
        for (int k = 0; k < n; ++k) {
            int best = INT_MAX;
            for (int i = lane; i < n; i += kWave) {
                const int v = (int)(key_in[cc.big_start + i] & 0xFFFFFFFF);
                if (v > last && v < best) best = v;
            }
            best = uniform(wave_min(best));
            if (lane == 0) {
                key_out[cc.big_start + k] = ((long long)cell << 32) | (unsigned)best;
                row_out[cc.big_start + k] = point_row(best, DHW, HW);
            }
            last = best;
        }
    }
}

// LSS_DEBUG builds: the finished CSR -- cell_start non-decreasing from 0 with cell_start[ncells] <=
// nprime, every cell id in [-1, ncells) -- checked after every build.
__global__ __launch_bounds__(kBlock) void k_debug_csr(const int32_t* __restrict__ cell_start, int ncells,
                                                      const int32_t* __restrict__ cell_of, int nprime) {
    const int t = blockIdx.x * kBlock + threadIdx.x;
    if (t == 0) dassert(cell_start[0] == 0, kDbgCsrMonotone, cell_start[0], 0);
    if (t < ncells) dassert(cell_start[t] <= cell_start[t + 1], kDbgCsrMonotone, t, ncells);
    if (t == ncells) dassert(cell_start[t] <= nprime, kDbgCsrTotal, cell_start[t], nprime);
    if (t < nprime) dassert(cell_of[t] >= -1 && cell_of[t] < ncells, kDbgCell, cell_of[t], ncells);
}

// ----------------------------------------------------------------------------- BEV rows (channels-last)
struct BevGeo {
    int X, Y, Z;
    int ncells;
    int nrows;              // feature rows (LSS_DEBUG bound of the gathered row index)
};

// Element offset of cell k's row in the channels-last (B, X, Y, Z*C) BEV:
// cell ((b*Z + z)*X + x)*Y + y -> ((b*X + x)*Y + y)*Z*C + z*C
__device__ __forceinline__ size_t cell_row_offset(int cell, const BevGeo& g) {
    if (g.Z == 1) return (size_t)cell * kC;  // rows of consecutive cells are contiguous
    const int XY = g.X * g.Y;
    const int bz = cell / XY, xy = cell - bz * XY;
    const int b = bz / g.Z, z = bz - b * g.Z;
    return (((size_t)b * XY + xy) * g.Z + z) * kC;
}
template <typename OutT>
__device__ __forceinline__ OutT* cell_row(OutT* out, int cell, const BevGeo& g) {
    return out + cell_row_offset(cell, g);
}

// ----------------------------------------------------------------------------- lift prep
// One block = 64 consecutive pixels x 4 waves. Wave w owns depth bins d = w, w+4, ... and
// context channels 16w..16w+15 of every pixel, so all of a thread's loads are issued back to
// back (one memory round trip). depth = softmax_D(logits) is written in the reference's
// (B*N, D, H, W) layout (coalesced over pixels); the context is transposed through LDS to
// pixel-major rows ctx_t[q*64 + c] (coalesced 256-B rows).
template <typename InT, typename CT, int NI>  // NI = depth bins per wave part: D <= 4 * NI
__global__ __launch_bounds__(kBlock) void k_lift_prep(const InT* __restrict__ dn, int D, int HW, int npix,
                                                      float* __restrict__ depth, CT* __restrict__ ctx_t) {
    __shared__ float s_ctx[kC][65];
    __shared__ float s_red[2][4][64];
    const int q0 = xcd_block() * 64;  // XCD x: one contiguous run of pixel tiles (the splat's CSR order)
    if (q0 >= npix) return;  // block-uniform
    const int px = threadIdx.x & 63, part = threadIdx.x >> 6;
    const int q = q0 + px;
    const bool live = q < npix;
    // clamped, unconditional loads (no branch between them, so all are in flight at once); a dead
    // lane's values feed nothing that is written
    const int qc = min(q, npix - 1);
    const int bn = qc / HW, hw = qc - bn * HW;
    const InT* src = dn + (size_t)bn * (D + kC) * HW + hw;
    float cv[16], l[NI];
#pragma unroll
    for (int i = 0; i < 16; ++i) cv[i] = to_f32(src[(size_t)(D + part * 16 + i) * HW]);
#pragma unroll
    for (int i = 0; i < NI; ++i) l[i] = to_f32(src[(size_t)min(part + 4 * i, D - 1) * HW]);
    float m = -INFINITY;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        if (part + 4 * i >= D) l[i] = -INFINITY;
        m = fmaxf(m, l[i]);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) s_ctx[part * 16 + i][px] = cv[i];
    s_red[0][part][px] = m;
    __syncthreads();
    m = fmaxf(fmaxf(s_red[0][0][px], s_red[0][1][px]), fmaxf(s_red[0][2][px], s_red[0][3][px]));
    float e[NI], sum = 0.f;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        e[i] = (part + 4 * i < D) ? expf(l[i] - m) : 0.f;
        sum += e[i];
    }
    s_red[1][part][px] = sum;
    __syncthreads();
    sum = (s_red[1][0][px] + s_red[1][1][px]) + (s_red[1][2][px] + s_red[1][3][px]);
    if (live) {
        float* dst = depth + (size_t)bn * D * HW + hw;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int d = part + 4 * i;
            if (d < D) dst[(size_t)d * HW] = e[i] / sum;
        }
    }
    for (int i = threadIdx.x; i < 64 * kC; i += kBlock) {
        const int r = i >> 6, c = i & 63;
        if (q0 + r < npix) ctx_t[(size_t)(q0 + r) * kC + c] = from_f32<CT>(s_ctx[c][r]);
    }
}

// ----------------------------------------------------------------------------- depthnet + lift prep (fused)
// General shapes (any K <= 512 with K % 16 == 0, any H*W; k_depthnet_lift2 / 3 take up1's K = 512).
// CamEncode's depthnet 1x1 conv (K -> D + C channels, with bias) fused with the lift's first half
// (src/models.py:47, 55-59): logits = W.x + b on MFMA (v_mfma_f32_32x32x16_bf16: bf16 in, fp32
// accumulate), rounded to bf16 as the autocast conv's output is, then depth = softmax over the D
// bins (fp32, the reference's (B*N, D, H, W) layout) and the context rows ctx_t (bf16,
// pixel-major) -- the depthnet output itself is never written. One block = 32 pixels x 4 waves:
// the pixels' K input channels are staged in LDS as [pixel][k] (one 16-B LDS read per MFMA B
// fragment); wave w computes output channels [32w, 32w + 32) over all of K with A fragments (16 B
// of a weight row) read straight from L2.
constexpr int kDnPix = 32;    // pixels per block
constexpr int kDnMaxK = 512;  // input channels (up1 outputs 512, src/models.py:45)
constexpr int kDnMaxO = 128;  // D + C <= 4 waves x 32 output channels

__global__ __launch_bounds__(kBlock) void k_depthnet_lift(const bf16* __restrict__ feat, const bf16* __restrict__ weight,
                                                          const bf16* __restrict__ bias, int K, int D, int HW,
                                                          int npix, float* __restrict__ depth, bf16* __restrict__ ctx_t) {
    using bf16x8 = __attribute__((ext_vector_type(8))) short;
    using f32x16 = __attribute__((ext_vector_type(16))) float;
    __shared__ __attribute__((aligned(16))) bf16 s_x[kDnPix][kDnMaxK + 8];  // [pixel][k]; +8: spread the banks
    __shared__ float s_lg[kDnMaxO][kDnPix + 1];                               // bf16-rounded logits [o][pixel]
    __shared__ float s_red[2][kBlock / kDnPix][kDnPix];
    const int q0 = xcd_block() * kDnPix;
    if (q0 >= npix) return;  // block-uniform
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // stage: element (k, p), pixels fastest. With HW % 8 == 0 an aligned run of 8 pixels never
    // crosses an image, so each thread moves 16 B (8 pixels of one channel) per load.
    if ((HW & 7) == 0) {
        // every load of the thread first (one memory round trip), then the LDS writes
        constexpr int kIt = kDnMaxK * (kDnPix / 8) / kBlock;
        uint4 v[kIt];
#pragma unroll
        for (int t = 0; t < kIt; ++t) {
            const int i = threadIdx.x + t * kBlock;
            const int k = i / (kDnPix / 8), p8 = (i - k * (kDnPix / 8)) * 8, q = q0 + p8;
            v[t] = make_uint4(0u, 0u, 0u, 0u);
            if (k < K && q < npix) {
                const int bn = q / HW, hw = q - bn * HW;
                v[t] = *reinterpret_cast<const uint4*>(feat + ((size_t)bn * K + k) * HW + hw);
            }
        }
#pragma unroll
        for (int t = 0; t < kIt; ++t) {
            const int i = threadIdx.x + t * kBlock;
            const int k = i / (kDnPix / 8), p8 = (i - k * (kDnPix / 8)) * 8;
            if (k < K) {
                const unsigned short* e = reinterpret_cast<const unsigned short*>(&v[t]);
#pragma unroll
                for (int j = 0; j < 8; ++j) reinterpret_cast<unsigned short*>(&s_x[p8 + j][0])[k] = e[j];
            }
        }
    } else {
        for (int i = threadIdx.x; i < K * kDnPix; i += kBlock) {
            const int k = i / kDnPix, p = i - k * kDnPix, q = q0 + p;
            bf16 v = __float2bfloat16(0.f);
            if (q < npix) {
                const int bn = q / HW, hw = q - bn * HW;
                v = feat[((size_t)bn * K + k) * HW + hw];
            }
            s_x[p][k] = v;
        }
    }
    __syncthreads();
    const int O = D + kC;
    const int r = lane & 31, h = lane >> 5;
    const int o = wave * 32 + r;
    const bf16* wrow = weight + (size_t)min(o, O - 1) * K + 8 * h;
    float bv[16];  // bias of the lane's 16 output rows, loaded ahead (not one round trip per row later)
#pragma unroll
    for (int i = 0; i < 16; ++i) bv[i] = __bfloat162float(bias[min(wave * 32 + (i & 3) + 8 * (i >> 2) + 4 * h, O - 1)]);
    f32x16 acc = {};
    // four weight fragments (L2 reads) in flight ahead of their MFMAs
    for (int k0 = 0; k0 < K; k0 += 64) {
        bf16x8 a[4], b[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int kk = min(k0 + 16 * u, K - 16);  // K % 16 == 0; a clamped step is skipped below
            a[u] = *reinterpret_cast<const bf16x8*>(wrow + kk);
            if (o >= O) a[u] = bf16x8{};
            b[u] = *reinterpret_cast<const bf16x8*>(&s_x[r][kk + 8 * h]);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (k0 + 16 * u < K) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[u], b[u], acc, 0, 0, 0);
    }
    // D/C layout: column (pixel) = lane & 31, row (output channel) = (i & 3) + 8 (i >> 2) + 4 (lane >> 5)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int og = wave * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
        if (og < O) s_lg[og][r] = __bfloat162float(__float2bfloat16(acc[i] + bv[i]));
    }
    __syncthreads();
    // softmax over the D bins of each pixel: thread (part, p) covers bins part, part + 8, ...
    constexpr int kParts = kBlock / kDnPix;
    const int p = threadIdx.x % kDnPix, part = threadIdx.x / kDnPix;
    float m = -INFINITY;
    for (int d = part; d < D; d += kParts) m = fmaxf(m, s_lg[d][p]);
    s_red[0][part][p] = m;
    __syncthreads();
    m = s_red[0][0][p];
#pragma unroll
    for (int j = 1; j < kParts; ++j) m = fmaxf(m, s_red[0][j][p]);
    float sum = 0.f;
    for (int d = part; d < D; d += kParts) sum += expf(s_lg[d][p] - m);
    s_red[1][part][p] = sum;
    __syncthreads();
    sum = 0.f;
#pragma unroll
    for (int j = 0; j < kParts; ++j) sum += s_red[1][j][p];
    const int q = q0 + p;
    if (q < npix) {
        const int bn = q / HW, hw = q - bn * HW;
        float* dst = depth + (size_t)bn * D * HW + hw;
        for (int d = part; d < D; d += kParts) dst[(size_t)d * HW] = expf(s_lg[d][p] - m) / sum;
    }
    // context rows: 64 consecutive channels of a pixel = one 128-B row
    for (int i = threadIdx.x; i < kDnPix * kC; i += kBlock) {
        const int pp = i / kC, c = i - pp * kC;
        if (q0 + pp < npix) ctx_t[(size_t)(q0 + pp) * kC + c] = __float2bfloat16(s_lg[D + c][pp]);
    }
}

// ---- depthnet + lift, version 2: one block = 32 pixels x 8 waves, v_mfma_f32_16x16x32_bf16.
// Wave m owns output rows [16m, 16m + 16) (its weight rows: 16 x K bf16, loaded once per lane straight
// into the A fragments -- K/32 16-B loads, all in flight with the feature loads); the block's feature
// tile is staged in LDS exactly as it lies in memory ([k][pixel], 8 consecutive pixels of one channel
// per 16-B load and per ds_write_b128), and the B fragments (8 channels of one pixel per lane) come out
// of it transposed by ds_read_b64_tr_b16 (gfx950: 4 rows x 16 columns of 16-bit elements, delivered
// column-major), two per K step. Then logits + bias rounded to bf16 (the autocast conv's output), depth
// softmax over the first D rows, context rows -- as k_depthnet_lift.
// pixels per block (16-pixel MFMA column tiles): 48 -> 176 blocks at B=8 (32 -> 264 blocks, 8 CUs run two)
constexpr int kDn2Pix = 48;
constexpr int kDn2Waves = 8;                   // 8 x 16 = 128 output rows >= D + C
constexpr int kDn2Block = kDn2Waves * kWave;

template <int K, int PX>  // input channels (compile-time: straight-line code, every load up front), pixels per block
__global__ __launch_bounds__(kDn2Block) void k_depthnet_lift2(const bf16* __restrict__ feat,
                                                              const bf16* __restrict__ weight,
                                                              const bf16* __restrict__ bias, int D, int HW,
                                                              int npix, float* __restrict__ depth,
                                                              bf16* __restrict__ ctx_t) {
    static_assert(K % 32 == 0 && K <= kDnMaxK, "K steps of 32 staged in LDS");
    static_assert(PX % 16 == 0, "16-pixel MFMA column tiles");
    constexpr int kRow = PX * 2 + 8;  // LDS bytes per channel row (+8: spread the banks, 8-B aligned)
    constexpr int kTiles = PX / 16;
    using bf16x8 = __attribute__((ext_vector_type(8))) short;
    using v4s = __attribute__((ext_vector_type(4))) short;
    using f32x4 = __attribute__((ext_vector_type(4))) float;
    __shared__ __attribute__((aligned(16))) unsigned char s_x[K * kRow];  // [k][pixel] bf16
    __shared__ float s_lg[kDnMaxO][PX + 1];                                  // bf16-rounded logits
    __shared__ float s_red[2][kDn2Block / PX][PX];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int q0 = xcd_block() * PX;  // XCD x takes a contiguous run of pixel tiles
    if (q0 >= npix) return;  // block-uniform
    const int O = D + kC;
    constexpr int kParts = kDn2Block / PX;  // threads past kParts * PX sit the softmax out
    constexpr int kPerPart = (64 + kParts - 1) / kParts;  // D <= 64 (D + C <= kDnMaxO)
    const int p = threadIdx.x % PX, part = threadIdx.x / PX;
    const bool sm = part < kParts;
    // ---- loads: this wave's weight rows (A fragments) and the block's feature tile, all in flight
    const int arow = wave * 16 + (lane & 15);
    const int kq = 8 * (lane >> 4);  // k offset of the lane's 8 elements inside a 32-wide K step
    constexpr int kSteps = K / 32;
    // Loads are unconditional (clamped addresses, no branches, so none waits on another): rows past O
    // only feed logits that are never written, and the pixel columns of a clamped tail only feed their
    // own discarded outputs.
    const int g = lane >> 4, c16 = lane & 15;
    const bf16* wrow = weight + (size_t)min(arow, O - 1) * K + kq;
    bf16x8 a[kSteps];
#pragma unroll
    for (int s = 0; s < kSteps; ++s) a[s] = *reinterpret_cast<const bf16x8*>(wrow + 32 * s);
    float bv[4];  // the bias of this lane's 4 output rows, in flight with the rest
#pragma unroll
    for (int i = 0; i < 4; ++i) bv[i] = __bfloat162float(bias[min(wave * 16 + 4 * g + i, O - 1)]);
    constexpr int kFeatIt = K * (PX / 8) / kDn2Block;  // 16-B feature loads per thread
    static_assert(K * (PX / 8) % kDn2Block == 0, "whole feature loads per thread");
    uint4 fv[kFeatIt];
#pragma unroll
    for (int t = 0; t < kFeatIt; ++t) {
        const int i = threadIdx.x + t * kDn2Block;
        const int k = i / (PX / 8), q = min(q0 + (i % (PX / 8)) * 8, npix - 8);
        const int bn = q / HW, hw = q - bn * HW;  // HW % 8 == 0: 8 pixels never straddle an image
        fv[t] = *reinterpret_cast<const uint4*>(feat + ((size_t)bn * K + k) * HW + hw);
    }
#pragma unroll
    for (int t = 0; t < kFeatIt; ++t) {
        const int i = threadIdx.x + t * kDn2Block;
        const int k = i / (PX / 8), p8 = (i % (PX / 8)) * 8;
        *reinterpret_cast<uint4*>(s_x + k * kRow + p8 * 2) = fv[t];
    }
    __syncthreads();
    // ---- MFMA: two 16-pixel column tiles, K/32 steps; B fragments by transposed LDS reads
    f32x4 acc[kTiles];
#pragma unroll
    for (int t = 0; t < kTiles; ++t) acc[t] = f32x4{};
    const int tq = c16 >> 2, tp = c16 & 3;
#pragma unroll
    for (int s = 0; s < kSteps; ++s) {
#pragma unroll
        for (int t = 0; t < kTiles; ++t) {
            // lane 4q+p of a 16-lane group addresses row q, columns 4p..4p+3 of a 4 x 16 block; lane c of
            // the group receives column c (pixel 16t + c), rows 0..3 (4 consecutive channels)
            const unsigned char* base = s_x + (32 * s + 8 * g + tq) * kRow + (16 * t + 4 * tp) * 2;
            const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) v4s*)(base));
            const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) v4s*)(base + 4 * kRow));
            const bf16x8 b = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s], b, acc[t], 0, 0, 0);
        }
    }
    // C/D: column (pixel) = lane & 15, row (output) = 4 (lane >> 4) + i
#pragma unroll
    for (int t = 0; t < kTiles; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int o = wave * 16 + 4 * g + i;
            if (o < O) s_lg[o][16 * t + c16] = __bfloat162float(__float2bfloat16(acc[t][i] + bv[i]));
        }
    __syncthreads();
    // ---- softmax over the D bins of each pixel: thread (part, p) covers bins part, part + 16, ...
    float m = -INFINITY;
    for (int d = part; sm && d < D; d += kParts) m = fmaxf(m, s_lg[d][p]);
    if (sm) s_red[0][part][p] = m;
    __syncthreads();
    m = s_red[0][0][p];
#pragma unroll
    for (int j = 1; j < kParts; ++j) m = fmaxf(m, s_red[0][j][p]);
    float sum = 0.f;
    for (int d = part; sm && d < D; d += kParts) sum += expf(s_lg[d][p] - m);
    if (sm) s_red[1][part][p] = sum;
    __syncthreads();
    sum = 0.f;
#pragma unroll
    for (int j = 0; j < kParts; ++j) sum += s_red[1][j][p];
    const int q = q0 + p;
    if (sm && q < npix) {
        const int bn = q / HW, hw = q - bn * HW;
        float* dst = depth + (size_t)bn * D * HW + hw;
#pragma unroll
        for (int i = 0; i < kPerPart; ++i) {
            const int d = part + kParts * i;
            if (d < D) dst[(size_t)d * HW] = expf(s_lg[d][p] - m) / sum;
        }
    }
    for (int i = threadIdx.x; i < PX * kC; i += kDn2Block) {
        const int pp = i / kC, c = i - pp * kC;
        if (q0 + pp < npix) ctx_t[(size_t)(q0 + pp) * kC + c] = __float2bfloat16(s_lg[D + c][pp]);
    }
}

// ---- depthnet + lift, version 3: pixel-major (channels-last) features, one block per CU.
// The feature map (B*N, K, H, W) as the channels-last tensor of a channels-last Up stage: pixel q's K
// channels are one contiguous K*2-byte row, so a block's pixel tile is ONE contiguous run of memory
// (every line it touches is wholly its own) instead of K strided runs of 2*PX bytes (the NCHW tile of
// k_depthnet_lift2 touched ~1.8 lines per 96 useful bytes and waited 6.5 us for them in the step).
// The grid is one block per CU (the pixel count split as evenly as possible: c3's 8,448 pixels are
// 256 tiles of 33), so every CU takes in its share of the features plus the weights, which every
// block reads (from L2). The tile is staged in LDS as [pixel][k] (row stride K*2 + 16 B: the 16 rows
// of a B fragment fall on different banks) and the B fragments (8 channels of one pixel per lane) are
// plain 16-B LDS reads. Rows past the tile's pixel count are clamped copies of its last row and only
// feed output columns that are never written. A fragments and epilogue (bias, bf16 rounding, softmax,
// context rows) as k_depthnet_lift2; identical results.
#ifndef LSS_DN3_BPC
#define LSS_DN3_BPC 1  // experiments: lift blocks per CU (2 -- 512 blocks of ~17 pixels at c3, two resident per
                       // CU -- measured 11.0 vs 8.9 us in-step, profiles/r06/lift_blocks_per_cu_ab.txt)
#endif
constexpr int kDn3Waves = 8;             // 8 x 16 = 128 output rows >= D + C
constexpr int kDn3Block = kDn3Waves * kWave;
constexpr int kDn3MaxPix = 48;           // pixels per block at most: three 16-column MFMA tiles
// K slices of k_depthnet_lift3's loads: slice 0 multiplied while the rest arrive (c3 in-step 11.3 -> 10.9 us;
// 4 slices no better, profiles/r03/s3/trace_lift3_slices*.txt)
constexpr int kDn3Slices = 2;

// The depthnet weights in k_depthnet_lift3's A-fragment order (lss_depthnet_pack): piece (wave w,
// K step s, lane l) = the 8 bf16 weights of output row min(16 w + (l & 15), O - 1), channels
// 32 s + 8 (l >> 4) .. + 7, at piece index (w K/32 + s) 64 + l. A wave's fragment load for one K
// step is then one contiguous 1 KB (eight whole lines) instead of 64 B of each of 16 rows (16 lines,
// each fetched again by the next K step). Rounded to bf16 as torch's .to(torch.bfloat16) (nearest
// even); `plain` gets the same values row-major (the backward's GEMM operand), bias_out the bias.
__device__ __forceinline__ bf16 to_bf16(float x) { return __float2bfloat16(x); }
__device__ __forceinline__ bf16 to_bf16(bf16 x) { return x; }
template <typename WT>
__global__ __launch_bounds__(kBlock) void k_depthnet_pack(const WT* __restrict__ weight, const WT* __restrict__ bias,
                                                          int O, int K, bf16* __restrict__ packed,
                                                          bf16* __restrict__ plain, bf16* __restrict__ bias_out) {
    const int ksteps = K / 32;
    const int t = blockIdx.x * kBlock + threadIdx.x;
    if (bias_out && t < O) bias_out[t] = to_bf16(bias[t]);
    if (t >= kDn3Waves * ksteps * kWave) return;
    const int l = t % kWave, st = (t / kWave) % ksteps, w = t / (kWave * ksteps);
    const int r = 16 * w + (l & 15), k0 = 32 * st + 8 * (l >> 4);
    const WT* src = weight + (size_t)min(r, O - 1) * K + k0;
    bf16 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = to_bf16(src[j]);
    *reinterpret_cast<uint4*>(packed + (size_t)t * 8) = *reinterpret_cast<const uint4*>(v);
    if (plain && r < O) *reinterpret_cast<uint4*>(plain + (size_t)r * K + k0) = *reinterpret_cast<const uint4*>(v);
}

// One block per CU (8 waves, 2 per SIMD): up to 256 VGPRs per lane. Without the waves-per-EU bound
// the compiler budgets 128 (the 4 waves per SIMD two blocks' LDS would allow) and kept the feature
// loads in scratch: stores behind vmcnt waits, reloads behind a vmcnt(0) -- the stage serialised.
template <int K, bool PACKED>
__global__ __launch_bounds__(kDn3Block) __attribute__((amdgpu_waves_per_eu(1, 2 * LSS_DN3_BPC))) void k_depthnet_lift3(const bf16* __restrict__ feat,
                                                              const bf16* __restrict__ weight,
                                                              const bf16* __restrict__ bias, int D, int HW,
                                                              int npix, int nlift, float* __restrict__ depth,
                                                              bf16* __restrict__ ctx_t) {
    static_assert(K % 32 == 0 && K <= kDnMaxK, "K steps of 32");
    constexpr int PX = kDn3MaxPix;
    constexpr int kTiles = PX / 16;
    constexpr int kRow = K * 2 + 16;  // LDS bytes per pixel row
    using bf16x8 = __attribute__((ext_vector_type(8))) short;
    using f32x4 = __attribute__((ext_vector_type(4))) float;
    __shared__ __attribute__((aligned(16))) unsigned char s_x[PX * kRow];  // [pixel][k] bf16
    __shared__ float s_lg[kDnMaxO][PX + 1];                                // bf16-rounded logits
    __shared__ float s_red[2][kDn3Block / PX][PX];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // XCD x takes one contiguous run of pixel tiles (c3: sample x), as the splat's chunk blocks take
    // the CSR: the context rows a splat gathers were written through its own XCD's L2
    const int blk = xcd_block();
    if (blk >= nlift) return;
    // pixel tile [q0, q1): the pixels split as evenly as possible over the nlift blocks
    const int q0 = (int)(((long)npix * blk) / nlift), q1 = (int)(((long)npix * (blk + 1)) / nlift);
    const int np = q1 - q0;  // 1 <= np <= PX (the host sizes nlift so)
    const int O = D + kC;
    [[maybe_unused]] const int tslot = blk * kDn3Waves + wave;  // LSS_TRACE builds only
    LSS_STAMP(tslot, 0);
    constexpr int kParts = kDn3Block / PX;                 // softmax: threads (part, p) of the block
    constexpr int kPerPart = (64 + kParts - 1) / kParts;   // D <= 64 (D + C <= kDnMaxO)
    const int p = threadIdx.x % PX, part = threadIdx.x / PX;
    const bool sm = part < kParts;
    // ---- loads, all in flight together, in kParts K slices: slice h of the tile (channels
    // [h K/kParts, (h+1) K/kParts) of every pixel row, 16 B per thread and load), then this wave's
    // weight A fragments for the slice's K steps; then the bias values (clamped addresses, no
    // branches). Loads complete in order, so slice 0 is staged and multiplied while the later slices
    // are still arriving (the per-CU intake, ~161 KB at c3, is the stage's bound).
    constexpr int kSlices = kDn3Slices;
    constexpr int kCPR = K * 2 / 16;                     // 16-B pieces per pixel row
    constexpr int kSCPR = kCPR / kSlices;                // ... per pixel row and slice
    constexpr int kSChunks = PX * kSCPR;                 // 16-B pieces of a slice
    constexpr int kSIt = (kSChunks + kDn3Block - 1) / kDn3Block;
    constexpr int kSteps = K / 32;
    constexpr int kSSteps = kSteps / kSlices;
    static_assert(kCPR % kSlices == 0 && kSteps % kSlices == 0, "K slices");
    const unsigned char* tile = reinterpret_cast<const unsigned char*>(feat + (size_t)q0 * K);
    const int arow = wave * 16 + (lane & 15);
    const int kq = 8 * (lane >> 4);
    const int g = lane >> 4, c16 = lane & 15;
    const bf16* wrow = weight + (size_t)min(arow, O - 1) * K + kq;
    // (unconditional even for a wave past the output rows -- its clamped row is one cached line per
    // K step -- so the compiler can count every load: a load under a branch makes it wait for the
    // worst case, and the tile's LDS writes then waited for most of the weights)
    u32x4 fv[kSlices][kSIt];  // (a native vector type: an array of the uint4 struct stayed in scratch)
    bf16x8 a[kSteps];
#pragma unroll
    for (int h = 0; h < kSlices; ++h) {
#pragma unroll
        for (int t = 0; t < kSIt; ++t) {
            const int i = threadIdx.x + t * kDn3Block;
            const int r = min(i / kSCPR, np - 1), c = h * kSCPR + i % kSCPR;
            fv[h][t] = *reinterpret_cast<const u32x4*>(tile + (size_t)r * K * 2 + c * 16);
        }
#pragma unroll
        for (int s = h * kSSteps; s < (h + 1) * kSSteps; ++s) {
            if (PACKED)  // lss_depthnet_pack's order: each wave-instruction reads one contiguous 1 KB
                a[s] = *reinterpret_cast<const bf16x8*>(weight + ((size_t)(wave * kSteps + s) * kWave + lane) * 8);
            else
                a[s] = *reinterpret_cast<const bf16x8*>(wrow + 32 * s);
        }
    }
    float bv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) bv[i] = __bfloat162float(bias[min(wave * 16 + 4 * g + i, O - 1)]);
    // ---- per slice: stage it in LDS, then its MFMA steps over kTiles 16-pixel column tiles. All
    // tiles always (compile-time trip counts: the LDS reads and MFMAs pipeline); columns past the
    // tile's pixels read clamped rows and only feed logits that are never read. Same K order as one
    // slice: identical results. The slice index is a compile-time constant in each call (a loop over
    // it left fv[h][...] dynamically indexed, and the compiler kept the loaded features in scratch).
    f32x4 acc[kTiles];
#pragma unroll
    for (int t = 0; t < kTiles; ++t) acc[t] = f32x4{};
    auto slice = [&](auto hc) {
        constexpr int h = decltype(hc)::value;
#pragma unroll
        for (int t = 0; t < kSIt; ++t) {
            const int i = threadIdx.x + t * kDn3Block;
            if (kSChunks % kDn3Block == 0 || i < kSChunks)
                *reinterpret_cast<u32x4*>(s_x + (i / kSCPR) * kRow + (h * kSCPR + i % kSCPR) * 16) = fv[h][t];
        }
        __syncthreads();
        if (h == 0) LSS_STAMP(tslot, 1);
        // (every wave, also one past the output rows: a branch here would let the compiler sink the
        // weight loads into it, behind the barrier, one round trip per K step)
#pragma unroll
        for (int s = h * kSSteps; s < (h + 1) * kSSteps; ++s) {
#pragma unroll
            for (int t = 0; t < kTiles; ++t) {
                // lane (g, c16) of the B fragment: pixel 16t + c16, channels 32s + 8g .. + 7
                const bf16x8 b =
                    *reinterpret_cast<const bf16x8*>(s_x + (16 * t + c16) * kRow + (32 * s + 8 * g) * 2);
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s], b, acc[t], 0, 0, 0);
            }
        }
    };
    static_assert(kSlices == 2, "two K slices");
    slice(std::integral_constant<int, 0>{});
    slice(std::integral_constant<int, 1>{});
    // C/D: column (pixel) = lane & 15, row (output) = 4 (lane >> 4) + i
#pragma unroll
    for (int t = 0; t < kTiles; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int o = wave * 16 + 4 * g + i;
            if (o < O) s_lg[o][16 * t + c16] = __bfloat162float(__float2bfloat16(acc[t][i] + bv[i]));
        }
    __syncthreads();
    LSS_STAMP(tslot, 2);
    // ---- softmax over the D bins of each pixel: thread (part, p) covers bins part, part + kParts, ...
    const bool pl = sm && p < np;
    float m = -INFINITY;
    for (int d = part; pl && d < D; d += kParts) m = fmaxf(m, s_lg[d][p]);
    if (sm) s_red[0][part][p] = m;
    __syncthreads();
    m = s_red[0][0][p];
#pragma unroll
    for (int j = 1; j < kParts; ++j) m = fmaxf(m, s_red[0][j][p]);
    float sum = 0.f;
    for (int d = part; pl && d < D; d += kParts) {
        const float e = expf(s_lg[d][p] - m);
        s_lg[d][p] = e;  // (this thread's own bins: read back below instead of a second expf)
        sum += e;
    }
    if (sm) s_red[1][part][p] = sum;
    __syncthreads();
    sum = 0.f;
#pragma unroll
    for (int j = 0; j < kParts; ++j) sum += s_red[1][j][p];
    if (pl) {
        const int q = q0 + p;
        const int bn = q / HW, hw = q - bn * HW;
        float* dst = depth + (size_t)bn * D * HW + hw;
#pragma unroll
        for (int i = 0; i < kPerPart; ++i) {
            const int d = part + kParts * i;
            if (d < D) dst[(size_t)d * HW] = s_lg[d][p] / sum;
        }
    }
    // context rows: the tile's np rows of 64 bf16 are one contiguous run; 8 channels per 16-B store
    for (int i = threadIdx.x; i < np * (kC / 8); i += kDn3Block) {
        const int pp = i / (kC / 8), c8 = (i - pp * (kC / 8)) * 8;
        bf16 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = __float2bfloat16(s_lg[D + c8 + j][pp]);
        *reinterpret_cast<uint4*>(ctx_t + (size_t)(q0 + pp) * kC + c8) = *reinterpret_cast<const uint4*>(v);
    }
    LSS_STAMP(tslot, 3);
}

// Flat fp32 master -> bf16 working copy (flat_params.FlatParams, once per forward), the depthnet weight
// also written in k_depthnet_lift3's fragment order from the same fp32 values: blocks [0, ncast) round
// 16 elements per thread (four 16-B loads, two 16-B stores; nearest even, as torch's .to(bfloat16)), blocks
// [0, npack) -- dispatched first, beside the cast -- are k_depthnet_pack's pieces. One launch where the
// step had a cast and a pack.
__global__ __launch_bounds__(kBlock) void k_flat_cast_bf16(const float* __restrict__ src, bf16* __restrict__ dst,
                                                          long n, int npack, const float* __restrict__ dn_weight, int O,
                                                          int K, bf16* __restrict__ packed) {
    if ((int)blockIdx.x >= npack) {
        // 16 elements per thread: four 16-B loads in flight, then two 16-B stores
        const long i = ((long)(blockIdx.x - npack) * kBlock + threadIdx.x) * 16;
        if (i + 16 <= n) {
            float4 a[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) a[q] = *reinterpret_cast<const float4*>(src + i + 4 * q);
            bf16 v[16];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                v[4 * q] = __float2bfloat16(a[q].x);
                v[4 * q + 1] = __float2bfloat16(a[q].y);
                v[4 * q + 2] = __float2bfloat16(a[q].z);
                v[4 * q + 3] = __float2bfloat16(a[q].w);
            }
            *reinterpret_cast<uint4*>(dst + i) = *reinterpret_cast<const uint4*>(v);
            *reinterpret_cast<uint4*>(dst + i + 8) = *reinterpret_cast<const uint4*>(v + 8);
        } else {
            for (long j = i; j < n; ++j) dst[j] = __float2bfloat16(src[j]);
        }
        return;
    }
    const int ksteps = K / 32;
    const int t = blockIdx.x * kBlock + threadIdx.x;
    if (t >= kDn3Waves * ksteps * kWave) return;
    const int l = t % kWave, st = (t / kWave) % ksteps, w = t / (kWave * ksteps);
    const float* row = dn_weight + (size_t)min(16 * w + (l & 15), O - 1) * K + 32 * st + 8 * (l >> 4);
    bf16 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = __float2bfloat16(row[j]);
    *reinterpret_cast<uint4*>(packed + (size_t)t * 8) = *reinterpret_cast<const uint4*>(v);
}

// 16 bytes of fp32 or bf16 row elements -> fp32.
__device__ __forceinline__ void unpack16(const uint4& u, const float*, float* o) {
    o[0] = __uint_as_float(u.x); o[1] = __uint_as_float(u.y); o[2] = __uint_as_float(u.z); o[3] = __uint_as_float(u.w);
}
__device__ __forceinline__ void unpack16(const uint4& u, const bf16*, float* o) {
    const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        o[2 * i] = __uint_as_float(w[i] << 16);
        o[2 * i + 1] = __uint_as_float(w[i] & 0xFFFF0000u);
    }
}

// ----------------------------------------------------------------------------- splat forward
struct SplatGeo {
    int X, Y, Z, YT, ntiles_y;
    int ncells, nprime, nrows;  // bounds of the data-derived indices (LSS_DEBUG checks): cells, points, feature rows
};

constexpr int kYtMax = 128;  // cells per NCHW tile at most (LDS sizing)

// 16-byte vector stores of 16/sizeof(T) elements.
__device__ __forceinline__ void store_vec(float* dst, const float* src) {
    *reinterpret_cast<float4*>(dst) = *reinterpret_cast<const float4*>(src);
}
__device__ __forceinline__ void store_vec(bf16* dst, const float* src) {
    const float4 a = *reinterpret_cast<const float4*>(src);
    const float4 b = *reinterpret_cast<const float4*>(src + 4);
    bf16 v[8] = {__float2bfloat16(a.x), __float2bfloat16(a.y), __float2bfloat16(a.z), __float2bfloat16(a.w),
                 __float2bfloat16(b.x), __float2bfloat16(b.y), __float2bfloat16(b.z), __float2bfloat16(b.w)};
    *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(v);
}

// A cell with more than 64 entries, canonical order: streamed 64 at a time (rare), lane = channel.
template <bool FUSED, typename RT>
__device__ float reduce_big_cell(int start, int nprime, const long long* __restrict__ key,
                                 const int32_t* __restrict__ row, const float* __restrict__ depth,
                                 const RT* __restrict__ rows_base, int lane, int* cell_out, int nrows) {
    const int cell = (int)(key[start] >> 32);
    *cell_out = cell;
    float acc = 0.f;
    for (int b = start;; b += kWave) {
        const int e = b + lane;
        const long long k = e < nprime ? key[e] : -1ll;
        const bool mine = (int)(k >> 32) == cell;
        const unsigned long long m = __ballot(mine);
        const int n = __popcll(m);  // entries of the cell are contiguous from b
        const int r = mine ? dchk(FUSED ? row[e] : (int)(k & 0xFFFFFFFF), nrows, kDbgSplatRow) : 0;
        const float w = (FUSED && mine) ? depth[dchk((int)(k & 0xFFFFFFFF), nprime, kDbgSplatPoint)] : 1.f;
        for (int i = 0; i < n; ++i) {
            const float v = to_f32(rows_base[(size_t)__builtin_amdgcn_readlane(r, i) * kC + lane]);
            acc = FUSED ? fmaf(readlane_f(w, i), v, acc) : __fadd_rn(acc, v);
        }
        if (n < kWave) break;
    }
    return acc;
}

// ----------------------------------------------------------------------------- splat forward, channels-last
// The production layout (BevEncode runs channels-last): every BEV cell is one contiguous row of C
// values. One launch, two block roles, four independent waves per block, no block barriers:
//   chunk waves: the wave of chunk w owns the cells that START among canonical entries
//     [64w, 64w + 64) and reads the window [64w - 1, 64w + 128) (cells have <= 64 entries there;
//     a longer one is streamed by reduce_big_cell). Round trip 1: keys and context-row indices.
//     Round trip 2: the depth weights and every owned entry's context row, 16-B lane slices, all in
//     flight at once. The rows are summed lane group by lane group in canonical order (ascending
//     point id per cell, the NCHW tile kernel's order, so both layouts agree bit for bit); each
//     finished cell's row is stored straight to the BEV. No global load follows a store, so stores
//     never sit in front of a load's wait.
//   zero waves: zu x 64 consecutive cells each (zu <= kMaxZeroUnits, chosen per launch); the rows of
//     the empty cells are written as zeros with 16-B non-temporal stores, so every BEV element is
//     written exactly once.
// The CSR's sentinel tail (key -1 past the last entry, lss_csr_build) spares a load of the count.
#ifndef LSS_SPLAT_ROLES
#define LSS_SPLAT_ROLES 0  // experiments only: 1 runs the chunk waves alone, 2 the zero fill alone
#endif
// (Round 4 held the zero waves dispatched beside the chunk waves back for an s_sleep of 2,048 cycles,
// sized per launch from the wave slots, so the chunk waves' round trips met a quieter memory system:
// 12.4 -> 11.6 us in-step then. Once the chunk waves retire their gathers before their row stores
// (LSS_SPLAT_WAITALL) the hold-back cost time instead -- 11.74 / 11.59 without vs 12.53 / 11.86 us
// with it in-step, 12.7 vs 13.3 us kernel-stamped (profiles/r05/prof_ab_splat_holdback.txt) -- and
// was removed.)
#ifndef LSS_SPLAT_SKIP
#define LSS_SPLAT_SKIP 0  // experiments only (wrong sums): 1 rows from 8 L1-resident rows, 2 one depth line, 4 no row stores
#endif
// 64-cell zero-fill units per zero wave, zu in [1, kMaxZeroUnits], chosen per launch (splat_zero_units):
// the fewest that let every chunk wave AND every zero wave be resident at once. At c3 the 5,386 chunk
// waves leave 1,782 of the 7,168 wave slots, so 1 unit per wave (5,000 zero waves) ran the last 3,200
// zero waves as a second generation behind the chunk waves; 3 units (1,667 waves) fit: in-step 12.21 ->
// 11.63 us (2 units: 11.98, 4: 11.78; profiles/r06/splat_zu_ab.txt). When the chunk waves alone fill
// the slots (c5) the zero fill is a second generation anyway and keeps 1 unit per wave. (Rounds 3-4
// measured 2-16 units slower with 6 resident waves per SIMD, where no zu made the grid one generation.)
#ifndef LSS_SPLAT_ZU
#define LSS_SPLAT_ZU 0  // experiments only: > 0 forces that many units per zero wave
#endif
constexpr int kMaxZeroUnits = 4;
#ifndef LSS_SPLAT_WAVES
#define LSS_SPLAT_WAVES 4
#endif
constexpr int kSplatWaves = LSS_SPLAT_WAVES;  // waves per block of the channels-last splat (waves are
                                              // independent; 2 / 7 / 8 measured slower, round 4)
constexpr int kSplatBlock = kSplatWaves * kWave;
#ifndef LSS_SPLAT_OCC
#define LSS_SPLAT_OCC 7
#endif
constexpr int kSplatMinWaves = LSS_SPLAT_OCC;  // occupancy floor (waves per SIMD): 72 VGPRs, 16 KB LDS per block

// Zero-fill units [u0, u0 + zu): cells [64u, 64u + 64) each; empty cells' rows written as zeros.
template <typename OutT>
__device__ void zero_empty_rows(int u0, int zu, const int32_t* __restrict__ cell_start, const BevGeo& g,
                                OutT* __restrict__ out, int lane) {
    unsigned long long emask[kMaxZeroUnits];
#pragma unroll
    for (int i = 0; i < kMaxZeroUnits; ++i) {  // every unit's cell starts in flight together
        const int k = (u0 + i) * kWave + lane;
        bool empty = false;
        if (i < zu && k < g.ncells) empty = cell_start[k] == cell_start[k + 1];
        emask[i] = __ballot(empty);
    }
    constexpr int EPL = 16 / sizeof(OutT), LPR = kC / EPL, RPS = kWave / LPR;
#pragma unroll
    for (int i = 0; i < kMaxZeroUnits; ++i) {
        const int k0 = (u0 + i) * kWave;
        for (int r0 = 0; r0 < kWave; r0 += RPS) {
            const int r = r0 + lane / LPR;
            if ((emask[i] >> r) & 1ull)
                __builtin_nontemporal_store(u32x4{0u, 0u, 0u, 0u},
                                            reinterpret_cast<u32x4*>(cell_row(out, k0 + r, g) + (lane % LPR) * EPL));
        }
    }
}

// Owned entries of a chunk, relative to its base: [s, end); big >= 0: the last owned cell starts at
// `big` and runs past the 128-entry window (it is excluded from [s, end)).
struct Span {
    int s, end, big;
};

__device__ __forceinline__ Span chunk_span(int c0, int c1, int prevcell, int lane) {
    const int up = __shfl(c0, (lane + 63) & 63, kWave);
    const int before = lane == 0 ? prevcell : up;
    const unsigned long long sm = __ballot(c0 >= 0 && c0 != before);  // cell starts (cell -1: past the end)
    if (!sm) return Span{0, 0, -1};
    const int first = __builtin_ctzll(sm), last = 63 - __builtin_clzll(sm);
    const int lastcell = __builtin_amdgcn_readlane(c0, last);
    const unsigned long long m0 = __ballot(lane > last && c0 != lastcell);
    if (m0) return Span{first, (int)__builtin_ctzll(m0), -1};
    const unsigned long long m1 = __ballot(c1 != lastcell);
    if (m1) return Span{first, kWave + (int)__builtin_ctzll(m1), -1};
    return Span{first, last, last};
}

template <typename RT> struct RowSlice {
    static constexpr int EPL = 16 / sizeof(RT);  // row elements per 16-B lane slice
    static constexpr int LPR = kC / EPL;         // lanes per row = lanes per group: 16 (fp32), 8 (bf16)
    static constexpr int NG = kWave / LPR;       // groups per wave: 4, 8
};

template <int EPL>
__device__ __forceinline__ void store_slice(float* dst, const float* a) {
#pragma unroll
    for (int i = 0; i < EPL; i += 4) *reinterpret_cast<float4*>(dst + i) = make_float4(a[i], a[i + 1], a[i + 2], a[i + 3]);
}
template <int EPL>
__device__ __forceinline__ void store_slice(bf16* dst, const float* a) {
    bf16 v[EPL];
#pragma unroll
    for (int i = 0; i < EPL; ++i) v[i] = __float2bfloat16(a[i]);
    if constexpr (EPL == 4) *reinterpret_cast<uint2*>(dst) = *reinterpret_cast<const uint2*>(v);
    else *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(v);
}

// Entries in flight per lane group. A group holds at most ceil(128 / NG) entries (16 with bf16 rows),
// so with 16 every group issues all its gathers before its first row store: a load issued after a
// store would wait for that store too (vmcnt counts both, in order), and stores are slow while the
// zero fill saturates the write path.
constexpr int kUnroll = 8;
#ifndef LSS_SPLAT_WAITALL
#define LSS_SPLAT_WAITALL 1
#endif

// s_waitcnt vmcnt(0), expcnt and lgkmcnt left at their maxima (gfx9 encoding: vmcnt[3:0] | expcnt[6:4] |
// lgkmcnt[11:8] | vmcnt_hi[15:14])
constexpr int kWaitVm0 = 0x0F70;

// Entry metadata of a chunk's 128-entry window, staged once in LDS: (row, point, cell).
struct alignas(16) EntryMeta {
    int row, p, cell, pad;
};

// Depth weights of a lane group's next entries [e, e + KU): lane j of the group loads the weight of
// entry e + j, so ONE wave-wide gather serves all groups, then each weight is broadcast inside the
// group through the LDS crossbar (ds_bpermute).
template <int LPR, int KU>
__device__ __forceinline__ float group_weight_load(const EntryMeta* __restrict__ meta,
                                                   const float* __restrict__ depth, int e, int last, int lane,
                                                   int nprime) {
    static_assert(LPR >= KU, "one lane per entry of the batch");
    if (LSS_SPLAT_SKIP & 2) return depth[lane % LPR];
    return depth[dchk(meta[min(e + lane % LPR, last)].p, nprime, kDbgSplatPoint)];
}
// weight of entry e + u of the group (broadcast from the group's lane u; one VGPR held across the wait)
#ifndef LSS_SPLAT_DPPW
#define LSS_SPLAT_DPPW 1
#endif
// 8-lane groups (bf16 rows): lane U of every group by two DPP moves -- a quad broadcast of lane U & 3,
// then the other quad of each group takes it from its neighbour quad (row_shr:4 into banks 1 / 3, or
// row_shl:4 into banks 0 / 2) -- instead of a ds_bpermute through the LDS crossbar
template <int U>
__device__ __forceinline__ float bcast8(float wd) {
    constexpr int k = U & 3;
    const int q = __builtin_amdgcn_update_dpp(0, __float_as_int(wd), k * 0x55, 0xf, 0xf, false);  // quad_perm [k,k,k,k]
    if constexpr (U < 4) return __int_as_float(__builtin_amdgcn_update_dpp(q, q, 0x114, 0xf, 0xA, false));
    else return __int_as_float(__builtin_amdgcn_update_dpp(q, q, 0x104, 0xf, 0x5, false));
}
template <int LPR>
__device__ __forceinline__ float group_weight(float wd, int u, int lane) {
    if constexpr (LPR == 8 && LSS_SPLAT_DPPW) {
        switch (u) {  // (u is a constant in every unrolled use)
            case 0: return bcast8<0>(wd);
            case 1: return bcast8<1>(wd);
            case 2: return bcast8<2>(wd);
            case 3: return bcast8<3>(wd);
            case 4: return bcast8<4>(wd);
            case 5: return bcast8<5>(wd);
            case 6: return bcast8<6>(wd);
            default: return bcast8<7>(wd);
        }
    }
    return __shfl(wd, lane - lane % LPR + u, kWave);
}

template <bool FUSED, typename RT, typename OutT>
__device__ __forceinline__ void splat_chunk(int w, int nprime, const float* __restrict__ depth,
                                            const RT* __restrict__ rows_base,
                                            const long long* __restrict__ sorted_key,
                                            const int32_t* __restrict__ sorted_row, const BevGeo& g,
                                            OutT* __restrict__ out, EntryMeta* __restrict__ meta,
                                            float* __restrict__ part, int lane) {
    using RS = RowSlice<RT>;
    // round trip 1: keys (cell << 32 | point), context rows, the previous entry's cell
    const int base = w * kWave;
    const int e0 = base + lane, e1 = base + kWave + lane;
    const long long k0 = e0 < nprime ? sorted_key[e0] : -1ll;
    const long long k1 = e1 < nprime ? sorted_key[e1] : -1ll;
    int rs0 = 0, rs1 = 0;
    if (FUSED) {
        rs0 = e0 < nprime ? sorted_row[e0] : 0;
        rs1 = e1 < nprime ? sorted_row[e1] : 0;
    }
    const int prevcell = base > 0 ? (int)(sorted_key[base - 1] >> 32) : -2;
    const int c0 = (int)(k0 >> 32), c1 = (int)(k1 >> 32);
    const int p0 = (int)(k0 & 0xFFFFFFFF), p1 = (int)(k1 & 0xFFFFFFFF);
    if (!FUSED) {
        rs0 = p0;
        rs1 = p1;
    }
    LSS_STAMP(w, 1);
    const Span sp = chunk_span(c0, c1, prevcell, lane);
    const int s = uniform(sp.s), end = uniform(sp.end), big = uniform(sp.big);
    if (end > 0) {
        meta[lane] = EntryMeta{rs0, p0, c0, 0};
        meta[kWave + lane] = EntryMeta{rs1, p1, c1, 0};
        __builtin_amdgcn_wave_barrier();
        // The owned entries [s, end) (n <= 128) are split evenly over the NG groups of LPR lanes:
        // group q sums entries [s + n*q/NG, s + n*(q+1)/NG) cell by cell; lane j of a group owns row
        // elements [EPL*j, EPL*j + EPL). A cell cut by group boundaries is summed in pieces: every
        // group after the one holding its first entry leaves its piece in part[q] (a group's only
        // LDS piece: the cell it starts inside of); the group holding the first entry keeps its own
        // piece in registers (its last cell) and, after a wave barrier, adds the later groups'
        // pieces in group order and stores the row. One row slot per group (2 KB per wave) keeps
        // the block at 16 KB of LDS, so 8 blocks (32 waves) fit a CU and the zero fill is resident
        // beside the chunk waves. The association depends only on the CSR (deterministic).
        const int n = end - s;
        const int grp = lane / RS::LPR, col = (lane % RS::LPR) * RS::EPL;
        auto gbeg = [&](int q) { return s + (n * q) / RS::NG; };
        const int gs = gbeg(grp), ge = gbeg(grp + 1);
        const int first_cell = gs < ge ? meta[gs].cell : -1;
        const bool head_split = gs < ge && gs > s && meta[gs - 1].cell == first_cell;
        const bool tail_split = gs < ge && ge < end && meta[ge].cell == meta[ge - 1].cell;
        float acc[RS::EPL];
#pragma unroll
        for (int i = 0; i < RS::EPL; ++i) acc[i] = 0.f;
        int cur = -1;
        auto put = [&](float* dst, int c) {
#pragma unroll
            for (int i = 0; i < RS::EPL; i += 4)
                *reinterpret_cast<float4*>(dst + c + i) = make_float4(acc[i], acc[i + 1], acc[i + 2], acc[i + 3]);
        };
        auto finish = [&](bool last, int c) {  // the cell `cur` ends at this point of the group
            if (cur == first_cell && head_split) put(part + grp * kC, c);  // a later piece of a cut cell
            else if (!(last && tail_split) && !(LSS_SPLAT_SKIP & 4))
                store_slice<RS::EPL>(cell_row(out, dchk(cur, g.ncells, kDbgSplatCell), g) + c, acc);
            // else: the first piece of a cut cell stays in acc (combined after the barrier)
        };
        // round trip 2 (one per kUnroll entries of a group): row slices and depth weights in flight together
        for (int e = gs; e < ge; e += kUnroll) {
            uint4 v[kUnroll];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const int4 m = *reinterpret_cast<const int4*>(&meta[min(e + u, ge - 1)]);  // (row, p, cell, -)
                const int mr = (LSS_SPLAT_SKIP & 1) ? (m.x & 7) : m.x;
                v[u] = *reinterpret_cast<const uint4*>(rows_base + (size_t)dchk(mr, g.nrows, kDbgSplatRow) * kC + col);
            }
            const float wd = FUSED ? group_weight_load<RS::LPR, kUnroll>(meta, depth, e, ge - 1, lane, nprime) : 0.f;
#if LSS_SPLAT_WAITALL
#pragma unroll
            for (int u = 0; u < kUnroll; ++u)  // (uses here keep the compiler from sinking a gather below the wait)
                asm volatile("" : : "v"(v[u].x), "v"(v[u].y), "v"(v[u].z), "v"(v[u].w));
            // Every gather of the batch retired here, before the loop below stores a finished cell's row:
            // vmcnt also counts stores (gfx9), so a wait for a later row issued after such a store --
            // the compiler's wait for row u, with a conditional store in front, is vmcnt(0) -- would
            // wait for that store's write to complete, a round trip per finished cell in the busiest
            // write phase of the kernel. An explicit s_waitcnt is known to the compiler's wait
            // insertion, so no row use after it waits again.
            __builtin_amdgcn_s_waitcnt(kWaitVm0);
#endif
            if (LSS_TRACE && e == gs && grp == 0) LSS_STAMP(w, 2);
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                if (e + u < ge) {
                    const int cl = meta[e + u].cell;
                    if (cl != cur) {
                        if (cur >= 0) finish(false, col);
#pragma unroll
                        for (int i = 0; i < RS::EPL; ++i) acc[i] = 0.f;
                        cur = cl;
                    }
                    float x[RS::EPL];
                    unpack16(v[u], (const RT*)nullptr, x);
                    const float wu = FUSED ? group_weight<RS::LPR>(wd, u, lane) : 1.f;
#pragma unroll
                    for (int i = 0; i < RS::EPL; ++i) acc[i] = FUSED ? fmaf(wu, x[i], acc[i]) : __fadd_rn(acc[i], x[i]);
                }
            }
        }
        // (the lane's column recomputed after the loop: kept live across it, it was the one VGPR over
        // the 72 of 7 waves per SIMD and went to scratch -- a reload round trip at every wave's end)
        const int tcol = (fresh_lane() % RS::LPR) * RS::EPL;
        if (cur >= 0) finish(true, tcol);
        __builtin_amdgcn_wave_barrier();
        // the cell cut at this group's end, if it starts in this group: its first piece (acc) plus
        // the later groups' pieces in group order (empty groups skipped; the cell ends where a
        // group's first cell is another one)
        if (tail_split && !(head_split && cur == first_cell)) {
            for (int q = grp + 1; q < RS::NG; ++q) {
                const int qs = gbeg(q);
                if (qs == gbeg(q + 1)) continue;  // empty group
                if (meta[qs].cell != cur) break;
#pragma unroll
                for (int i = 0; i < RS::EPL; ++i) acc[i] = __fadd_rn(acc[i], part[q * kC + tcol + i]);
            }
            if (!(LSS_SPLAT_SKIP & 4)) store_slice<RS::EPL>(cell_row(out, dchk(cur, g.ncells, kDbgSplatCell), g) + tcol, acc);
        }
    }
    if (big >= 0) {
        int cell;
        const float a2 = reduce_big_cell<FUSED, RT>(base + big, nprime, sorted_key, sorted_row, depth, rows_base, lane,
                                                    &cell, g.nrows);
        cell_row(out, dchk(cell, g.ncells, kDbgSplatCell), g)[lane] = from_f32<OutT>(a2);
    }
}

#ifndef LSS_SPLAT_ZFIRST
#define LSS_SPLAT_ZFIRST 0  // dispatch order: 0 chunk groups first, 1 zero-fill groups first
#endif

template <bool FUSED, typename RT, typename OutT>
__global__ __launch_bounds__(kSplatBlock, kSplatMinWaves) void k_splat_fwd_nhwc(const float* __restrict__ depth,
                                                           const RT* __restrict__ rows_base,
                                                           const int32_t* __restrict__ cell_start,
                                                           const long long* __restrict__ sorted_key,
                                                           const int32_t* __restrict__ sorted_row, BevGeo g,
                                                           int nprime, int nchunk_blocks, int nzero_blocks,
                                                           int zu, OutT* __restrict__ out) {
    __shared__ EntryMeta s_meta[kSplatWaves][2 * kWave];
    __shared__ __attribute__((aligned(16))) float s_part[kSplatWaves][RowSlice<RT>::NG * kC];
    const int lane = threadIdx.x & 63;
    const int wave = uniform(threadIdx.x >> 6);
    // Blocks come in groups of 8, one per XCD (blocks are dealt round-robin over the 8 XCDs): the
    // chunk groups first, then the zero-fill groups (c3: all 5,386 chunk waves start at t = 0 in the
    // 7,168 wave slots, the zero waves take the slots left). The chunk blocks of XCD x take one
    // contiguous run of chunks, whose context rows (a few cameras) then stay in that L2.
    const int ncg = (nchunk_blocks + 7) >> 3, nzg = (nzero_blocks + 7) >> 3;
    const int gi = blockIdx.x >> 3, x = blockIdx.x & 7;
    const int zgi = LSS_SPLAT_ZFIRST ? gi : gi - ncg, cgi = LSS_SPLAT_ZFIRST ? gi - nzg : gi;
    const bool zero_role = LSS_SPLAT_ZFIRST ? gi < nzg : gi >= ncg;
    if (!zero_role) {
        if (LSS_SPLAT_ROLES == 2) return;
        const int cb = x * ncg + cgi;
        if (cb >= nchunk_blocks) return;
        const int w = cb * kSplatWaves + wave;
        // the last chunk block's spare waves own no entries (and must not read the entry before their
        // base, past the end of sorted_key)
        if (w * kWave >= nprime) return;
        LSS_STAMP(w, 0);
        splat_chunk<FUSED, RT, OutT>(w, nprime, depth, rows_base, sorted_key, sorted_row, g, out, s_meta[wave],
                                     s_part[wave], lane);
        LSS_STAMP(w, 3);
#if LSS_TRACE
        if (lane == 0 && w < 16384) g_lss_trace[w][4] = ((unsigned long long)__builtin_amdgcn_s_getreg(20 | (31 << 11)) << 32) |
                                                    (unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11));
#endif
    } else {
        if (LSS_SPLAT_ROLES == 1) return;
        const int zb = x * nzg + zgi;
        if (zb >= nzero_blocks) return;
        const int u = (zb * kSplatWaves + wave) * zu;
        [[maybe_unused]] const int zslot = nchunk_blocks * kSplatWaves + zb * kSplatWaves + wave;
        LSS_STAMP(zslot, 0);
        if (u * kWave < g.ncells) zero_empty_rows<OutT>(u, zu, cell_start, g, out, lane);
        LSS_STAMP(zslot, 3);
#if LSS_TRACE
        if (lane == 0 && zslot < 16384) g_lss_trace[zslot][4] = ((unsigned long long)__builtin_amdgcn_s_getreg(20 | (31 << 11)) << 32) |
                                                        (unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11));
#endif
    }
}

// ---- NCHW (the reference layout), version 2: one block = one tile of YT consecutive cells of a BEV
// row (b, z, x, y0..y0 + YT), 4 waves = 4 * NG lane groups of LPR lanes (8 lanes x 16 B per context
// row for bf16 rows, the NHWC chunk's gather shape: 8 rows per wave instruction). The tile's cells are
// split over the groups at cell boundaries with the entries balanced; a group sums its cells one by one
// in canonical order (acc = fma(w, x, acc) entry by entry, the association of k_splat_fwd, so both
// kernels agree bit for bit), KU entries in flight per batch, and leaves each cell's row in an LDS
// tile [channel][y] zeroed beforehand (empty cells stay zero). The block then writes the tile one
// channel plane run at a time with 16-B stores.
constexpr int kN2Waves = 4;  // waves per NCHW tile block (more lane groups share a dense tile's entries)
// LDS row stride of the NCHW tile: YT rounded up to 16 B. At YT = 100 the tile is 25.6 KB, so 6 blocks
// fit a CU (1,536 of c2's 1,600 tiles resident at once instead of 1,280).
// (the round-2 stride YT + 4, 27 KB / 5 blocks per CU, was slower: c2 in-step 16.4 vs 15.3 us,
// profiles/r03/pad0_eval.txt)
__host__ __device__ constexpr int nchw2_stride(int yt) { return (yt + 3) & ~3; }
constexpr int kN2Block = kN2Waves * kWave;

template <bool FUSED, typename RT, typename OutT>
__global__ __launch_bounds__(kN2Block) void k_splat_fwd_nchw2(const float* __restrict__ depth,
                                                             const RT* __restrict__ rows_base,
                                                             const int32_t* __restrict__ cell_start,
                                                             const long long* __restrict__ sorted_key,
                                                             const int32_t* __restrict__ sorted_row, SplatGeo sg,
                                                             int ntiles, OutT* __restrict__ out) {
    using RS = RowSlice<RT>;
    constexpr int KU = 8;                         // context rows in flight per group and batch
    constexpr int KPL = (KU + RS::LPR - 1) / RS::LPR;  // keys fetched per lane per batch
    constexpr int NGB = kN2Waves * RS::NG;        // lane groups per block
    extern __shared__ __attribute__((aligned(16))) float lds[];
    __shared__ int s_start[kYtMax + 1];
    // consecutive tiles (one sample's rows) on one XCD, as the CSR build wrote them
    // (a tile's channels split over 2 / 4 blocks, for more lane groups per dense tile, was slower:
    // c2 20.5 / 32.9 vs 18.6 us, round 4)
    const int tile = xcd_block();
    if (tile >= ntiles) return;    // block-uniform (the grid is rounded up to a multiple of 8)
    const int bzx = tile / sg.ntiles_y;
    const int y0 = (tile - bzx * sg.ntiles_y) * sg.YT;
    const int ny = min(sg.YT, sg.Y - y0);
    const int x = bzx % sg.X, bz = bzx / sg.X;
    const int cell0 = bzx * sg.Y + y0;
    const int S = nchw2_stride(sg.YT);  // LDS row stride (floats; 16-B aligned rows)
    [[maybe_unused]] const int tslot = tile * kN2Waves + (threadIdx.x >> 6);  // LSS_TRACE builds only
    LSS_STAMP(tslot, 0);
    for (int i = threadIdx.x; i <= ny; i += kN2Block) s_start[i] = cell_start[cell0 + i];
    __syncthreads();
    LSS_STAMP(tslot, 1);
    const int s0 = s_start[0], s1 = s_start[ny];
    const bool empty = s0 == s1;
    if (!empty) {
        for (int i = threadIdx.x * 4; i < kC * S; i += kN2Block * 4)
            *reinterpret_cast<float4*>(lds + i) = make_float4(0.f, 0.f, 0.f, 0.f);
        const int lane = threadIdx.x & 63;
        const int wgrp = lane / RS::LPR;  // the lane's group inside the wave
        const int j = lane % RS::LPR, col = j * RS::EPL;
        // the group's cells [cb, ce): first cell whose start is >= the group's share of the entries.
        // lower_bound(t) over the non-decreasing s_start[0..ny] = the count of starts below t: two
        // ballots per target over the starts held one per lane (y <= 127; s_start[128] = s1 is never
        // below a target), no dependent LDS reads
        const int span = s1 - s0;
        const int sa = s_start[min(lane, ny)], sb = s_start[min(lane + kWave, ny)];
        const bool ina = lane <= ny, inb = lane + kWave <= ny;
        auto lower = [&](int t) {
            return __popcll(__ballot(ina && sa < t)) + __popcll(__ballot(inb && sb < t));
        };
        int cb = 0, ce = ny;
#pragma unroll
        for (int q = 0; q < RS::NG; ++q) {  // every lane runs every group's search (ballots are wave-wide)
            const int gq = (threadIdx.x >> 6) * RS::NG + q;
            const int lo = gq == 0 ? 0 : lower(s0 + (int)(((long)gq * span) / NGB));
            const int hi = gq == NGB - 1 ? ny : lower(s0 + (int)(((long)(gq + 1) * span) / NGB));
            if (q == wgrp) {
                cb = lo;
                ce = hi;
            }
        }
        const int eend = s_start[ce];
        float acc[RS::EPL];
#pragma unroll
        for (int i = 0; i < RS::EPL; ++i) acc[i] = 0.f;
        int cur = -1;
        auto flush = [&]() {
            float* dst = lds + (size_t)col * S + dchk(cur - cell0, ny, kDbgSplatCell);
#pragma unroll
            for (int i = 0; i < RS::EPL; ++i) dst[i * S] = acc[i];
        };
        const int gl0 = lane - j;  // the group's first lane
        // keys of a batch: lane j of the group holds entries e + j + LPR * t, t < KPL (clamped; the
        // clamped copies are never summed)
        long long kk[KPL];
        int rr[KPL];
        auto fetch_keys = [&](int e) {
#pragma unroll
            for (int t = 0; t < KPL; ++t) {
                const int ej = min(e + j + RS::LPR * t, eend - 1);
                kk[t] = sorted_key[ej];
                rr[t] = FUSED ? sorted_row[ej] : 0;
            }
        };
        int e = s_start[cb];
        if (e < eend) fetch_keys(e);  // in flight across the barrier
        __syncthreads();  // the tile is zeroed before any cell lands in it
        LSS_STAMP(tslot, 4);
        for (; e < eend; e += KU) {
            // this batch's depth weights and context-row slices (round trip 2), then the next batch's
            // keys (round trip 1 of the next batch, in flight behind them: no extra wait)
            float wt[KPL];
            int cc[KPL];
#pragma unroll
            for (int t = 0; t < KPL; ++t) {
                const int pt = dchk((int)(kk[t] & 0xFFFFFFFF), sg.nprime, kDbgSplatPoint);
                cc[t] = (int)(kk[t] >> 32);
                wt[t] = FUSED ? depth[pt] : 1.f;
                if (!FUSED) rr[t] = pt;
            }
            uint4 v[KU];
#pragma unroll
            for (int u = 0; u < KU; ++u) {
                const int r = dchk(__shfl(rr[u / RS::LPR], gl0 + u % RS::LPR, kWave), sg.nrows, kDbgSplatRow);
                v[u] = *reinterpret_cast<const uint4*>(rows_base + (size_t)r * kC + col);
            }
            if (e + KU < eend) fetch_keys(e + KU);
#pragma unroll
            for (int u = 0; u < KU; ++u) {
                const int c = __shfl(cc[u / RS::LPR], gl0 + u % RS::LPR, kWave);
                const float w = __shfl(wt[u / RS::LPR], gl0 + u % RS::LPR, kWave);
                if (e + u < eend) {
                    if (c != cur) {
                        if (cur >= 0) flush();
#pragma unroll
                        for (int i = 0; i < RS::EPL; ++i) acc[i] = 0.f;
                        cur = c;
                    }
                    float xv[RS::EPL];
                    unpack16(v[u], (const RT*)nullptr, xv);
#pragma unroll
                    for (int i = 0; i < RS::EPL; ++i) acc[i] = FUSED ? fmaf(w, xv[i], acc[i]) : __fadd_rn(acc[i], xv[i]);
                }
            }
        }
        if (cur >= 0) flush();
        __syncthreads();
    }
    LSS_STAMP(tslot, 2);
    // the tile, channel plane by channel plane: (B, Z*C, X, Y), channel z*C + c
    const size_t XY = (size_t)sg.X * sg.Y;
    OutT* obase = out + (size_t)bz * kC * XY + (size_t)x * sg.Y + y0;
    constexpr int VN = 16 / (int)sizeof(OutT);
    if ((sg.Y % VN) == 0 && (ny % VN) == 0 && (y0 % VN) == 0) {
        const int nq = ny / VN;
        for (int i = threadIdx.x; i < kC * nq; i += kN2Block) {
            const int c = i / nq, yv = (i - c * nq) * VN;
            float vals[VN];
#pragma unroll
            for (int t = 0; t < VN; t += 4) {
                const float4 f = empty ? make_float4(0.f, 0.f, 0.f, 0.f)
                                       : *reinterpret_cast<const float4*>(lds + (size_t)c * S + yv + t);
                vals[t] = f.x; vals[t + 1] = f.y; vals[t + 2] = f.z; vals[t + 3] = f.w;
            }
            store_vec(obase + c * XY + yv, vals);
        }
    } else {
        for (int i = threadIdx.x; i < kC * ny; i += kN2Block) {
            const int c = i / ny, yy = i - c * ny;
            obase[c * XY + yy] = from_f32<OutT>(empty ? 0.f : lds[(size_t)c * S + yy]);
        }
    }
    LSS_STAMP(tslot, 3);
}

// ----------------------------------------------------------------------------- backward
template <typename GT>
__global__ __launch_bounds__(kBlock) void k_bev_rows(const GT* __restrict__ dbev, const int32_t* __restrict__ cell_start,
                                                     SplatGeo sg, GT* __restrict__ rows) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    __shared__ int s_start[kYtMax + 1];
    const int tile = blockIdx.x;
    const int bzx = tile / sg.ntiles_y;
    const int y0 = (tile - bzx * sg.ntiles_y) * sg.YT;
    const int ny = min(sg.YT, sg.Y - y0);
    const int x = bzx % sg.X;
    const int bz = bzx / sg.X;
    const int cell0 = bzx * sg.Y + y0;
    // the tile's cell starts in one round trip (occupancy of every cell read from LDS below)
    for (int i = threadIdx.x; i <= ny; i += kBlock) s_start[i] = cell_start[cell0 + i];
    __syncthreads();
    if (s_start[0] == s_start[ny]) return;  // nothing pooled here (block-uniform)
    const int S = sg.YT + 1;  // odd stride: the row-gather reads (lane = channel) are conflict-free
    const size_t XY = (size_t)sg.X * sg.Y;
    const GT* gbase = dbev + (size_t)bz * kC * XY + (size_t)x * sg.Y + y0;
    constexpr int VN = 16 / (int)sizeof(GT);
    if ((sg.Y % VN) == 0 && (ny % VN) == 0 && (y0 % VN) == 0) {
        // 16-B loads, several in flight per thread before any LDS store
        const int nq = ny / VN, total = kC * nq;
        constexpr int kIt = 8;  // 64 x 100 cells: <= 7 loads per thread, all in flight
        for (int i0 = threadIdx.x; i0 < total; i0 += kBlock * kIt) {
            uint4 v[kIt];
#pragma unroll
            for (int t = 0; t < kIt; ++t) {
                const int i = min(i0 + t * kBlock, total - 1);
                const int c = i / nq, yv = (i - c * nq) * VN;
                v[t] = *reinterpret_cast<const uint4*>(gbase + c * XY + yv);
            }
#pragma unroll
            for (int t = 0; t < kIt; ++t) {
                const int i = i0 + t * kBlock;
                if (i < total) {
                    const int c = i / nq, yv = (i - c * nq) * VN;
                    float f[VN];
                    unpack16(v[t], (const GT*)nullptr, f);
#pragma unroll
                    for (int e = 0; e < VN; ++e) lds[c * S + yv + e] = f[e];
                }
            }
        }
    } else {
        for (int i = threadIdx.x; i < kC * ny; i += kBlock) {
            const int c = i / ny, yy = i - c * ny;
            lds[c * S + yy] = to_f32(gbase[c * XY + yy]);
        }
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int wave = uniform(threadIdx.x >> 6);
    for (int yy = wave; yy < ny; yy += kBlock / kWave) {
        if (s_start[yy + 1] > s_start[yy]) rows[(size_t)(cell0 + yy) * kC + lane] = from_f32<GT>(lds[lane * S + yy]);
    }
}

// Row index of cell k's gradient row: compact rows buffer, or the channels-last dbev itself
// (-1 stays -1). Integer divisions: computed once per point, before any gather.
template <bool NHWC>
__device__ __forceinline__ int grad_row(int cell, const SplatGeo& sg) {
    if (!NHWC || sg.Z == 1 || cell < 0) return cell;  // Z == 1: (b, xy) order is the cell order
    const int XY = sg.X * sg.Y;
    const int bz = cell / XY, xy = cell - bz * XY;
    const int b = bz / sg.Z, z = bz - b * sg.Z;
    return (b * XY + xy) * sg.Z + z;
}
template <bool NHWC>
__device__ __forceinline__ size_t row_offset(int cell, const SplatGeo& sg) {
    return (size_t)grad_row<NHWC>(cell, sg) * kC;
}

// One wave per pixel, registers only: lane (sub, j) holds rows r = k*RPI + sub, channels
// [EPL*j, EPL*j + EPL) of the pixel's D gradient rows, 64 rows (depth bins) per chunk, CH chunks
// (D <= 64 CH). d_ctx: per-lane sums over its rows of every chunk, then a butterfly over the RPI row
// groups; d_depth: per-row dot over the lane's channels, then a butterfly over the LPR lanes of the
// row; lane l keeps bin 64k + l of chunk k. Fixed association order (deterministic). The general form
// of the pixel-tile kernel below (any H*W, any D <= 64*CH).
template <typename GT, typename DT, typename CT, bool NHWC, int CH>
__global__ __launch_bounds__(kBlock) void k_splat_bwd_reg(const GT* __restrict__ g, const int32_t* __restrict__ cell_of,
                                                          const float* __restrict__ depth,
                                                          const CT* __restrict__ ctx_t, int D, int HW, int npix,
                                                          SplatGeo sg, DT* __restrict__ d_dn) {
    constexpr int EPL = 16 / sizeof(GT);    // row elements per 16-B lane load
    constexpr int LPR = kC / EPL;           // lanes per row
    constexpr int RPI = kWave / LPR;        // rows per wave-instruction
    constexpr int NI = kWave / RPI;         // instructions for 64 rows
    const int lane = threadIdx.x & 63;
    const int q = blockIdx.x * (kBlock / kWave) + uniform(threadIdx.x >> 6);
    if (q >= npix) return;  // wave-uniform
    const int bn = q / HW, hw = q - bn * HW;
    const size_t pbase = (size_t)bn * D * HW + hw;  // point (bn, d = 0, hw)
    const int sub = lane / LPR, col = (lane % LPR) * EPL;
    float cx[EPL];
#pragma unroll
    for (int e = 0; e < EPL; ++e) cx[e] = to_f32(ctx_t[(size_t)q * kC + col + e]);
    float dc[EPL];
#pragma unroll
    for (int e = 0; e < EPL; ++e) dc[e] = 0.f;
    float my_depth[CH], dd[CH];
#pragma unroll
    for (int ch = 0; ch < CH; ++ch) {
        const int d = ch * kWave + lane;
        const int dl_ = min(d, D - 1);  // clamped, unconditional loads (see keep_if)
        my_depth[ch] = keep_if(d < D, depth[pbase + (size_t)dl_ * HW]);
        int my_cell = cell_of[pbase + (size_t)dl_ * HW];
        my_cell = d < D ? grad_row<NHWC>(my_cell, sg) : -1;  // gradient row index (-1 stays -1)
        uint4 raw[NI];
#pragma unroll
        for (int k = 0; k < NI; ++k) {
            const int cell = __shfl(my_cell, (k * RPI + sub) & 63, kWave);  // -1 beyond D
            // rows past D (cell -1) read row 0 (one line for the whole instruction) and are zeroed
            raw[k] = keep_if(cell >= 0, *reinterpret_cast<const uint4*>(
                                            g + (size_t)dchk(max(cell, 0), sg.nrows, kDbgBwdRow) * kC + col));
        }
        float part[NI];
#pragma unroll
        for (int k = 0; k < NI; ++k) {
            const float w = __shfl(my_depth[ch], (k * RPI + sub) & 63, kWave);  // 0 beyond D
            float f[EPL];
            unpack16(raw[k], (const GT*)nullptr, f);
            float t = 0.f;
#pragma unroll
            for (int e = 0; e < EPL; ++e) {
                dc[e] = fmaf(f[e], w, dc[e]);
                t = fmaf(f[e], cx[e], t);
            }
            part[k] = t;
        }
        // d_depth of row k*RPI + sub: sum over the LPR lanes of the row
#pragma unroll
        for (int k = 0; k < NI; ++k)
#pragma unroll
            for (int o = 1; o < LPR; o <<= 1) part[k] += __shfl_xor(part[k], o, kWave);
        // lane l takes row l of the chunk: instruction l / RPI, held by the lanes of row group l % RPI
        float v_dd = 0.f;
#pragma unroll
        for (int k = 0; k < NI; ++k) {
            const float v = __shfl(part[k], (lane % RPI) * LPR, kWave);
            if (lane / RPI == k) v_dd = v;
        }
        dd[ch] = d < D ? v_dd : 0.f;
    }
    // d_ctx: sum over the RPI row groups (lanes j, j + LPR, j + 2 LPR, ...)
#pragma unroll
    for (int o = LPR; o < kWave; o <<= 1)
#pragma unroll
        for (int e = 0; e < EPL; ++e) dc[e] += __shfl_xor(dc[e], o, kWave);
    // softmax backward: dl = depth * (dd - sum_d depth * dd)
    float sd = 0.f;
#pragma unroll
    for (int ch = 0; ch < CH; ++ch) sd += my_depth[ch] * dd[ch];
    const float s = wave_sum(sd);
    DT* dst = d_dn + (size_t)bn * (D + kC) * HW + hw;
#pragma unroll
    for (int ch = 0; ch < CH; ++ch) {
        const int d = ch * kWave + lane;
        if (d < D) dst[(size_t)d * HW] = from_f32<DT>(my_depth[ch] * (dd[ch] - s));
    }
    if (sub == 0)
#pragma unroll
        for (int e = 0; e < EPL; ++e) dst[(size_t)(D + col + e) * HW] = from_f32<DT>(dc[e]);
}

// k_splat_bwd_tile shape for bf16 gradient rows, D <= 48 (experiment switches for build_variant)
#ifndef LSS_BWD_WAVES
#define LSS_BWD_WAVES 4  // round 6: 4 pixels per block, 8.6 vs 9.0-9.2 us in-step (profiles/r06/splat_bwd_shape_ab.txt)
#endif
#ifndef LSS_BWD_PPW
#define LSS_BWD_PPW 1
#endif
#ifndef LSS_BWD_MINW
#define LSS_BWD_MINW 5
#endif
#ifndef LSS_BWD_DPP
#define LSS_BWD_DPP 1  // experiment switch: 0 = the reductions as __shfl_xor butterflies (ds_bpermute)
#endif
constexpr int kBwdBigWaves = LSS_BWD_WAVES, kBwdBigPpw = LSS_BWD_PPW, kBwdBigMinW = LSS_BWD_MINW;

// Pixel-tile form of k_splat_bwd_reg. The per-pixel form reads the D depth weights and cells of its
// pixel at a stride of H*W (one cache line per value) and writes d_depthnet_out one element per
// channel (D + C lines per pixel, 2 bytes each). Here a block of WAVES waves takes PX = WAVES * PPW
// consecutive pixels (a tile may straddle two images): their weights, cells and context rows are
// read as contiguous runs into LDS; each wave takes PPW pixels, issues ALL their gradient-row gathers
// before any arithmetic (one round trip), reduces each as k_splat_bwd_reg does (fixed association),
// and leaves d_logits / d_ctx in an LDS tile that the block writes channel by channel in runs of RUN
// consecutive pixels of one image.
//
// Tile shape: 4 waves x 1 pixel (the product since round 6: with 71 VGPRs a CU holds 7 such blocks, 28
// waves, where it held 3 blocks of 8 -- 24 waves: in-step 8.60 / 8.64 vs 8.96-9.21 us on the same boxes;
// 4 x 1 at 6 or 8 waves per SIMD: 8.69 / 12.3 us, the VGPR cap spills; profiles/r06/splat_bwd_shape_ab.txt).
// Before: 8 waves x 1 pixel. A one-round shape -- 4 waves x 3 pixels, all of c3's
// 8,448 pixels resident at once (704 blocks for 768 slots) where 8 x 1 needs 1,056 blocks for 768
// -- measured no faster (in-step 9.7 vs 9.5 us with the DPP reductions, 11.8 vs 11.7 before them;
// profiles/r05/prof_ab_bwd_*): the per-pixel reduction, not the block rounds, was the long phase.
// Kept as the LSS_BWD_WAVES / LSS_BWD_PPW / LSS_BWD_MINW experiment switches.
template <typename GT, typename DT, typename CT, bool NHWC, int MAXD, int WAVES, int PPW, int MINW>
__global__ __launch_bounds__(WAVES * kWave) __attribute__((amdgpu_waves_per_eu(MINW))) void k_splat_bwd_tile(
    const GT* __restrict__ g, const int32_t* __restrict__ cell_of, const float* __restrict__ depth,
    const CT* __restrict__ ctx_t, int D, int HW, int npix, SplatGeo sg, DT* __restrict__ d_dn) {
    constexpr int kBwdBlock = WAVES * kWave;
    constexpr int EPL = 16 / sizeof(GT);  // row elements per 16-B lane load
    constexpr int LPR = kC / EPL;         // lanes per row
    constexpr int RPI = kWave / LPR;      // rows per wave-instruction
    constexpr int NI = MAXD / RPI;        // instructions for MAXD rows
    constexpr int PX = WAVES * PPW;       // pixels per block
    constexpr int kOE = 16 / (int)sizeof(DT);
    constexpr int RUN = PX % kOE == 0 ? kOE : 4;  // pixels per store: 16 B, or 4 pixels
    static_assert(PX % RUN == 0, "whole store runs per tile");
    static_assert(PPW * NI <= 32, "validity bits");
    __shared__ float s_dep[MAXD + 1][PX];  // + a spare row for the lanes past the end
    __shared__ int s_cell[MAXD + 1][PX];
    __shared__ float s_ctx[PX + 1][kC];  // + a spare tile for the lanes past the end
    __shared__ float s_out[MAXD + kC][PX + 1];
    const int q0 = xcd_block() * PX;
    if (q0 >= npix) return;  // block-uniform
    [[maybe_unused]] const int tslot = blockIdx.x * WAVES + (threadIdx.x >> 6);  // LSS_TRACE builds only
    LSS_STAMP(tslot, 0);
    // PX <= HW: the tile lies in image bn0 up to pixel jcut, in image bn0 + 1 after it
    const int bn0 = q0 / HW, hw0 = q0 - bn0 * HW, jcut = HW - hw0;
    // Every load below is unconditional (clamped index; an out-of-range value is dropped at the LDS
    // write or zeroed by a select), so the compiler issues them back to back: one round trip for the
    // staging, one for the gathers.
    constexpr int kCtx16 = PX * kC * (int)sizeof(CT) / 16;  // 16-B pieces of the tile's context rows
    constexpr int kCE = 16 / (int)sizeof(CT);
    static_assert(kCtx16 <= kBwdBlock, "one context piece per thread");
    const uint4 craw = reinterpret_cast<const uint4*>(ctx_t + (size_t)q0 * kC)[min((int)threadIdx.x, kCtx16 - 1)];
    constexpr int kStage = (MAXD * PX + kBwdBlock - 1) / kBwdBlock;
    float dv[kStage];
    int cv[kStage];
#pragma unroll
    for (int t = 0; t < kStage; ++t) {
        const int i = min((int)threadIdx.x + t * kBwdBlock, D * PX - 1);
        const int d = i / PX, j = i - d * PX;
        const size_t at = j < jcut ? ((size_t)bn0 * D + d) * HW + hw0 + j : ((size_t)(bn0 + 1) * D + d) * HW + (j - jcut);
        dv[t] = depth[at];
        cv[t] = cell_of[at];
    }
    __builtin_amdgcn_sched_barrier(0);  // every staging load issued before the first wait
#pragma unroll
    for (int t = 0; t < kStage; ++t) cv[t] = grad_row<NHWC>(cv[t], sg);  // gradient row index, or -1
    // LDS writes without branches either (a lane past the end writes the spare row MAXD)
#pragma unroll
    for (int t = 0; t < kStage; ++t) {
        const int i = min((int)threadIdx.x + t * kBwdBlock, MAXD * PX - 1);
        const int at = i < D * PX ? i : MAXD * PX + (i % PX);  // the spare row MAXD is never read
        s_dep[at / PX][at % PX] = dv[t];
        s_cell[at / PX][at % PX] = cv[t];
    }
    {
        float f[kCE];
        unpack16(craw, (const CT*)nullptr, f);
        const int e0 = min((int)threadIdx.x, kCtx16) * kCE;  // kCtx16: the spare tile s_ctx[PX]
#pragma unroll
        for (int e = 0; e < kCE; ++e) s_ctx[(e0 + e) / kC][(e0 + e) % kC] = f[e];
    }
    __syncthreads();
    LSS_STAMP(tslot, 1);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int sub = lane / LPR, col = (lane % LPR) * EPL;
    // all row indices from LDS first, then every gather back to back; validity as one packed word
    // (a mask register per gather held until its use cost one VGPR each)
    int rows[PPW][NI];
#pragma unroll
    for (int i = 0; i < PPW; ++i)
#pragma unroll
        for (int k = 0; k < NI; ++k) rows[i][k] = s_cell[min(k * RPI + sub, D - 1)][wave * PPW + i];
    __builtin_amdgcn_sched_barrier(0);
    uint4 raw[PPW][NI];
    unsigned vbits = 0;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
#pragma unroll
        for (int k = 0; k < NI; ++k) {
            // rows past D repeat row D - 1 (same line, no extra traffic); their values are zeroed
            const int row = rows[i][k];
            raw[i][k] = *reinterpret_cast<const uint4*>(g + (size_t)dchk(max(row, 0), sg.nrows, kDbgBwdRow) * kC + col);
            vbits |= (k * RPI + sub < D && row >= 0 ? 1u : 0u) << (i * NI + k);
        }
    }
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
        __builtin_amdgcn_sched_barrier(0);  // one pixel's reduction at a time (register pressure)
        const int jj = wave * PPW + i;
        const float my_depth = lane < D ? s_dep[lane][jj] : 0.f;
        float cx[EPL], dc[EPL], part[NI];
#pragma unroll
        for (int e = 0; e < EPL; ++e) {
            cx[e] = s_ctx[jj][col + e];
            dc[e] = 0.f;
        }
#pragma unroll
        for (int k = 0; k < NI; ++k) {
            const int r = k * RPI + sub;
            const float w = r < D ? s_dep[r][jj] : 0.f;
            float f[EPL];
            unpack16(keep_if((vbits >> (i * NI + k)) & 1u, raw[i][k]), (const GT*)nullptr, f);
            float t = 0.f;
#pragma unroll
            for (int e = 0; e < EPL; ++e) {
                dc[e] = fmaf(f[e], w, dc[e]);
                t = fmaf(f[e], cx[e], t);
            }
            part[k] = t;
        }
#if LSS_BWD_DPP
        // d_ctx over the RPI row groups, d_depth over the LPR lanes of a row (exact in lane 0 of each
        // row group, which the select below reads): DPP / permlane levels, the butterfly's association
#pragma unroll
        for (int e = 0; e < EPL; ++e) dc[e] = xsum_range<LPR, kWave / 2>(dc[e]);
#pragma unroll
        for (int k = 0; k < NI; ++k) part[k] = xsum_range<1, LPR / 2>(part[k]);
#else
#pragma unroll
        for (int o = LPR; o < kWave; o <<= 1)
#pragma unroll
            for (int e = 0; e < EPL; ++e) dc[e] += __shfl_xor(dc[e], o, kWave);
#pragma unroll
        for (int k = 0; k < NI; ++k)
#pragma unroll
            for (int o = 1; o < LPR; o <<= 1) part[k] += __shfl_xor(part[k], o, kWave);
#endif
        float dd = 0.f;
#pragma unroll
        for (int k = 0; k < NI; ++k) {
            const float v = __shfl(part[k], (lane % RPI) * LPR, kWave);
            if (lane / RPI == k) dd = v;
        }
        if (lane >= D) dd = 0.f;
#if LSS_BWD_DPP
        const float s = wave_sum_dpp(my_depth * dd);
#else
        const float s = wave_sum(my_depth * dd);
#endif
        if (lane < D) s_out[lane][jj] = my_depth * (dd - s);
        if (sub == 0)
#pragma unroll
            for (int e = 0; e < EPL; ++e) s_out[D + col + e][jj] = dc[e];
    }
    LSS_STAMP(tslot, 2);
    __syncthreads();
    // d_depthnet_out: runs of RUN consecutive pixels of one channel (HW % RUN == 0 and q0 % RUN == 0:
    // a run never straddles two images)
    constexpr int kRuns = PX / RUN;
    constexpr int kSt = ((MAXD + kC) * kRuns + kBwdBlock - 1) / kBwdBlock;
#pragma unroll
    for (int t = 0; t < kSt; ++t) {
        const int i = threadIdx.x + t * kBwdBlock;
        if (i < (D + kC) * kRuns) {
            const int ch = i / kRuns, j0 = (i - ch * kRuns) * RUN;
            const int bn = j0 < jcut ? bn0 : bn0 + 1, hw = j0 < jcut ? hw0 + j0 : j0 - jcut;
            DT v[RUN];
#pragma unroll
            for (int e = 0; e < RUN; ++e) v[e] = from_f32<DT>(s_out[ch][j0 + e]);
            DT* dst = d_dn + ((size_t)bn * (D + kC) + ch) * HW + hw;
            if constexpr (RUN * sizeof(DT) == 16) {
                uint4 u;
                __builtin_memcpy(&u, v, 16);
                *reinterpret_cast<uint4*>(dst) = u;
            } else {
                uint2 u;
                __builtin_memcpy(&u, v, 8);
                *reinterpret_cast<uint2*>(dst) = u;
            }
        }
    }
    LSS_STAMP(tslot, 3);
}

template <typename GT, bool NHWC>
__global__ __launch_bounds__(kBlock) void k_splat_bwd_lifted(const GT* __restrict__ g, const int32_t* __restrict__ cell_of,
                                                             int nprime, SplatGeo sg, float* __restrict__ dx) {
    const long i = (long)blockIdx.x * kBlock + threadIdx.x;
    const int p = (int)(i >> 4);
    if (p >= nprime) return;
    const int j = (int)(i & 15) * 4;
    const int cell = cell_of[p];
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (cell >= 0) {
        const GT* r = g + row_offset<NHWC>(cell, sg) + j;
        v = make_float4(to_f32(r[0]), to_f32(r[1]), to_f32(r[2]), to_f32(r[3]));
    }
    *reinterpret_cast<float4*>(dx + (size_t)p * kC + j) = v;
}

// ----------------------------------------------------------------------------- QuickCumsum operator boundary
// The reference's op-level interface (QuickCumsum / cumsum_trick, src/tools.py:182-219): rows x
// (n, C) already sorted by rank; one output row per run of equal ranks. The reference sums a run as
// the difference of two fp32-rounded prefix sums; here each run is summed directly, in row order, in
// fp32 (closer to the exact sum; the backward gather is identical).
__global__ __launch_bounds__(kBlock) void k_seg_flags(const long long* __restrict__ ranks, int n,
                                                      int32_t* __restrict__ flag) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i < n) flag[i] = (i == 0 || ranks[i] != ranks[i - 1]) ? 1 : 0;
}

// excl = exclusive scan of flag (excl[n] = number of runs): run id of row i and first row of each run.
__global__ __launch_bounds__(kBlock) void k_seg_finish(const int32_t* __restrict__ flag,
                                                       const int32_t* __restrict__ excl, int n,
                                                       int32_t* __restrict__ seg_of, int32_t* __restrict__ seg_start,
                                                       int32_t* __restrict__ nseg) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i < n) {
        const int f = flag[i], e = excl[i];
        seg_of[i] = e + f - 1;
        if (f) seg_start[e] = i;
    }
    if (i == 0) {
        const int t = excl[n];
        seg_start[t] = n;
        *nseg = t;
    }
}

// One wave per run: lane = channel (C in slices of 64), rows summed in order; key_out[j] = the
// keys (geom_feats) row of the run's LAST row, as geom_feats[kept] (src/tools.py:200).
__global__ __launch_bounds__(kBlock) void k_seg_sum(const float* __restrict__ x, int C,
                                                    const int32_t* __restrict__ seg_start, int nseg,
                                                    const long long* __restrict__ keys, int kw,
                                                    long long* __restrict__ key_out, float* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int w = blockIdx.x * (kBlock / kWave) + uniform(threadIdx.x >> 6);
    if (w >= nseg) return;
    const int s = seg_start[w], e = seg_start[w + 1];
    for (int c0 = 0; c0 < C; c0 += kWave) {
        const int c = c0 + lane;
        if (c < C) {
            float acc = 0.f;
            int r = s;
            for (; r + 4 <= e; r += 4) {  // four independent loads in flight, summed in order
                const float a = x[(size_t)r * C + c], b = x[(size_t)(r + 1) * C + c];
                const float d = x[(size_t)(r + 2) * C + c], f = x[(size_t)(r + 3) * C + c];
                acc = __fadd_rn(__fadd_rn(__fadd_rn(__fadd_rn(acc, a), b), d), f);
            }
            for (; r < e; ++r) acc = __fadd_rn(acc, x[(size_t)r * C + c]);
            out[(size_t)w * C + c] = acc;
        }
    }
    if (keys != nullptr)
        for (int k = lane; k < kw; k += kWave) key_out[(size_t)w * kw + k] = keys[(size_t)(e - 1) * kw + k];
}

// QuickCumsum.backward (src/tools.py:212-219): dx[i] = g[run of row i] -- a pure gather.
__global__ __launch_bounds__(kBlock) void k_seg_gather(const float* __restrict__ g, int C,
                                                       const int32_t* __restrict__ seg_of, long n_elems,
                                                       float* __restrict__ dx, int nseg) {
    const long i = (long)blockIdx.x * kBlock + threadIdx.x;
    if ((C & 3) == 0) {
        const long e = i * 4;
        if (e >= n_elems) return;
        const long r = e / C;
        const int c = (int)(e - r * C);
        *reinterpret_cast<float4*>(dx + e) = *reinterpret_cast<const float4*>(g + (size_t)dchk(seg_of[r], nseg, kDbgSegRun) * C + c);
    } else {
        if (i >= n_elems) return;
        const long r = i / C;
        dx[i] = g[(size_t)dchk(seg_of[r], nseg, kDbgSegRun) * C + (int)(i - r * C)];
    }
}

// ----------------------------------------------------------------------------- host helpers
inline int grid_blocks(long n, int per) { return (int)((n + per - 1) / per); }

// Compute units of the current device, cached per device id (the library's only global state).
inline int device_cus() {
    static std::atomic<int> cache[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    int n = cache[dev].load(std::memory_order_relaxed);
    if (n <= 0) {
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        cache[dev].store(n, std::memory_order_relaxed);
    }
    return n;
}

// Zero-fill units per zero wave of k_splat_fwd_nhwc: the fewest (<= kMaxZeroUnits) with which the chunk
// waves and the zero waves are all resident at once (kSplatMinWaves waves per SIMD, 4 SIMDs per CU);
// 1 when no choice fits.
inline int splat_zero_units(long chunk_waves, long units) {
    if (LSS_SPLAT_ZU > 0) return std::min(LSS_SPLAT_ZU, kMaxZeroUnits);
    const long slots = (long)device_cus() * 4 * kSplatMinWaves;
    for (int zu = 1; zu <= kMaxZeroUnits; ++zu)
        if (chunk_waves + grid_blocks(grid_blocks(units, zu), kSplatWaves) * (long)kSplatWaves <= slots) return zu;
    return 1;
}

inline int choose_yt(int Y) {
    if (Y <= kYtMax) return Y;
    for (int t = kYtMax; t >= 16; t -= 4)
        if (Y % t == 0) return t;
    return kYtMax;
}

// nrows: rows of the feature / gradient buffer the kernel gathers from (0: the dims' pixels)
inline SplatGeo splat_geo(const lss_grid_t* g, const lss_dims_t* d, long nrows = 0) {
    SplatGeo s;
    s.X = g->nx[0];
    s.Y = g->nx[1];
    s.Z = g->nx[2];
    s.YT = choose_yt(s.Y);
    s.ntiles_y = (s.Y + s.YT - 1) / s.YT;
    const long pix = (long)d->B * d->N * d->H * d->W;
    s.ncells = (int)std::min<long>((long)d->B * s.Z * s.X * s.Y, INT_MAX);
    s.nprime = (int)std::min<long>(pix * d->D, INT_MAX);
    s.nrows = (int)std::min<long>(nrows > 0 ? nrows : pix, INT_MAX);
    return s;
}

inline int launch_status() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

// LSS_DEBUG builds: the CSR invariants after every build (k_debug_csr); nothing in release builds.
inline void debug_check_csr(const int32_t* cell_start, int ncells, const int32_t* cell_of, int nprime, hipStream_t s) {
    if (!LSS_DEBUG) return;
    hipLaunchKernelGGL(k_debug_csr, dim3(grid_blocks(std::max(ncells + 1, nprime), kBlock)), dim3(kBlock), 0, s,
                       cell_start, ncells, cell_of, nprime);
}

inline bool dims_ok(const lss_dims_t* d) {
    return d && d->B > 0 && d->N > 0 && d->D > 0 && d->H > 0 && d->W > 0 && d->C == kC;
}

inline bool grid_ok(const lss_grid_t* g) {
    return g && g->nx[0] > 0 && g->nx[1] > 0 && g->nx[2] > 0 && g->dx[0] > 0.f && g->dx[1] > 0.f && g->dx[2] > 0.f;
}

// The empty-row fill that rides along a lift launch: channels-last BEV geometry and the number of
// 8-block fill groups. bev == nullptr: no fill (0 groups).
}  // namespace

// ============================================================================= C ABI
extern "C" {

int lss_abi_version(void) { return LSS_ABI_VERSION; }

#if LSS_TRACE
// Diagnostics builds only (not in lss_hip.h): copy the per-wave stamps of the last splat to the host.
int lss_debug_trace(unsigned long long* host, int nrows) {
    if (nrows > 16384) nrows = 16384;
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_lss_trace), sizeof(unsigned long long) * 5 * nrows, 0,
                                    hipMemcpyDeviceToHost);
}
int lss_debug_trace_clear(void) {
    static unsigned long long zeros[16384][5];
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_lss_trace), zeros, sizeof(zeros), 0, hipMemcpyHostToDevice);
}
#endif

int lss_event_create(lss_event_t* ev) {
    if (!ev) return LSS_EINVAL;
    hipEvent_t e;
    const hipError_t r = hipEventCreate(&e);
    *ev = (lss_event_t)e;
    return (int)r;
}

int lss_event_destroy(lss_event_t ev) { return ev ? (int)hipEventDestroy((hipEvent_t)ev) : LSS_EINVAL; }

int lss_event_elapsed_ms(lss_event_t start, lss_event_t stop, float* ms) {
    if (!start || !stop || !ms) return LSS_EINVAL;
    hipError_t r = hipEventSynchronize((hipEvent_t)stop);
    if (r != hipSuccess) return (int)r;
    return (int)hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop);
}

int lss_event_record(lss_event_t ev, lss_stream_t stream) {
    if (!ev) return LSS_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    unsigned long long id = 0;
    hipGraph_t graph = nullptr;
    const hipGraphNode_t* deps = nullptr;
    size_t ndeps = 0;
    hipError_t r = hipStreamGetCaptureInfo_v2(s, &st, &id, &graph, &deps, &ndeps);
    if (r != hipSuccess) return (int)r;
    if (st != hipStreamCaptureStatusActive) return (int)hipEventRecord((hipEvent_t)ev, s);
    hipGraphNode_t node;
    r = hipGraphAddEventRecordNode(&node, graph, deps, ndeps, (hipEvent_t)ev);
    if (r != hipSuccess) return (int)r;
    return (int)hipStreamUpdateCaptureDependencies(s, &node, 1, hipStreamSetCaptureDependencies);
}

const char* lss_error_string(int code) {
    if (code == 0) return "success";
    if (code == LSS_EINVAL) return "lss: invalid argument";
    if (code == LSS_EUNSUPPORTED) return "lss: unsupported configuration (see include/lss_hip.h: C == 64, D <= 256; fused depthnet D + C <= 128)";
    if (code > 0) return hipGetErrorString((hipError_t)code);
    return "lss: unknown error";
}

int lss_geometry_cells(const float* frustum, const float* rots, const float* trans, const float* kinv,
                       const float* pinv, const float* post_trans, const lss_dims_t* dims, const lss_grid_t* grid,
                       float* out_geom, int32_t* cell_of, int32_t* cell_count, int32_t* slot_of,
                       lss_stream_t stream) {
    if (!dims_ok(dims) || !grid_ok(grid) || !frustum || !rots || !trans || !kinv || !pinv || !post_trans || !cell_of)
        return LSS_EINVAL;
    if (cell_count && !slot_of) return LSS_EINVAL;
    const long DHW = (long)dims->D * dims->H * dims->W;
    const long nprime = (long)dims->B * dims->N * DHW;
    if (nprime >= INT_MAX) return LSS_EUNSUPPORTED;
    hipLaunchKernelGGL(k_geometry_cells, dim3(grid_blocks(nprime, kGeoBlock)), dim3(kGeoBlock), 0,
                       (hipStream_t)stream, frustum, rots, trans, kinv, pinv, post_trans, dims->N, (int)DHW,
                       (int)nprime, *grid, out_geom, cell_of, cell_count, slot_of);
    return launch_status();
}

int lss_cells_from_geom(const float* geom, int32_t nprime, int32_t points_per_batch, const lss_grid_t* grid,
                        int32_t* cell_of, int32_t* cell_count, int32_t* slot_of, lss_stream_t stream) {
    if (!geom || !cell_of || nprime <= 0 || points_per_batch <= 0 || !grid_ok(grid)) return LSS_EINVAL;
    if (cell_count && !slot_of) return LSS_EINVAL;
    hipLaunchKernelGGL(k_cells_from_geom, dim3(grid_blocks(nprime, kGeoBlock)), dim3(kGeoBlock), 0, (hipStream_t)stream,
                       geom, nprime, points_per_batch, *grid, cell_of, cell_count, slot_of);
    return launch_status();
}

size_t lss_csr_scratch_bytes(int32_t ncells, int32_t nprime) {
    const size_t partial = sizeof(int32_t) * (size_t)((ncells + kScanItems - 1) / kScanItems + 1);
    return ((partial + 255) & ~(size_t)255) + sizeof(long long) * (size_t)nprime;
}

int lss_csr_build(const int32_t* cell_of, const int32_t* slot_of, int32_t nprime, const int32_t* cell_count,
                  int32_t ncells, const lss_dims_t* dims, int32_t* cell_start, long long* sorted_key,
                  int32_t* sorted_row, void* scratch, lss_stream_t stream) {
    if (!cell_of || !slot_of || !cell_count || !cell_start || !sorted_key || !sorted_row || !scratch || nprime <= 0 ||
        ncells <= 0)
        return LSS_EINVAL;
    int DHW = nprime, HW = nprime;  // no dims: the row of point p is p (per-point rows)
    if (dims != nullptr) {
        if (!dims_ok(dims)) return LSS_EINVAL;
        DHW = dims->D * dims->H * dims->W;
        HW = dims->H * dims->W;
        if ((long)dims->B * dims->N * DHW != nprime) return LSS_EINVAL;
    }
    const int nb = (ncells + kScanItems - 1) / kScanItems;
    int32_t* partial = static_cast<int32_t*>(scratch);
    const size_t poff = ((sizeof(int32_t) * (size_t)(nb + 1)) + 255) & ~(size_t)255;
    long long* tmp_key = reinterpret_cast<long long*>(static_cast<char*>(scratch) + poff);
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(k_scan_partials, dim3(nb), dim3(1024), 0, s, cell_count, ncells, partial);
    hipLaunchKernelGGL(k_scan_apply, dim3(xcd_grid(nb)), dim3(1024), 0, s, cell_count, ncells, partial, cell_start);
    hipLaunchKernelGGL(k_scatter, dim3(grid_blocks(nprime, kBlock)), dim3(kBlock), 0, s, cell_of, slot_of, nprime,
                       cell_start, tmp_key);
    const int nchunks = (nprime + kWave - 1) / kWave;
    hipLaunchKernelGGL(k_csr_canon, dim3(xcd_grid(grid_blocks(nchunks, kBlock / kWave))), dim3(kBlock), 0, s, tmp_key,
                       cell_start + ncells, nchunks, nprime, DHW, HW, sorted_key, sorted_row);
    debug_check_csr(cell_start, ncells, cell_of, nprime, s);
    return launch_status();
}

size_t lss_csr_workspace_bytes(int32_t ncells) {
    const size_t nb = (size_t)((ncells + kScanItems - 1) / kScanItems);
    return sizeof(ScanWs) + sizeof(unsigned long long) * nb;  // header, look-back granules
}

int lss_csr_build_ws(const int32_t* cell_of, const int32_t* slot_of, int32_t nprime, int32_t* cell_count,
                     int32_t ncells, const lss_dims_t* dims, int32_t* cell_start, long long* sorted_key,
                     int32_t* sorted_row, void* scratch, void* workspace, lss_stream_t stream) {
    if (!cell_of || !slot_of || !cell_count || !cell_start || !sorted_key || !sorted_row || !scratch || !workspace ||
        nprime <= 0 || ncells <= 0)
        return LSS_EINVAL;
    int DHW = nprime, HW = nprime;  // no dims: the row of point p is p (per-point rows)
    if (dims != nullptr) {
        if (!dims_ok(dims)) return LSS_EINVAL;
        DHW = dims->D * dims->H * dims->W;
        HW = dims->H * dims->W;
        if ((long)dims->B * dims->N * DHW != nprime) return LSS_EINVAL;
    }
    const int nb = (ncells + kScanItems - 1) / kScanItems;
    const size_t poff = ((sizeof(int32_t) * (size_t)(nb + 1)) + 255) & ~(size_t)255;  // as lss_csr_build
    long long* tmp_key = reinterpret_cast<long long*>(static_cast<char*>(scratch) + poff);
    ScanWs* ws = static_cast<ScanWs*>(workspace);
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(k_scan_lookback, dim3(nb), dim3(1024), 0, s, cell_count, ncells, ws, cell_start, -1);
    hipLaunchKernelGGL(k_scatter_ws, dim3(grid_blocks(std::max(nprime, ncells), kBlock)), dim3(kBlock), 0, s, cell_of,
                       slot_of, nprime, cell_start, tmp_key, cell_count, ncells, ws);
    const int nchunks = (nprime + kWave - 1) / kWave;
    hipLaunchKernelGGL(k_csr_canon, dim3(xcd_grid(grid_blocks(nchunks, kBlock / kWave))), dim3(kBlock), 0, s, tmp_key,
                       cell_start + ncells, nchunks, nprime, DHW, HW, sorted_key, sorted_row);
    debug_check_csr(cell_start, ncells, cell_of, nprime, s);
    return launch_status();
}

// ---- ordered plans (ABI 22)
// lists buffer: [ncells * kOrdList int32 records][nprime int2 overflow records], 16-B aligned parts
static size_t ord_list_bytes(int32_t ncells) {
    return ((sizeof(int32_t) * (size_t)ncells * kOrdList) + 255) & ~(size_t)255;
}
size_t lss_csr_lists_bytes(int32_t ncells, int32_t nprime) {
    if (ncells <= 0 || nprime <= 0) return 0;
    return ord_list_bytes(ncells) + sizeof(int2) * (size_t)nprime;
}
// points of one sample (the most a cell can hold) and blocks per sample must fit the cell word's fields
static bool ord_fits(long ppb) { return ppb > 0 && ppb < (1L << kOrdCountBits) - 2L * kGeoBlock; }

int lss_geometry_cells_ordered(const float* frustum, const float* rots, const float* trans, const float* kinv,
                               const float* pinv, const float* post_trans, const lss_dims_t* dims,
                               const lss_grid_t* grid, float* out_geom, int32_t* cell_of, int32_t* cell_word,
                               int32_t* rank_of, void* lists, void* workspace, lss_stream_t stream) {
    if (!dims_ok(dims) || !grid_ok(grid) || !frustum || !rots || !trans || !kinv || !pinv || !post_trans || !cell_of ||
        !cell_word || !rank_of || !lists || !workspace || (reinterpret_cast<uintptr_t>(lists) & 15))
        return LSS_EINVAL;
    const long DHW = (long)dims->D * dims->H * dims->W;
    const long nprime = (long)dims->B * dims->N * DHW;
    if (nprime >= INT_MAX || !ord_fits((long)dims->N * DHW)) return LSS_EUNSUPPORTED;
    const int ncells = grid->nx[0] * grid->nx[1] * grid->nx[2] * dims->B;
    int32_t* list = static_cast<int32_t*>(lists);
    int2* ovf = reinterpret_cast<int2*>(static_cast<char*>(lists) + ord_list_bytes(ncells));
    hipLaunchKernelGGL(k_geometry_cells_ord, dim3(xcd_grid(grid_blocks(nprime, kGeoBlock))), dim3(kGeoBlock), 0,
                       (hipStream_t)stream, frustum, rots, trans, kinv, pinv, post_trans, dims->N, (int)DHW,
                       (int)nprime, *grid, out_geom, cell_of, cell_word, rank_of, list, ovf,
                       &static_cast<ScanWs*>(workspace)->ovf_count);
    return launch_status();
}

int lss_cells_from_geom_ordered(const float* geom, int32_t nprime, int32_t points_per_batch, const lss_grid_t* grid,
                                int32_t* cell_of, int32_t* cell_word, int32_t* rank_of, void* lists,
                                void* workspace, lss_stream_t stream) {
    if (!geom || !cell_of || !cell_word || !rank_of || !lists || !workspace || nprime <= 0 || points_per_batch <= 0 ||
        !grid_ok(grid) || (reinterpret_cast<uintptr_t>(lists) & 15) || nprime % points_per_batch != 0)
        return LSS_EINVAL;
    if (!ord_fits(points_per_batch)) return LSS_EUNSUPPORTED;
    const int ncells = grid->nx[0] * grid->nx[1] * grid->nx[2] * (nprime / points_per_batch);
    int32_t* list = static_cast<int32_t*>(lists);
    int2* ovf = reinterpret_cast<int2*>(static_cast<char*>(lists) + ord_list_bytes(ncells));
    hipLaunchKernelGGL(k_cells_from_geom_ord, dim3(xcd_grid(grid_blocks(nprime, kGeoBlock))), dim3(kGeoBlock), 0,
                       (hipStream_t)stream, geom, nprime, points_per_batch, *grid, cell_of, cell_word, rank_of, list,
                       ovf, &static_cast<ScanWs*>(workspace)->ovf_count);
    return launch_status();
}

int lss_csr_build_ordered(const int32_t* cell_of, const int32_t* rank_of, int32_t nprime, int32_t* cell_word,
                          int32_t ncells, const lss_dims_t* dims, const void* lists, int32_t* cell_start,
                          long long* sorted_key, int32_t* sorted_row, void* workspace, lss_stream_t stream) {
    if (!cell_of || !rank_of || !cell_word || !lists || !cell_start || !sorted_key || !sorted_row || !workspace ||
        nprime <= 0 || ncells <= 0 || (reinterpret_cast<uintptr_t>(lists) & 15))
        return LSS_EINVAL;
    int DHW = nprime, HW = nprime;  // no dims: the row of point p is p (per-point rows)
    if (dims != nullptr) {
        if (!dims_ok(dims)) return LSS_EINVAL;
        DHW = dims->D * dims->H * dims->W;
        HW = dims->H * dims->W;
        if ((long)dims->B * dims->N * DHW != nprime) return LSS_EINVAL;
    }
    const int nb = (ncells + kScanItems - 1) / kScanItems;
    ScanWs* ws = static_cast<ScanWs*>(workspace);
    const int32_t* list = static_cast<const int32_t*>(lists);
    const int2* ovf = reinterpret_cast<const int2*>(static_cast<const char*>(lists) + ord_list_bytes(ncells));
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(k_scan_lookback, dim3(nb), dim3(1024), 0, s, cell_word, ncells, ws, cell_start, kOrdCountMask);
    hipLaunchKernelGGL(k_scatter_ord, dim3(xcd_grid(grid_blocks(std::max(nprime, ncells), kBlock))), dim3(kBlock), 0, s,
                       cell_of, rank_of, nprime, cell_start, list, ovf, DHW, HW, sorted_key, sorted_row, cell_word,
                       ncells, ws);
    debug_check_csr(cell_start, ncells, cell_of, nprime, s);
    return launch_status();
}

int lss_debug_checks(void) { return LSS_DEBUG ? 1 : 0; }

int lss_debug_status(int32_t* out4, int32_t clear) {
    if (!out4) return LSS_EINVAL;
    hipError_t r = hipMemcpyFromSymbol(out4, HIP_SYMBOL(g_lss_dbg), sizeof(int32_t) * 4, 0, hipMemcpyDeviceToHost);
    if (r != hipSuccess) return (int)r;
    if (clear) {
        static const int32_t zeros[4] = {0, 0, 0, 0};
        r = hipMemcpyToSymbol(HIP_SYMBOL(g_lss_dbg), zeros, sizeof(zeros), 0, hipMemcpyHostToDevice);
    }
    return (int)r;
}

int lss_lift_prep(const void* depthnet_out, int32_t in_dtype, const lss_dims_t* dims, float* depth, void* ctx_t,
                  int32_t ctx_dtype, lss_stream_t stream) {
    if (!dims_ok(dims) || !depthnet_out || !depth || !ctx_t) return LSS_EINVAL;
    if (dims->D > 256) return LSS_EUNSUPPORTED;
    const int HW = dims->H * dims->W;
    const int npix = dims->B * dims->N * HW;
    const dim3 grid(xcd_grid(grid_blocks(npix, 64))), block(kBlock);
    hipStream_t s = (hipStream_t)stream;
    // depth bins per wave part: 16 (D <= 64, the reference's D = 41), 32, 64
#define LSS_PREP_NI(IT, CT, NI)                                                                                    \
    hipLaunchKernelGGL((k_lift_prep<IT, CT, NI>), grid, block, 0, s, (const IT*)depthnet_out, dims->D, HW, npix,  \
                       depth, (CT*)ctx_t)
#define LSS_PREP(IT, CT)                                                                                           \
    do {                                                                                                           \
        if (dims->D <= 64) LSS_PREP_NI(IT, CT, 16);                                                                \
        else if (dims->D <= 128) LSS_PREP_NI(IT, CT, 32);                                                          \
        else LSS_PREP_NI(IT, CT, 64);                                                                              \
    } while (0)
    if (in_dtype == LSS_F32 && ctx_dtype == LSS_F32) LSS_PREP(float, float);
    else if (in_dtype == LSS_F32 && ctx_dtype == LSS_BF16) LSS_PREP(float, bf16);
    else if (in_dtype == LSS_BF16 && ctx_dtype == LSS_F32) LSS_PREP(bf16, float);
    else if (in_dtype == LSS_BF16 && ctx_dtype == LSS_BF16) LSS_PREP(bf16, bf16);
    else return LSS_EINVAL;
#undef LSS_PREP
#undef LSS_PREP_NI
    return launch_status();
}

int lss_depthnet_lift(const void* feat, const void* weight, const void* bias, int32_t dtype, int32_t K,
                      const lss_dims_t* dims, float* depth, void* ctx_t, int32_t ctx_dtype, lss_stream_t stream) {
    if (!dims_ok(dims) || !feat || !weight || !bias || !depth || !ctx_t) return LSS_EINVAL;
    if (dtype != LSS_BF16 || ctx_dtype != LSS_BF16) return LSS_EUNSUPPORTED;
    if (K <= 0 || K % 16 != 0 || K > kDnMaxK || dims->D + kC > kDnMaxO) return LSS_EUNSUPPORTED;
    const int HW = dims->H * dims->W;
    const long npix = (long)dims->B * dims->N * HW;
    if (npix >= INT_MAX) return LSS_EUNSUPPORTED;
    hipStream_t s = (hipStream_t)stream;
    if (K == 512 && HW % 8 == 0) {  // up1's 512 channels: k_depthnet_lift2, one block per CU (its LDS)
        hipLaunchKernelGGL((k_depthnet_lift2<512, kDn2Pix>), dim3(xcd_grid(grid_blocks(npix, kDn2Pix))),
                           dim3(kDn2Block), 0, s, (const bf16*)feat, (const bf16*)weight, (const bf16*)bias, dims->D,
                           HW, (int)npix, depth, (bf16*)ctx_t);
        return launch_status();
    }
    hipLaunchKernelGGL(k_depthnet_lift, dim3(xcd_grid(grid_blocks(npix, kDnPix))), dim3(kBlock), 0, s,
                       (const bf16*)feat, (const bf16*)weight, (const bf16*)bias, K, dims->D, HW, (int)npix, depth,
                       (bf16*)ctx_t);
    return launch_status();
}

static int depthnet_lift_nhwc(const void* feat, const void* weight, bool packed, const void* bias, int32_t dtype,
                              int32_t K, const lss_dims_t* dims, float* depth, void* ctx_t, int32_t ctx_dtype,
                              lss_stream_t stream) {
    if (!dims_ok(dims) || !feat || !weight || !bias || !depth || !ctx_t) return LSS_EINVAL;
    if (((uintptr_t)feat | (uintptr_t)weight) & 15) return LSS_EINVAL;  // 16-B vector loads of the rows
    if (dtype != LSS_BF16 || ctx_dtype != LSS_BF16) return LSS_EUNSUPPORTED;
    if (K != 512 || dims->D + kC > kDnMaxO) return LSS_EUNSUPPORTED;
    const int HW = dims->H * dims->W;
    const long npix = (long)dims->B * dims->N * HW;
    if (npix >= INT_MAX / 2) return LSS_EUNSUPPORTED;
    // one block per CU, more only when a CU's share would pass kDn3MaxPix pixels; never more than
    // the pixels (every block holds at least one)
    const long nlift = std::min<long>(npix, std::max<long>((long)LSS_DN3_BPC * device_cus(),
                                                           (npix + kDn3MaxPix - 1) / kDn3MaxPix));
    hipStream_t s = (hipStream_t)stream;
    if (packed)
        hipLaunchKernelGGL((k_depthnet_lift3<512, true>), dim3(xcd_grid(nlift)), dim3(kDn3Block), 0, s, (const bf16*)feat,
                           (const bf16*)weight, (const bf16*)bias, dims->D, HW, (int)npix, (int)nlift, depth,
                           (bf16*)ctx_t);
    else
        hipLaunchKernelGGL((k_depthnet_lift3<512, false>), dim3(xcd_grid(nlift)), dim3(kDn3Block), 0, s, (const bf16*)feat,
                           (const bf16*)weight, (const bf16*)bias, dims->D, HW, (int)npix, (int)nlift, depth,
                           (bf16*)ctx_t);
    return launch_status();
}

int lss_depthnet_lift_nhwc(const void* feat, const void* weight, const void* bias, int32_t dtype, int32_t K,
                           const lss_dims_t* dims, float* depth, void* ctx_t, int32_t ctx_dtype, lss_stream_t stream) {
    return depthnet_lift_nhwc(feat, weight, false, bias, dtype, K, dims, depth, ctx_t, ctx_dtype, stream);
}

int lss_depthnet_lift_nhwc_packed(const void* feat, const void* packed, const void* bias, int32_t K,
                                  const lss_dims_t* dims, float* depth, void* ctx_t, int32_t ctx_dtype,
                                  lss_stream_t stream) {
    return depthnet_lift_nhwc(feat, packed, true, bias, LSS_BF16, K, dims, depth, ctx_t, ctx_dtype, stream);
}

int lss_depthnet_pack(const void* weight, const void* bias, int32_t dtype, int32_t O, int32_t K, void* packed,
                      void* plain, void* bias_out, lss_stream_t stream) {
    if (!weight || !packed || (bias_out && !bias)) return LSS_EINVAL;
    if (((uintptr_t)packed | (uintptr_t)plain) & 15) return LSS_EINVAL;
    if (K <= 0 || K % 32 != 0 || K > kDnMaxK || O <= 0 || O > kDn3Waves * 16) return LSS_EUNSUPPORTED;
    const int n = std::max(kDn3Waves * (K / 32) * kWave, (int)O);
    hipStream_t s = (hipStream_t)stream;
    if (dtype == LSS_F32)
        hipLaunchKernelGGL(k_depthnet_pack<float>, dim3(grid_blocks(n, kBlock)), dim3(kBlock), 0, s, (const float*)weight,
                           (const float*)bias, (int)O, (int)K, (bf16*)packed, (bf16*)plain, (bf16*)bias_out);
    else if (dtype == LSS_BF16)
        hipLaunchKernelGGL(k_depthnet_pack<bf16>, dim3(grid_blocks(n, kBlock)), dim3(kBlock), 0, s, (const bf16*)weight,
                           (const bf16*)bias, (int)O, (int)K, (bf16*)packed, (bf16*)plain, (bf16*)bias_out);
    else
        return LSS_EINVAL;
    return launch_status();
}

int lss_flat_cast_bf16(const float* src, void* dst, int64_t n, const float* dn_weight, int32_t O, int32_t K,
                       void* packed, lss_stream_t stream) {
    if (!src || !dst || n < 0 || (((uintptr_t)src | (uintptr_t)dst) & 15)) return LSS_EINVAL;
    if (packed && (!dn_weight || ((uintptr_t)packed & 15))) return LSS_EINVAL;
    if (packed && (K <= 0 || K % 32 != 0 || K > kDnMaxK || O <= 0 || O > kDn3Waves * 16)) return LSS_EUNSUPPORTED;
    const long ncast_l = (n + 16L * kBlock - 1) / (16L * kBlock);
    if (ncast_l >= INT_MAX / 2) return LSS_EUNSUPPORTED;
    const int ncast = (int)ncast_l;
    const int npack = packed ? grid_blocks(kDn3Waves * (K / 32) * kWave, kBlock) : 0;
    if (ncast + npack == 0) return 0;
    hipLaunchKernelGGL(k_flat_cast_bf16, dim3(ncast + npack), dim3(kBlock), 0, (hipStream_t)stream, src, (bf16*)dst,
                       (long)n, npack, dn_weight, (int)O, (int)K, (bf16*)packed);
    return launch_status();
}

int lss_splat_fwd(const float* depth, const void* ctx_t, int32_t ctx_dtype, const float* x_rows,
                  const int32_t* cell_start, const long long* sorted_key, const int32_t* sorted_row,
                  const lss_dims_t* dims, const lss_grid_t* grid, void* out, int32_t out_dtype, int32_t out_layout,
                  lss_stream_t stream, lss_event_t ev_start, lss_event_t ev_stop) {
    hipEvent_t e0 = (hipEvent_t)ev_start, e1 = (hipEvent_t)ev_stop;
    if (!dims_ok(dims) || !grid_ok(grid) || !cell_start || !sorted_key || !out) return LSS_EINVAL;
    const bool fused = x_rows == nullptr;
    if (fused && (!depth || !ctx_t || !sorted_row)) return LSS_EINVAL;
    if (fused && ctx_dtype != LSS_F32 && ctx_dtype != LSS_BF16) return LSS_EINVAL;
    if (out_dtype != LSS_F32 && out_dtype != LSS_BF16) return LSS_EINVAL;
    if (out_layout != LSS_NCHW && out_layout != LSS_NHWC) return LSS_EINVAL;
    const long nprime_l = (long)dims->B * dims->N * dims->D * dims->H * dims->W;
    if (nprime_l >= INT_MAX - 2 * kWave) return LSS_EUNSUPPORTED;
    const int nprime = (int)nprime_l;
    const SplatGeo sg = splat_geo(grid, dims, fused ? 0 : nprime_l);  // lifted mode: one row per point
    const bool ctx_bf16 = fused && ctx_dtype == LSS_BF16;
    const void* rows = fused ? ctx_t : (const void*)x_rows;
    hipStream_t s = (hipStream_t)stream;
    if (out_layout == LSS_NHWC) {
        BevGeo g;
        g.X = sg.X; g.Y = sg.Y; g.Z = sg.Z;
        g.ncells = dims->B * sg.Z * sg.X * sg.Y;
        g.nrows = sg.nrows;
        const int nchunks = grid_blocks(nprime, kWave);
        const int nchunk_blocks = grid_blocks(nchunks, kSplatWaves);
        const int zu = splat_zero_units(nchunk_blocks * kSplatWaves, grid_blocks(g.ncells, kWave));
        const int nzero_blocks = grid_blocks(grid_blocks(grid_blocks(g.ncells, kWave), zu), kSplatWaves);
        const dim3 gr(8 * (grid_blocks(nchunk_blocks, 8) + grid_blocks(nzero_blocks, 8))), bl(kSplatBlock);
// kernel-stamped events only when asked for: a plain launch is what a hipGraph capture records
#define LSS_NHWC_FWD(F, RT, T)                                                                                     \
    do {                                                                                                           \
        if (e0 || e1)                                                                                              \
            hipExtLaunchKernelGGL((k_splat_fwd_nhwc<F, RT, T>), gr, bl, 0, s, e0, e1, 0, depth, (const RT*)rows,   \
                                  cell_start, sorted_key, sorted_row, g, nprime, nchunk_blocks, nzero_blocks, zu,  \
                                  (T*)out);                                                                        \
        else                                                                                                       \
            hipLaunchKernelGGL((k_splat_fwd_nhwc<F, RT, T>), gr, bl, 0, s, depth, (const RT*)rows, cell_start,     \
                               sorted_key, sorted_row, g, nprime, nchunk_blocks, nzero_blocks, zu, (T*)out);       \
    } while (0)
        if (out_dtype == LSS_F32) {
            if (!fused) LSS_NHWC_FWD(false, float, float);
            else if (ctx_bf16) LSS_NHWC_FWD(true, bf16, float);
            else LSS_NHWC_FWD(true, float, float);
        } else {
            if (!fused) LSS_NHWC_FWD(false, float, bf16);
            else if (ctx_bf16) LSS_NHWC_FWD(true, bf16, bf16);
            else LSS_NHWC_FWD(true, float, bf16);
        }
#undef LSS_NHWC_FWD
        return launch_status();
    }
    if (sg.YT > kYtMax) return LSS_EUNSUPPORTED;  // (choose_yt never picks more)
    const int nblocks = dims->B * sg.Z * sg.X * sg.ntiles_y;
    const dim3 gr2(xcd_grid((long)nblocks)), bl2(kN2Block);
    const size_t lds2 = (size_t)kC * nchw2_stride(sg.YT) * sizeof(float);
#define LSS_SPLAT2(F, RT, T)                                                                                      \
    do {                                                                                                          \
        if (e0 || e1)                                                                                             \
            hipExtLaunchKernelGGL((k_splat_fwd_nchw2<F, RT, T>), gr2, bl2, (uint32_t)lds2, s, e0, e1, \
                                  0, depth, (const RT*)rows, cell_start, sorted_key, sorted_row, sg, nblocks,     \
                                  (T*)out);                                                                       \
        else                                                                                                      \
            hipLaunchKernelGGL((k_splat_fwd_nchw2<F, RT, T>), gr2, bl2, lds2, s, depth,              \
                               (const RT*)rows, cell_start, sorted_key, sorted_row, sg, nblocks, (T*)out);        \
    } while (0)
    if (out_dtype == LSS_F32) {
        if (!fused) LSS_SPLAT2(false, float, float);
        else if (ctx_bf16) LSS_SPLAT2(true, bf16, float);
        else LSS_SPLAT2(true, float, float);
    } else {
        if (!fused) LSS_SPLAT2(false, float, bf16);
        else if (ctx_bf16) LSS_SPLAT2(true, bf16, bf16);
        else LSS_SPLAT2(true, float, bf16);
    }
#undef LSS_SPLAT2
    return launch_status();
}

int lss_bev_rows(const void* dbev, int32_t g_dtype, const int32_t* cell_start, const lss_dims_t* dims,
                 const lss_grid_t* grid, void* rows, lss_stream_t stream) {
    if (!dims_ok(dims) || !grid_ok(grid) || !dbev || !cell_start || !rows) return LSS_EINVAL;
    SplatGeo sg = splat_geo(grid, dims);
    sg.nrows = sg.ncells;  // gradient rows: one per cell
    const int nblocks = dims->B * sg.Z * sg.X * sg.ntiles_y;
    const size_t lds = (size_t)kC * (sg.YT + 1) * sizeof(float);
    hipStream_t s = (hipStream_t)stream;
    if (g_dtype == LSS_F32)
        hipLaunchKernelGGL(k_bev_rows<float>, dim3(nblocks), dim3(kBlock), lds, s, (const float*)dbev, cell_start, sg,
                           (float*)rows);
    else if (g_dtype == LSS_BF16)
        hipLaunchKernelGGL(k_bev_rows<bf16>, dim3(nblocks), dim3(kBlock), lds, s, (const bf16*)dbev, cell_start, sg,
                           (bf16*)rows);
    else
        return LSS_EINVAL;
    return launch_status();
}

int lss_splat_bwd(const void* g, int32_t g_dtype, int32_t rows_layout, const int32_t* cell_of, const float* depth,
                  const void* ctx_t, int32_t ctx_dtype, const lss_dims_t* dims, const lss_grid_t* grid,
                  void* d_depthnet_out, int32_t d_dtype, lss_stream_t stream) {
    if (!dims_ok(dims) || !grid_ok(grid) || !g || !cell_of || !depth || !ctx_t || !d_depthnet_out) return LSS_EINVAL;
    if (dims->D > 4 * kWave) return LSS_EUNSUPPORTED;  // D <= 256 (the register kernel's 4 chunks)
    SplatGeo sg = splat_geo(grid, dims);
    sg.nrows = sg.ncells;  // gradient rows: one per cell
    const int HW = dims->H * dims->W;
    const int npix = dims->B * dims->N * HW;
    const int wpb = kBlock / kWave;
    const dim3 gr(grid_blocks(npix, wpb)), bl(kBlock);
    hipStream_t s = (hipStream_t)stream;
    const bool nhwc = rows_layout == LSS_NHWC;
    const int D = dims->D;
    // pixel tiles (D <= 64; whole tiles, at most one image boundary per tile, store runs inside one
    // image) or the register kernel, 64 depth bins per chunk
    auto tile_ok = [&](int px) { return npix % px == 0 && px <= HW && HW % 4 == 0 && (px % 8 != 0 || HW % 8 == 0); };
#define LSS_BWD_REGK(GT, DT, CT, NH)                                                                              \
    do {                                                                                                          \
        if (D <= kWave)                                                                                           \
            hipLaunchKernelGGL((k_splat_bwd_reg<GT, DT, CT, NH, 1>), gr, bl, 0, s, (const GT*)g, cell_of, depth,  \
                               (const CT*)ctx_t, D, HW, npix, sg, (DT*)d_depthnet_out);                           \
        else if (D <= 2 * kWave)                                                                                  \
            hipLaunchKernelGGL((k_splat_bwd_reg<GT, DT, CT, NH, 2>), gr, bl, 0, s, (const GT*)g, cell_of, depth,  \
                               (const CT*)ctx_t, D, HW, npix, sg, (DT*)d_depthnet_out);                           \
        else                                                                                                      \
            hipLaunchKernelGGL((k_splat_bwd_reg<GT, DT, CT, NH, 4>), gr, bl, 0, s, (const GT*)g, cell_of, depth,  \
                               (const CT*)ctx_t, D, HW, npix, sg, (DT*)d_depthnet_out);                           \
    } while (0)
#define LSS_BWD_TILE(GT, DT, CT, NH, MAXD, WV, PPW, MINW)                                                        \
    hipLaunchKernelGGL((k_splat_bwd_tile<GT, DT, CT, NH, MAXD, WV, PPW, MINW>), dim3(xcd_grid(npix / ((WV) * (PPW)))), \
                       dim3((WV) * kWave), 0, s, (const GT*)g, cell_of, depth, (const CT*)ctx_t, D, HW, npix, sg,      \
                       (DT*)d_depthnet_out)
#define LSS_BWD_NH(GT, DT, CT, NH)                                                                                \
    do {                                                                                                          \
        constexpr bool kB16 = sizeof(GT) == 2;                                                                    \
        if (kB16 && D <= 48 && tile_ok(kBwdBigWaves * kBwdBigPpw))                                                \
            LSS_BWD_TILE(GT, DT, CT, NH, 48, kB16 ? kBwdBigWaves : 8, kB16 ? kBwdBigPpw : 1,                     \
                         kB16 ? kBwdBigMinW : 4);                                                                 \
        else if (D <= 48 && tile_ok(8))                                                                           \
            LSS_BWD_TILE(GT, DT, CT, NH, 48, 8, 1, kB16 ? 5 : 4);                                                 \
        else if (D <= 64 && tile_ok(8))                                                                           \
            LSS_BWD_TILE(GT, DT, CT, NH, 64, 8, 1, kB16 ? 5 : 4);                                                 \
        else                                                                                                      \
            LSS_BWD_REGK(GT, DT, CT, NH);                                                                         \
    } while (0)
#define LSS_BWD(GT, DT, CT)                                                                                       \
    do { if (nhwc) LSS_BWD_NH(GT, DT, CT, true); else LSS_BWD_NH(GT, DT, CT, false); } while (0)
#define LSS_BWD2(GT, DT) \
    do { if (ctx_dtype == LSS_BF16) LSS_BWD(GT, DT, bf16); else LSS_BWD(GT, DT, float); } while (0)
    if (ctx_dtype != LSS_F32 && ctx_dtype != LSS_BF16) return LSS_EINVAL;
    if (g_dtype == LSS_F32 && d_dtype == LSS_F32) LSS_BWD2(float, float);
    else if (g_dtype == LSS_F32 && d_dtype == LSS_BF16) LSS_BWD2(float, bf16);
    else if (g_dtype == LSS_BF16 && d_dtype == LSS_F32) LSS_BWD2(bf16, float);
    else if (g_dtype == LSS_BF16 && d_dtype == LSS_BF16) LSS_BWD2(bf16, bf16);
    else return LSS_EINVAL;
#undef LSS_BWD2
#undef LSS_BWD
#undef LSS_BWD_NH
#undef LSS_BWD_TILE
#undef LSS_BWD_REGK
    return launch_status();
}

int lss_splat_bwd_lifted(const void* g, int32_t g_dtype, int32_t rows_layout, const int32_t* cell_of, int32_t nprime,
                         const lss_dims_t* dims, const lss_grid_t* grid, float* dx, lss_stream_t stream) {
    if (!dims_ok(dims) || !grid_ok(grid) || !g || !cell_of || !dx || nprime <= 0) return LSS_EINVAL;
    SplatGeo sg = splat_geo(grid, dims);
    sg.nrows = sg.ncells;  // gradient rows: one per cell
    const dim3 gr(grid_blocks(16L * nprime, kBlock)), bl(kBlock);
    hipStream_t s = (hipStream_t)stream;
    const bool nhwc = rows_layout == LSS_NHWC;
    if (g_dtype == LSS_F32) {
        if (nhwc) hipLaunchKernelGGL((k_splat_bwd_lifted<float, true>), gr, bl, 0, s, (const float*)g, cell_of, nprime, sg, dx);
        else hipLaunchKernelGGL((k_splat_bwd_lifted<float, false>), gr, bl, 0, s, (const float*)g, cell_of, nprime, sg, dx);
    } else if (g_dtype == LSS_BF16) {
        if (nhwc) hipLaunchKernelGGL((k_splat_bwd_lifted<bf16, true>), gr, bl, 0, s, (const bf16*)g, cell_of, nprime, sg, dx);
        else hipLaunchKernelGGL((k_splat_bwd_lifted<bf16, false>), gr, bl, 0, s, (const bf16*)g, cell_of, nprime, sg, dx);
    } else {
        return LSS_EINVAL;
    }
    return launch_status();
}

size_t lss_segment_scratch_bytes(int32_t n) {
    if (n < 0) return 0;
    const size_t partial = sizeof(int32_t) * (size_t)((n + kScanItems - 1) / kScanItems + 1);
    const size_t a = (partial + 255) & ~(size_t)255;
    const size_t f = ((sizeof(int32_t) * (size_t)n) + 255) & ~(size_t)255;
    return a + f + sizeof(int32_t) * ((size_t)n + 1);
}

int lss_segment_build(const long long* ranks, int32_t n, int32_t* seg_of, int32_t* seg_start, int32_t* nseg,
                      void* scratch, lss_stream_t stream) {
    if (!ranks || !seg_of || !seg_start || !nseg || !scratch || n <= 0 || n >= INT_MAX - kBlock) return LSS_EINVAL;
    const int nb = (n + kScanItems - 1) / kScanItems;
    char* base = static_cast<char*>(scratch);
    int32_t* partial = reinterpret_cast<int32_t*>(base);
    const size_t a = ((sizeof(int32_t) * (size_t)(nb + 1)) + 255) & ~(size_t)255;
    int32_t* flag = reinterpret_cast<int32_t*>(base + a);
    int32_t* excl = reinterpret_cast<int32_t*>(base + a + (((sizeof(int32_t) * (size_t)n) + 255) & ~(size_t)255));
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(k_seg_flags, dim3(grid_blocks(n, kBlock)), dim3(kBlock), 0, s, ranks, n, flag);
    hipLaunchKernelGGL(k_scan_partials, dim3(nb), dim3(1024), 0, s, flag, n, partial);
    hipLaunchKernelGGL(k_scan_apply, dim3(xcd_grid(nb)), dim3(1024), 0, s, flag, n, partial, excl);
    hipLaunchKernelGGL(k_seg_finish, dim3(grid_blocks(n, kBlock)), dim3(kBlock), 0, s, flag, excl, n, seg_of,
                       seg_start, nseg);
    return launch_status();
}

int lss_segment_sum(const float* x, int32_t C, const int32_t* seg_start, int32_t nseg, const long long* keys,
                    int32_t key_width, long long* key_out, float* out, lss_stream_t stream) {
    if (!x || !seg_start || !out || C <= 0 || nseg < 0 || (keys && (!key_out || key_width <= 0))) return LSS_EINVAL;
    if (nseg == 0) return 0;
    hipLaunchKernelGGL(k_seg_sum, dim3(grid_blocks(nseg, kBlock / kWave)), dim3(kBlock), 0, (hipStream_t)stream, x,
                       C, seg_start, nseg, keys, key_width, key_out, out);
    return launch_status();
}

int lss_segment_gather(const float* g, int32_t C, const int32_t* seg_of, int32_t n, float* dx, lss_stream_t stream) {
    if (!g || !seg_of || !dx || C <= 0 || n < 0) return LSS_EINVAL;
    if (n == 0) return 0;
    const long elems = (long)n * C;
    const long threads = (C & 3) == 0 ? elems / 4 : elems;
    hipLaunchKernelGGL(k_seg_gather, dim3(grid_blocks(threads, kBlock)), dim3(kBlock), 0, (hipStream_t)stream, g, C,
                       seg_of, elems, dx, INT_MAX);  // (the run count is not part of this ABI: sign check only)
    return launch_status();
}

}  // extern "C"

// lss_optim.hip -- gfx950 optimizer step of the training loop (train_simbev.py:245-248): gradient clipping
// (torch.nn.utils.clip_grad_norm_(params, max_norm)) fused with Adam (torch.optim.Adam, L2 weight decay,
// no amsgrad) over the flat fp32 master parameters, two launches for any number of parameter tensors:
//   1. sum of the squared gradients, one partial per block (fixed element ranges, fixed reduction order);
//      block 0 also advances every tensor's step counter (device-resident, as capturable Adam keeps it);
//   2. every block folds the partials in the same order (identical norm everywhere), clip factor
//      c = min(max_norm / (norm + 1e-6), 1), then for its elements: g = c grad + wd p,
//      m = b1 m + (1 - b1) g, v = b2 v + (1 - b2) g^2, p -= lr / (1 - b1^t) * m / (sqrt(v) / sqrt(1 - b2^t) + eps).
// torch's path runs a foreach norm, about eight scalar kernels, a foreach multiply of every gradient and the
// fused Adam kernel: the gradients are read three times and written once; here they are read twice.
// The clipped gradient itself is not written back (nothing reads it after the step).

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "lss_convs.h"

#pragma clang fp contract(fast)

namespace {

constexpr int kBlock = 256;
constexpr int kWave = 64;
constexpr int kMaxBlocks = 1024;       // norm-pass blocks (partials)
constexpr int kMaxAdamBlocks = 16384;  // Adam-pass blocks

struct Segs {
    float* p[LSS_ADAM_MAX_TENSORS];
    const float* g[LSS_ADAM_MAX_TENSORS];
    float* m[LSS_ADAM_MAX_TENSORS];
    float* v[LSS_ADAM_MAX_TENSORS];
    float* step[LSS_ADAM_MAX_TENSORS];
    long long start[LSS_ADAM_MAX_TENSORS + 1];  // prefix sums of the tensor sizes
    int count;
};

// the block's element range of the concatenated tensors, in multiples of 4 elements
__device__ __forceinline__ void block_range(long long total, long long& lo, long long& hi) {
    const long long per = ((total + gridDim.x - 1) / gridDim.x + 3) & ~3ll;
    lo = min((long long)blockIdx.x * per, total);
    hi = min(lo + per, total);
}

// f(segment, first, end) over the parts of [lo, hi) in each tensor
template <typename F>
__device__ __forceinline__ void for_segments(const Segs& s, long long lo, long long hi, F&& f) {
    for (int k = 0; k < s.count; ++k) {
        const long long a = max(lo, s.start[k]), b = min(hi, s.start[k + 1]);
        if (a < b) f(k, a - s.start[k], b - s.start[k]);
    }
}

__device__ __forceinline__ float block_sum(float x, float* s_w) {
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) x += __shfl_xor(x, o, kWave);
    __syncthreads();
    if ((threadIdx.x & (kWave - 1)) == 0) s_w[threadIdx.x / kWave] = x;
    __syncthreads();
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < kBlock / kWave; ++w) t += s_w[w];
    return t;  // every thread
}

__global__ __launch_bounds__(kBlock) void k_clip_sumsq(Segs s, float* __restrict__ partial) {
    __shared__ float s_w[kBlock / kWave];
    long long lo, hi;
    block_range(s.start[s.count], lo, hi);
    float acc = 0.f;
    for_segments(s, lo, hi, [&](int k, long long a, long long b) {
        const float* g = s.g[k];
        long long i = a + threadIdx.x * 4;
        // a segment's part starts on a 4-element boundary of the concatenation; its own alignment decides
        const bool vec = ((s.start[k] & 3) == 0) && ((reinterpret_cast<uintptr_t>(g) & 15) == 0);
        if (vec) {
            for (; i + 3 < b; i += kBlock * 4) {
                const float4 q = *reinterpret_cast<const float4*>(g + i);
                acc = fmaf(q.x, q.x, acc);
                acc = fmaf(q.y, q.y, acc);
                acc = fmaf(q.z, q.z, acc);
                acc = fmaf(q.w, q.w, acc);
            }
        }
        for (; i < b; i += kBlock * 4)
            for (long long j = i; j < min(i + 4, b); ++j) acc = fmaf(g[j], g[j], acc);
    });
    const float t = block_sum(acc, s_w);
    if (threadIdx.x == 0) partial[blockIdx.x] = t;
    if (blockIdx.x == 0 && (int)threadIdx.x < s.count) s.step[threadIdx.x][0] += 1.f;
}

__device__ __forceinline__ void adam_one(float& p, float g, float& m, float& v, float c, float wd, float b1, float b2,
                                         float step_size, float bc2_sqrt, float eps) {
    g = fmaf(wd, p, g * c);
    m = fmaf(b1, m, (1.f - b1) * g);
    v = fmaf(b2, v, (1.f - b2) * g * g);
    p -= step_size * m / (sqrtf(v) / bc2_sqrt + eps);
}

__global__ __launch_bounds__(kBlock) void k_clip_adam(Segs s, const float* __restrict__ partial, int npartial,
                                                      float max_norm, float lr, float b1, float b2, float eps,
                                                      float wd) {
    __shared__ float s_w[kBlock / kWave];
    float acc = 0.f;
    for (int i = threadIdx.x; i < npartial; i += kBlock) acc += partial[i];
    const float norm = sqrtf(block_sum(acc, s_w));
    // clip_coef.clamp(max=1) as torch computes it: a NaN / inf norm passes through (fminf would return
    // 1 for a NaN and leave the step unclipped), so every parameter goes non-finite as with torch
    const float q = max_norm / (norm + 1e-6f);
    const float c = q != q ? q : fminf(q, 1.f);
    long long lo, hi;
    block_range(s.start[s.count], lo, hi);
    for_segments(s, lo, hi, [&](int k, long long a, long long b) {
        const float t = s.step[k][0];
        const float step_size = lr / (1.f - powf(b1, t));
        const float bc2_sqrt = sqrtf(1.f - powf(b2, t));
        float* p = s.p[k];
        const float* g = s.g[k];
        float* m = s.m[k];
        float* v = s.v[k];
        long long i = a + threadIdx.x * 4;
        const bool vec = ((s.start[k] & 3) == 0) &&
                         (((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(g) |
                            reinterpret_cast<uintptr_t>(m) | reinterpret_cast<uintptr_t>(v)) & 15) == 0);
        if (vec) {
            for (; i + 3 < b; i += kBlock * 4) {
                float4 pp = *reinterpret_cast<float4*>(p + i), mm = *reinterpret_cast<float4*>(m + i),
                       vv = *reinterpret_cast<float4*>(v + i);
                const float4 gg = *reinterpret_cast<const float4*>(g + i);
                adam_one(pp.x, gg.x, mm.x, vv.x, c, wd, b1, b2, step_size, bc2_sqrt, eps);
                adam_one(pp.y, gg.y, mm.y, vv.y, c, wd, b1, b2, step_size, bc2_sqrt, eps);
                adam_one(pp.z, gg.z, mm.z, vv.z, c, wd, b1, b2, step_size, bc2_sqrt, eps);
                adam_one(pp.w, gg.w, mm.w, vv.w, c, wd, b1, b2, step_size, bc2_sqrt, eps);
                *reinterpret_cast<float4*>(p + i) = pp;
                *reinterpret_cast<float4*>(m + i) = mm;
                *reinterpret_cast<float4*>(v + i) = vv;
            }
        }
        for (; i < b; i += kBlock * 4)
            for (long long j = i; j < min(i + 4, b); ++j)
                adam_one(p[j], g[j], m[j], v[j], c, wd, b1, b2, step_size, bc2_sqrt, eps);
    });
}

}  // namespace

extern "C" {

int lss_clip_adam_partials(void) { return kMaxBlocks; }

int lss_clip_adam(int32_t count, float* const* params, const float* const* grads, float* const* exp_avg,
                  float* const* exp_avg_sq, float* const* step, const int64_t* numel, float max_norm, float lr,
                  float beta1, float beta2, float eps, float weight_decay, float* partial, void* stream) {
    if (count <= 0 || count > LSS_ADAM_MAX_TENSORS || !params || !grads || !exp_avg || !exp_avg_sq || !step ||
        !numel || !partial || !(max_norm > 0.f))
        return LSS_CONV_EINVAL;
    Segs s{};
    s.count = count;
    s.start[0] = 0;
    for (int k = 0; k < count; ++k) {
        if (!params[k] || !grads[k] || !exp_avg[k] || !exp_avg_sq[k] || !step[k] || numel[k] <= 0)
            return LSS_CONV_EINVAL;
        s.p[k] = params[k];
        s.g[k] = grads[k];
        s.m[k] = exp_avg[k];
        s.v[k] = exp_avg_sq[k];
        s.step[k] = step[k];
        for (int j = 0; j < k; ++j)  // each step counter is advanced once per call
            if (step[j] == step[k] || params[j] == params[k]) return LSS_CONV_EINVAL;
        s.start[k + 1] = s.start[k] + numel[k];
    }
    const long long total = s.start[count];
    // the norm pass: at most kMaxBlocks partials (each Adam block folds them all); the Adam pass: ~8 elements
    // per thread, so the stream of 28 B per parameter has many blocks' loads in flight
    long long nb = (total + kBlock * 16 - 1) / (kBlock * 16);
    nb = nb < 1 ? 1 : (nb > kMaxBlocks ? kMaxBlocks : nb);
    long long nb2 = (total + kBlock * 8 - 1) / (kBlock * 8);
    nb2 = nb2 < 1 ? 1 : (nb2 > kMaxAdamBlocks ? kMaxAdamBlocks : nb2);
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(k_clip_sumsq, dim3((unsigned)nb), dim3(kBlock), 0, st, s, partial);
    hipLaunchKernelGGL(k_clip_adam, dim3((unsigned)nb2), dim3(kBlock), 0, st, s, (const float*)partial, (int)nb, max_norm,
                       lr, beta1, beta2, eps, weight_decay);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

}  // extern "C"

// lss_ceiling.hip -- measurement kernels for bench.py's roofline (not on the model's path).
//
// The splat forward is bound by its HBM write stream (the dense BEV). Its honest ceiling is a
// hand-written streaming-store kernel over the same buffer: every lane writes 16-B vectors,
// consecutive lanes consecutive addresses (1 KB per wave-instruction), `per_thread` vectors per
// lane issued back to back with no load in between (a store never waits). The cache state before
// the launch is set by the caller with lss_ceiling_read (a read sweep: L2 / Infinity Cache full of
// clean lines) or a large store (full of dirty lines that the measured writes must evict).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

#include "lss_hip.h"

namespace {

using u32x4 = __attribute__((ext_vector_type(4))) unsigned;

// flavor 0: plain global_store_dwordx4, 1: non-temporal (nt), 2: device scope (sc1: written through
// the XCD's L2 and dropped from it, no dirty line left for the end-of-kernel write-back)
template <int FLAVOR>
__global__ __launch_bounds__(256) void k_ceiling_store(u32x4* __restrict__ dst, long nvec, int per_thread, unsigned v) {
    const long stride = (long)gridDim.x * blockDim.x;
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const u32x4 x = {v, v, v, v};
    for (int k = 0; k < per_thread; ++k, i += stride) {
        if (i < nvec) {
            if (FLAVOR == 1) __builtin_nontemporal_store(x, dst + i);
            else if (FLAVOR == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(dst + i), "v"(x) : "memory");
            else dst[i] = x;
        }
    }
}

// 16-B loads of `nvec` vectors, XOR-folded; the fold is written only if it equals a value no real
// sweep produces, so the loads cannot be dropped and nothing is written.
__global__ __launch_bounds__(256) void k_ceiling_read(const u32x4* __restrict__ src, long nvec,
                                                      unsigned* __restrict__ sink) {
    const long stride = (long)gridDim.x * blockDim.x;
    unsigned acc = 0;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += stride) {
        const u32x4 a = src[i];
        acc ^= a.x ^ a.y ^ a.z ^ a.w;
    }
    if (acc == 0x9E3779B9u && sink) sink[0] = acc;
}

}  // namespace

extern "C" {

int lss_ceiling_store(void* dst, size_t bytes, int32_t per_thread, int32_t flavor, lss_stream_t stream,
                      lss_event_t ev_start, lss_event_t ev_stop) {
    if (!dst || (bytes & 15) || ((uintptr_t)dst & 15) || per_thread < 1 || flavor < 0 || flavor > 2)
        return LSS_EINVAL;
    const long nvec = (long)(bytes / 16);
    const long threads = (nvec + per_thread - 1) / per_thread;
    const dim3 gr((unsigned)((threads + 255) / 256)), bl(256);
    hipStream_t s = (hipStream_t)stream;
    hipEvent_t e0 = (hipEvent_t)ev_start, e1 = (hipEvent_t)ev_stop;
    if (flavor == 2)
        hipExtLaunchKernelGGL(k_ceiling_store<2>, gr, bl, 0, s, e0, e1, 0, (u32x4*)dst, nvec, (int)per_thread, 0u);
    else if (flavor == 1)
        hipExtLaunchKernelGGL(k_ceiling_store<1>, gr, bl, 0, s, e0, e1, 0, (u32x4*)dst, nvec, (int)per_thread, 0u);
    else
        hipExtLaunchKernelGGL(k_ceiling_store<0>, gr, bl, 0, s, e0, e1, 0, (u32x4*)dst, nvec, (int)per_thread, 0u);
    return (int)hipGetLastError();
}

int lss_ceiling_read(const void* src, size_t bytes, void* sink, lss_stream_t stream) {
    if (!src || (bytes & 15) || ((uintptr_t)src & 15)) return LSS_EINVAL;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
    hipLaunchKernelGGL(k_ceiling_read, dim3(cus * 8), dim3(256), 0, (hipStream_t)stream, (const u32x4*)src,
                       (long)(bytes / 16), (unsigned*)sink);
    return (int)hipGetLastError();
}

}  // extern "C"

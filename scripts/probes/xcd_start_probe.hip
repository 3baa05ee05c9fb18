// Probe: when does each XCD start a kernel that follows another on the same stream? A predecessor
// writes B bytes (plain stores: dirty L2 lines; non-temporal stores; or nothing), on every XCD or from
// the blocks of one XCD only; then a stamping kernel records, per wave, its XCD and s_memrealtime at
// its start. Per XCD: the first / median start after the predecessor's last wave ended (its waves stamp
// their end too). Eager launches and the same pair replayed as a hipGraph.
//   hipcc --offload-arch=gfx950 -O3 -o scripts/probes/xcd_start_probe scripts/probes/xcd_start_probe.hip
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int xcc_id() { return __builtin_amdgcn_s_getreg(20 | (31 << 11)) & 0xf; }

// mode 0: plain 16-B stores, 1: non-temporal 16-B stores, 2: no stores. only_xcd >= 0: blocks on other
// XCDs exit at once. Lane 0 of each wave stamps its end into its own slot (one atomic word for all
// waves serialises at the memory side: ~90 per us).
__global__ void k_dirty(u32x4* buf, long n16, int mode, int only_xcd, unsigned long long* end_stamp) {
    const int x = xcc_id();
    if (only_xcd < 0 || x == only_xcd) {
        if (mode != 2) {
            const long stride = (long)gridDim.x * blockDim.x;
            for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
                const u32x4 v = {(unsigned)i, 1u, 2u, 3u};
                if (mode == 0) buf[i] = v;
                else __builtin_nontemporal_store(v, buf + i);
            }
        }
    }
    if ((threadIdx.x & 63) == 0)
        end_stamp[blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)] = __builtin_amdgcn_s_memrealtime();
}

__global__ void k_stamp(unsigned long long* out) {
    if ((threadIdx.x & 63) == 0) {
        const unsigned long long t = __builtin_amdgcn_s_memrealtime();
        const int w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
        out[2 * w] = t;
        out[2 * w + 1] = (unsigned long long)xcc_id();
    }
}

int main() {
    const long bytes = 64L << 20;
    const int sblocks = 2048, sthreads = 256, waves = sblocks * sthreads / 64;
    u32x4* buf;
    unsigned long long *stamps, *endp;
    hipMalloc(&buf, bytes);
    hipMalloc(&stamps, sizeof(unsigned long long) * 2 * waves);
    const int dwaves = 1024 * 256 / 64;
    hipMalloc(&endp, sizeof(unsigned long long) * dwaves);
    std::vector<unsigned long long> he(dwaves);
    hipStream_t s;
    hipStreamCreate(&s);
    std::vector<unsigned long long> h(2 * waves);
    struct V { const char* name; long mb; int mode; int only; int pblocks; int ext; };
    const V vs[] = {{"no stores", 0, 2, -1, 1024, 0},          {"plain 8 MB all XCDs", 8, 0, -1, 1024, 0},
                    {"plain 32 MB all XCDs", 32, 0, -1, 1024, 0}, {"nt 32 MB all XCDs", 32, 1, -1, 1024, 0},
                    {"plain 16 MB XCD 0 only", 16, 0, 0, 1024, 0}, {"plain 64 MB all XCDs", 64, 0, -1, 1024, 0},
                    {"132 blocks, 2.5 MB", 2, 0, -1, 132, 0},    {"132 blocks, 2.5 MB, ext+events", 2, 0, -1, 132, 1},
                    {"no stores, ext+events", 0, 2, -1, 1024, 1}, {"plain 8 MB, ext+events", 8, 0, -1, 1024, 1}};
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int graph = 0; graph < 2; ++graph) {
        printf("%s\n", graph ? "graph replays (pair captured once per variant)" : "eager launches");
        for (const V& v : vs) {
            if (graph && v.ext) continue;  // (kernel-stamped events are not captured)
            hipGraphExec_t ge = nullptr;
            auto launch = [&]() {
                hipLaunchKernelGGL(k_dirty, dim3(v.pblocks), dim3(256), 0, s, buf, (v.mb << 20) / 16, v.mode, v.only, endp);
                if (v.ext)
                    hipExtLaunchKernelGGL(k_stamp, dim3(sblocks), dim3(sthreads), 0, s, e0, e1, 0, stamps);
                else
                    hipLaunchKernelGGL(k_stamp, dim3(sblocks), dim3(sthreads), 0, s, stamps);
            };
            if (graph) {
                hipGraph_t g;
                hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
                launch();
                hipStreamEndCapture(s, &g);
                hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
            }
            for (int rep = 0; rep < 4; ++rep) {
                if (graph) hipGraphLaunch(ge, s);
                else launch();
                hipStreamSynchronize(s);
                if (rep < 1) continue;
                hipMemcpy(h.data(), stamps, sizeof(unsigned long long) * 2 * waves, hipMemcpyDeviceToHost);
                hipMemcpy(he.data(), endp, sizeof(unsigned long long) * dwaves, hipMemcpyDeviceToHost);
                const unsigned long long end = *std::max_element(he.begin(), he.begin() + v.pblocks * 4);
                printf("  %-24s rep %d: start after predecessor end (us) per XCD first/median:", v.name, rep);
                for (int x = 0; x < 8; ++x) {
                    std::vector<double> t;
                    for (int w = 0; w < waves; ++w)
                        if ((int)h[2 * w + 1] == x) t.push_back(((double)h[2 * w] - (double)end) / 100.0);
                    if (t.empty()) { printf(" -"); continue; }
                    std::sort(t.begin(), t.end());
                    printf(" %5.2f/%5.2f", t.front(), t[t.size() / 2]);
                }
                printf("\n");
            }
        }
    }
    return 0;
}

// Probe: which XCD (HW_REG_XCC_ID) runs blocks 0..15 of consecutive launches of differently sized
// grids, eagerly and inside a replayed hipGraph -- does blockIdx % 8 name the same XCD across kernels?
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_xcc(int* out, int n) {
    if (threadIdx.x == 0 && blockIdx.x < n) out[blockIdx.x] = __builtin_amdgcn_s_getreg(20 | (31 << 11)) & 0xf;
}

int main() {
    const int grids[] = {256, 1056, 704, 8, 13, 264, 256, 4096};
    const int ng = sizeof(grids) / sizeof(grids[0]);
    int* d;
    hipMalloc(&d, sizeof(int) * 16 * 64);
    int h[16 * 64];
    hipStream_t s;
    hipStreamCreate(&s);
    printf("eager launches (grid: XCC of blocks 0..15)\n");
    for (int rep = 0; rep < 3; ++rep)
        for (int i = 0; i < ng; ++i) {
            hipLaunchKernelGGL(k_xcc, dim3(grids[i]), dim3(64), 0, s, d + 16 * (rep * ng + i), 16);
        }
    hipStreamSynchronize(s);
    hipMemcpy(h, d, sizeof(int) * 16 * 3 * ng, hipMemcpyDeviceToHost);
    for (int rep = 0; rep < 3; ++rep)
        for (int i = 0; i < ng; ++i) {
            printf("rep %d grid %5d:", rep, grids[i]);
            for (int b = 0; b < 16; ++b) printf(" %d", h[16 * (rep * ng + i) + b]);
            printf("\n");
        }
    // the same sequence captured once and replayed three times
    hipGraph_t g;
    hipGraphExec_t ge;
    hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
    for (int i = 0; i < ng; ++i) hipLaunchKernelGGL(k_xcc, dim3(grids[i]), dim3(64), 0, s, d + 16 * i, 16);
    hipStreamEndCapture(s, &g);
    hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    printf("graph replays\n");
    for (int rep = 0; rep < 3; ++rep) {
        hipGraphLaunch(ge, s);
        hipStreamSynchronize(s);
        hipMemcpy(h, d, sizeof(int) * 16 * ng, hipMemcpyDeviceToHost);
        for (int i = 0; i < ng; ++i) {
            printf("replay %d grid %5d:", rep, grids[i]);
            for (int b = 0; b < 16; ++b) printf(" %d", h[16 * i + b]);
            printf("\n");
        }
    }
    return 0;
}

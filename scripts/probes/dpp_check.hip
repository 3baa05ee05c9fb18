// Probe: cross-lane primitives used by the splat backward's reductions vs the __shfl_xor butterfly,
// lane by lane (prints which lanes of each level are bit-identical).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

template <int CTRL>
__device__ float dpp_f(float v) { return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false)); }

__global__ void k(const float* in, float* out) {
    const int l = threadIdx.x;
    const float v = in[l];
    // 0..5: butterfly xor 1,2,4,8,16,32 via ds_bpermute; 6..: candidates
    out[0 * 64 + l] = v + __shfl_xor(v, 1, 64);
    out[1 * 64 + l] = v + __shfl_xor(v, 2, 64);
    out[2 * 64 + l] = v + __shfl_xor(v, 4, 64);
    out[3 * 64 + l] = v + __shfl_xor(v, 8, 64);
    out[4 * 64 + l] = v + __shfl_xor(v, 16, 64);
    out[5 * 64 + l] = v + __shfl_xor(v, 32, 64);
    out[6 * 64 + l] = v + dpp_f<0xB1>(v);   // quad_perm 1,0,3,2
    out[7 * 64 + l] = v + dpp_f<0x4E>(v);   // quad_perm 2,3,0,1
    out[8 * 64 + l] = v + dpp_f<0x124>(v);  // row_ror:4
    out[9 * 64 + l] = v + dpp_f<0x104>(v);  // row_shl:4
    out[10 * 64 + l] = v + dpp_f<0x114>(v); // row_shr:4
    out[11 * 64 + l] = v + dpp_f<0x128>(v); // row_ror:8
    {
        const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
        out[12 * 64 + l] = __uint_as_float(p[0]) + __uint_as_float(p[1]);
    }
    {
        const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
        out[13 * 64 + l] = __uint_as_float(p[0]) + __uint_as_float(p[1]);
    }
}

__device__ int wave_incl_scan(int v) {  // as lss_hip.hip
    int t = v + __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);
    t += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);
    t += __builtin_amdgcn_update_dpp(0, v, 0x113, 0xf, 0xf, false);
    t += __builtin_amdgcn_update_dpp(0, t, 0x114, 0xf, 0xe, false);
    t += __builtin_amdgcn_update_dpp(0, t, 0x118, 0xf, 0xc, false);
    t += __builtin_amdgcn_update_dpp(0, t, 0x142, 0xa, 0xf, false);
    t += __builtin_amdgcn_update_dpp(0, t, 0x143, 0xc, 0xf, false);
    return t;
}
__global__ void kscan(const int* in, int* out) { out[threadIdx.x] = wave_incl_scan(in[threadIdx.x]); }

int main() {
    float h[64], o[14 * 64];
    for (int i = 0; i < 64; ++i) h[i] = 1.0f + i * 1.0f / 1024 + (i * 37 % 11) * 1e-3f;
    float *din, *dout;
    hipMalloc(&din, sizeof h);
    hipMalloc(&dout, sizeof o);
    hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, din, dout);
    hipMemcpy(o, dout, sizeof o, hipMemcpyDeviceToHost);
    const char* names[] = {"quad_perm(1,0,3,2) vs xor1", "quad_perm(2,3,0,1) vs xor2", "row_ror:4 vs xor4",
                           "row_shl:4 vs xor4", "row_shr:4 vs xor4", "row_ror:8 vs xor8", "permlane16_swap vs xor16",
                           "permlane32_swap vs xor32"};
    const int ref[] = {0, 1, 2, 2, 2, 3, 4, 5};
    for (int c = 0; c < 8; ++c) {
        unsigned long long ok = 0;
        for (int l = 0; l < 64; ++l)
            if (memcmp(&o[(6 + c) * 64 + l], &o[ref[c] * 64 + l], 4) == 0) ok |= 1ull << l;
        printf("%-28s equal lanes mask %016llx\n", names[c], ok);
    }
    int hi[64], ho[64];
    for (int i = 0; i < 64; ++i) hi[i] = (i * 7919) % 1000 - 300;
    int *dii, *dio;
    hipMalloc(&dii, sizeof hi);
    hipMalloc(&dio, sizeof ho);
    hipMemcpy(dii, hi, sizeof hi, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(kscan, dim3(1), dim3(64), 0, 0, dii, dio);
    hipMemcpy(ho, dio, sizeof ho, hipMemcpyDeviceToHost);
    int run = 0, bad = 0;
    for (int i = 0; i < 64; ++i) { run += hi[i]; bad += ho[i] != run; }
    printf("wave_incl_scan (DPP) vs sequential prefix: %d lanes differ\n", bad);
    return bad != 0;
}

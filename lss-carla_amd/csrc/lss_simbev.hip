// lss_simbev.hip -- gfx950 kernels of the SimBEV input path (include/lss_simbev.h).
//
// One thread per output pixel of a camera image computes, with integer arithmetic identical to
// Pillow's, exactly the pixel the reference's PIL chain produces (src/tools.py:120-128):
//   rotate   inverse map of the output pixel through ImagingTransformAffine's 16.16 fixed-point walk
//            (nearest; outside -> 0), or ROTATE_180, or nothing;
//   flip     FLIP_LEFT_RIGHT of the cropped image;
//   crop     offset into the resized image (outside the resized image -> 0);
//   resize   Resample.c's two passes evaluated at that one pixel: for each vertical tap (source row),
//            the horizontal pass's value at that row, clipped to uint8 as Pillow's intermediate image
//            stores it, then the vertical accumulation, clipped again;
//   normalize ToTensor (/255) and Normalize((x - mean) / std), fp32, IEEE division.
// The horizontal values are recomputed per output row (<= ksize_v times each): a few hundred integer
// MACs per pixel, against reading a 322 KB image -- the kernel is bound by its fp32 output writes.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "lss_simbev.h"

namespace {

constexpr int kPrecisionBits = 32 - 8 - 2;  // Resample.c PRECISION_BITS
constexpr int kThreads = 256;

__device__ __forceinline__ int clip8(int acc) {
    const int v = acc >> kPrecisionBits;  // arithmetic shift: floor, as Pillow's clip8 lookup
    return v < 0 ? 0 : (v > 255 ? 255 : v);
}

// Horizontal pass value of source row r at resized column xr (or the source pixel when no pass).
__device__ __forceinline__ void hpass(const uint8_t* __restrict__ img, int src_w, int r, int xr,
                                      const int32_t* __restrict__ th, int hk, int* rgb) {
    const uint8_t* row = img + (size_t)r * src_w * 3;
    if (hk == 0) {
        rgb[0] = row[3 * xr];
        rgb[1] = row[3 * xr + 1];
        rgb[2] = row[3 * xr + 2];
        return;
    }
    const int32_t* t = th + (size_t)xr * (2 + hk);
    const int xmin = t[0], cnt = t[1];
    int a0 = 1 << (kPrecisionBits - 1), a1 = a0, a2 = a0;
    for (int k = 0; k < cnt; ++k) {
        const int c = t[2 + k];
        const uint8_t* px = row + 3 * (xmin + k);
        a0 += (int)px[0] * c;
        a1 += (int)px[1] * c;
        a2 += (int)px[2] * c;
    }
    rgb[0] = clip8(a0);
    rgb[1] = clip8(a1);
    rgb[2] = clip8(a2);
}

__global__ __launch_bounds__(kThreads) void k_simbev_images(const uint8_t* __restrict__ src, int src_h, int src_w,
                                                            const lss_img_aug_t* __restrict__ augs,
                                                            const int32_t* __restrict__ tables, int out_h,
                                                            int out_w, float* __restrict__ out) {
    const int img = blockIdx.y;
    const int pix = blockIdx.x * kThreads + threadIdx.x;
    if (pix >= out_h * out_w) return;
    const lss_img_aug_t p = augs[img];
    const int y = pix / out_w, x = pix - y * out_w;
    int rgb[3] = {0, 0, 0};
    int xs = x, ys = y;
    bool inside = true;
    if (p.rot_mode == 1) {  // ROTATE_180
        xs = out_w - 1 - x;
        ys = out_h - 1 - y;
    } else if (p.rot_mode == 3) {  // ROTATE_90 (square images only, as Image.rotate takes it)
        xs = out_w - 1 - y;
        ys = x;
    } else if (p.rot_mode == 4) {  // ROTATE_270
        xs = y;
        ys = out_h - 1 - x;
    } else if (p.rot_mode == 2) {
        // xx = a2 + y*a1 + x*a0 (the C loop's running int32 sums; no overflow: check_fixed)
        const long long xx = (long long)p.affine[2] + (long long)y * p.affine[1] + (long long)x * p.affine[0];
        const long long yy = (long long)p.affine[5] + (long long)y * p.affine[4] + (long long)x * p.affine[3];
        xs = (int)(xx >> 16);
        ys = (int)(yy >> 16);
        inside = xs >= 0 && xs < out_w && ys >= 0 && ys < out_h;
    }
    if (inside) {
        if (p.flip) xs = out_w - 1 - xs;
        const int xr = xs + p.crop[0], yr = ys + p.crop[1];
        if (xr >= 0 && xr < p.rs_w && yr >= 0 && yr < p.rs_h) {
            const uint8_t* im = src + (size_t)img * src_h * src_w * 3;
            const int32_t* th = tables + p.h_off;
            if (p.v_ksize == 0) {
                hpass(im, src_w, yr, xr, th, p.h_ksize, rgb);
            } else {
                const int32_t* tv = tables + p.v_off + (size_t)yr * (2 + p.v_ksize);
                const int ymin = tv[0], cnt = tv[1];
                int a0 = 1 << (kPrecisionBits - 1), a1 = a0, a2 = a0;
                for (int k = 0; k < cnt; ++k) {
                    int h[3];
                    hpass(im, src_w, ymin + k, xr, th, p.h_ksize, h);
                    const int c = tv[2 + k];
                    a0 += h[0] * c;
                    a1 += h[1] * c;
                    a2 += h[2] * c;
                }
                rgb[0] = clip8(a0);
                rgb[1] = clip8(a1);
                rgb[2] = clip8(a2);
            }
        }
    }
    // ToTensor + Normalize (torchvision: float32(uint8) / 255, then (x - mean) / std, fp32)
    const float mean[3] = {0.485f, 0.456f, 0.406f};
    const float stdv[3] = {0.229f, 0.224f, 0.225f};
    float* o = out + (size_t)img * 3 * out_h * out_w + pix;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float v = __fdiv_rn((float)rgb[c], 255.0f);
        o[(size_t)c * out_h * out_w] = __fdiv_rn(__fsub_rn(v, mean[c]), stdv[c]);
    }
}

// flipud of the vehicle classes 1..3 of one BEV: out[b, 0, i, j] = any(bev[b, 1..3, X-1-i, j] > 0).
__global__ __launch_bounds__(kThreads) void k_vehicle_mask(const uint8_t* __restrict__ bev, int ncls, int X, int Y,
                                                           long total, float* __restrict__ out) {
    const long i = (long)blockIdx.x * kThreads + threadIdx.x;
    if (i >= total) return;
    const long XY = (long)X * Y;
    const long b = i / XY;
    const long r = i - b * XY;
    const int row = (int)(r / Y), col = (int)(r - (long)row * Y);
    const uint8_t* s = bev + (size_t)b * ncls * XY + (size_t)(X - 1 - row) * Y + col;
    const bool v = s[XY] > 0 || s[2 * XY] > 0 || s[3 * XY] > 0;
    out[i] = v ? 1.0f : 0.0f;
}

// ---- host: Pillow's bicubic coefficient tables (Resample.c precompute_coeffs / normalize_coeffs_8bpc)
double bicubic_filter(double x) {
    const double a = -0.5;
    if (x < 0.0) x = -x;
    if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
    if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
    return 0.0;
}

int ksize_of(int in_size, int out_size) {
    double filterscale = (double)((float)in_size - 0.0f) / out_size;  // box (0, in) as floats, as Pillow
    if (filterscale < 1.0) filterscale = 1.0;
    const double support = 2.0 * filterscale;
    return (int)ceil(support) * 2 + 1;
}

}  // namespace

extern "C" {

int lss_resample_ksize(int32_t in_size, int32_t out_size) {
    if (in_size <= 0 || out_size <= 0) return -1;
    return ksize_of(in_size, out_size);
}

int lss_resample_coeffs(int32_t in_size, int32_t out_size, int32_t* table) {
    if (in_size <= 0 || out_size <= 0 || !table) return -1;
    const float in0 = 0.0f, in1 = (float)in_size;
    const double scale = (double)(in1 - in0) / out_size;
    double filterscale = scale;
    if (filterscale < 1.0) filterscale = 1.0;
    const double support = 2.0 * filterscale;
    const int ksize = (int)ceil(support) * 2 + 1;
    double* k = new double[ksize];
    for (int xx = 0; xx < out_size; ++xx) {
        const double center = in0 + (xx + 0.5) * scale;
        double ww = 0.0;
        const double ss = 1.0 / filterscale;
        int xmin = (int)(center - support + 0.5);
        if (xmin < 0) xmin = 0;
        int xmax = (int)(center + support + 0.5);
        if (xmax > in_size) xmax = in_size;
        xmax -= xmin;
        for (int x = 0; x < xmax; ++x) {
            const double w = bicubic_filter((x + xmin - center + 0.5) * ss);
            k[x] = w;
            ww += w;
        }
        for (int x = 0; x < xmax; ++x)
            if (ww != 0.0) k[x] /= ww;
        for (int x = xmax; x < ksize; ++x) k[x] = 0.0;
        int32_t* t = table + (size_t)xx * (2 + ksize);
        t[0] = xmin;
        t[1] = xmax;
        for (int x = 0; x < ksize; ++x)
            t[2 + x] = k[x] < 0 ? (int32_t)(-0.5 + k[x] * (1 << kPrecisionBits))
                                : (int32_t)(0.5 + k[x] * (1 << kPrecisionBits));
    }
    delete[] k;
    return 0;
}

int lss_simbev_images(const uint8_t* src, int32_t n, int32_t src_h, int32_t src_w, const lss_img_aug_t* aug,
                      const int32_t* tables, int32_t out_h, int32_t out_w, float* out, void* stream) {
    if (!src || !aug || !tables || !out || n <= 0 || src_h <= 0 || src_w <= 0 || out_h <= 0 || out_w <= 0) return -1;
    if (n > 65535) return -2;
    const dim3 grid((unsigned)((out_h * out_w + kThreads - 1) / kThreads), (unsigned)n);
    hipLaunchKernelGGL(k_simbev_images, grid, dim3(kThreads), 0, (hipStream_t)stream, src, src_h, src_w, aug, tables,
                       out_h, out_w, out);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

int lss_simbev_vehicle_mask(const uint8_t* bev, int32_t n, int32_t n_classes, int32_t X, int32_t Y, float* out,
                            void* stream) {
    if (!bev || !out || n <= 0 || n_classes < 4 || X <= 0 || Y <= 0) return -1;
    const long total = (long)n * X * Y;
    hipLaunchKernelGGL(k_vehicle_mask, dim3((unsigned)((total + kThreads - 1) / kThreads)), dim3(kThreads), 0,
                       (hipStream_t)stream, bev, n_classes, X, Y, total, out);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

}  // extern "C"

/*
 * lss_simbev.h -- C ABI of the SimBEV input path on MI355X (gfx950): per-camera image augmentation
 * and BEV label decoding on the device.
 *
 * Replaces, per camera, the pixel work of the reference's loader (shdragron/LSS-Carla):
 *   img_transform(img, ...)   src/tools.py:120-128   Image.resize -> crop -> FLIP_LEFT_RIGHT -> rotate
 *   normalize_img(img)        src/tools.py:167-171   ToTensor + Normalize(ImageNet mean / std)
 *   get_binimg(sample)        src/data_simbev.py:220-246   (bev[1] | bev[2] | bev[3]) > 0, np.flipud
 * bit for bit with Pillow's published algorithms (libImaging/Resample.c bicubic fixed-point resample,
 * libImaging/Geometry.c 16.16 fixed-point nearest affine) and torchvision's fp32 normalisation. JPEG
 * decoding and the augmentation draws (np.random, src/data_simbev.py:119-145) stay on the host.
 * Conventions as lss_hip.h: device pointers, asynchronous on `stream`, 0 = success, negative LSS_E*
 * codes for bad arguments, positive hipError_t for launch failures.
 */
#ifndef LSS_SIMBEV_H
#define LSS_SIMBEV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* One camera image's augmentation (sample_augmentation's draws, src/data_simbev.py:119-145). */
typedef struct lss_img_aug {
    int32_t src_h, src_w;          /* decoded image (H, W), 3 channels, uint8 HWC */
    int32_t rs_w, rs_h;            /* resize_dims (W', H') of Image.resize */
    int32_t crop[4];               /* PIL crop box (x0, y0, x1, y1) in the resized image; outside -> 0 */
    int32_t flip;                  /* FLIP_LEFT_RIGHT after the crop */
    int32_t rot_mode;              /* 0: rotate % 360 == 0 (copy), 1: ROTATE_180, 2: affine nearest,
                                      3 / 4: ROTATE_90 / ROTATE_270 (square images, 90 / 270 degrees) */
    int32_t affine[6];             /* rot_mode 2: a0..a5 of ImagingTransformAffine's fixed-point walk */
    int32_t h_off, h_ksize;        /* horizontal pass: table offset (in int32) and taps; h_ksize 0 = no pass */
    int32_t v_off, v_ksize;        /* vertical pass, likewise */
} lss_img_aug_t;

/* Pillow's precompute_coeffs + normalize_coeffs_8bpc for one pass of Image.resize (BICUBIC):
 * out_size rows of (xmin, count, k_0 .. k_{ksize-1}) int32, written to `table` (host memory,
 * out_size * (2 + ksize) ints, ksize from lss_resample_ksize). Host-only, no device work. */
int lss_resample_ksize(int32_t in_size, int32_t out_size);
int lss_resample_coeffs(int32_t in_size, int32_t out_size, int32_t* table);

/* n images (src: n * src_h * src_w * 3 uint8, every image the same size) -> out (n, 3, out_h, out_w)
 * fp32 = normalize_img(img_transform(img)) with the per-image parameters aug[n] and the coefficient
 * tables (device memory) they point into. out_h / out_w = the crop size (final_dim). */
int lss_simbev_images(const uint8_t* src, int32_t n, int32_t src_h, int32_t src_w, const lss_img_aug_t* aug,
                      const int32_t* tables, int32_t out_h, int32_t out_w, float* out, void* stream);

/* BEV labels: bev (n, n_classes, X, Y) uint8 (any value > 0 = set) -> out (n, 1, X, Y) fp32 =
 * flipud((bev[1] > 0) | (bev[2] > 0) | (bev[3] > 0)). n_classes >= 4. */
int lss_simbev_vehicle_mask(const uint8_t* bev, int32_t n, int32_t n_classes, int32_t X, int32_t Y, float* out,
                            void* stream);

#ifdef __cplusplus
}
#endif
#endif /* LSS_SIMBEV_H */

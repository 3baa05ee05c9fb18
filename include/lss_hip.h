/*
 * lss_hip.h -- C ABI of the MI355X (gfx950) Lift-Splat hot path.
 *
 * Drop-in boundary for the reference's hot path (shdragron/LSS-Carla,
 * src/models.py + src/tools.py). Every entry point takes plain device
 * pointers and sizes, is asynchronous on the caller's HIP stream, never
 * synchronises, never allocates, and returns 0 on success, a positive
 * hipError_t on a launch failure, or a negative LSS_E* code for bad
 * arguments. No exceptions cross the ABI; there is no global mutable state.
 * Thread-safe for distinct streams.
 *
 * Index conventions (all int32):
 *   point  p = ((bn*D + d)*H + h)*W + w,   bn = b*N + n      (reference flatten order,
 *                                                              src/models.py:205-209)
 *   pixel  q = bn*H*W + h*W + w
 *   cell   k = ((b*Z + z)*X + x)*Y + y,    -1 = dropped     (griddify order,
 *                                                              src/models.py:240-244)
 * H, W are the feature-map sizes (fH, fW = final_dim / 16). C must be 64
 * (camC is hard-coded, src/models.py:148); D <= 256 (the reference's dbound [4, 45, 1] gives
 * D = 41; [4, 45, 0.5] gives 82).
 */
#ifndef LSS_HIP_H
#define LSS_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LSS_ABI_VERSION 23

typedef struct lss_dims {
    int32_t B, N, D, H, W, C;
} lss_dims_t;

/* Voxel grid: lo = bx - dx/2 (fp32, src/models.py:212), dx, nx = (X, Y, Z). */
typedef struct lss_grid {
    float lo[3];
    float dx[3];
    int32_t nx[3];
} lss_grid_t;

enum { LSS_F32 = 0, LSS_BF16 = 1 };          /* element types */
enum { LSS_NCHW = 0, LSS_NHWC = 1 };         /* BEV memory layouts of a (B, Z*C, X, Y) tensor */
enum { LSS_EINVAL = -1, LSS_EUNSUPPORTED = -2 };

typedef void* lss_stream_t; /* a hipStream_t */
typedef void* lss_event_t;  /* a hipEvent_t */

int lss_abi_version(void);
const char* lss_error_string(int code);

/* Debug builds (liblss_hip_debug.so, compiled with -DLSS_DEBUG=1) check every data-derived global
 * index of the kernels -- cell ids, CSR positions and totals, point ids, feature and gradient rows --
 * before use; a failed check is recorded (the index is replaced by 0 instead of faulting) and the
 * kernels carry on. lss_debug_checks: 1 in a debug build, 0 otherwise. lss_debug_status copies
 * {failures, first failure's check code, its value, its bound} to out4 (host, 4 ints; all zero in a
 * release build) and zeroes the record if clear != 0. Synchronous (device-to-host copy). */
int lss_debug_checks(void);
int lss_debug_status(int32_t* out4, int32_t clear);

/* Profiling helpers: hipEvents for the optional kernel-timestamp arguments of lss_splat_fwd. */
int lss_event_create(lss_event_t* ev);
int lss_event_destroy(lss_event_t ev);
int lss_event_elapsed_ms(lss_event_t start, lss_event_t stop, float* ms); /* synchronises on stop */
/* Record ev on stream. While the stream is being captured into a hipGraph this adds an explicit
 * event-record node to the graph (so every replay stamps the event), not a capture dependency. */
int lss_event_record(lss_event_t ev, lss_stream_t stream);

/* Measurement kernels (bench.py's roofline ceiling; not on the model's path).
 * lss_ceiling_store: `bytes` (multiple of 16, dst 16-B aligned) written with 16-B vector stores,
 *   per_thread vectors per lane (grid-strided), flavor 0 plain / 1 non-temporal / 2 device scope
 *   (sc1: written through the XCD's L2); optional
 *   kernel-stamped events as lss_splat_fwd.
 * lss_ceiling_read: a 16-B-load sweep over `bytes` (sets the cache state before a timed launch);
 *   sink (4 B, device) is never written in practice. */
int lss_ceiling_store(void* dst, size_t bytes, int32_t per_thread, int32_t flavor, lss_stream_t stream,
                      lss_event_t ev_start, lss_event_t ev_stop);
int lss_ceiling_read(const void* src, size_t bytes, void* sink, lss_stream_t stream);

/* get_geometry (src/models.py:170-190) fused with quantise + bounds filter
 * (src/models.py:211-223). fp32, sequential non-FMA mat-vecs, IEEE division,
 * truncation toward zero. out_geom (Nprime*3) may be NULL. cell_of (Nprime)
 * receives the cell id or -1. If cell_count is non-NULL it must be zeroed
 * (B*Z*X*Y ints); each kept point atomically increments its cell's count and
 * slot_of[p] receives the pre-increment value (its slot inside the cell). */
int lss_geometry_cells(const float* frustum, const float* rots, const float* trans,
                       const float* kinv, const float* pinv, const float* post_trans,
                       const lss_dims_t* dims, const lss_grid_t* grid,
                       float* out_geom, int32_t* cell_of, int32_t* cell_count, int32_t* slot_of,
                       lss_stream_t stream);

/* Quantise a given (Nprime, 3) fp32 geometry (voxel_pooling(geom_feats, x) boundary,
 * src/models.py:204-223). Same outputs as lss_geometry_cells; points_per_batch =
 * Nprime / B (src/models.py:214). */
int lss_cells_from_geom(const float* geom, int32_t nprime, int32_t points_per_batch,
                        const lss_grid_t* grid, int32_t* cell_of, int32_t* cell_count,
                        int32_t* slot_of, lss_stream_t stream);

/* Counting-sort CSR of points by cell (replaces ranks + argsort, src/models.py:225-231):
 * cell_start (ncells+1) = exclusive scan of cell_count; sorted_key (Nprime capacity) = the kept
 * points grouped by cell in canonical order -- ascending cell, then ascending point id inside a
 * cell (the order the reference's stable argsort gives points of equal rank) -- each as the key
 * (cell << 32) | p, followed by the sentinel key -1 in every slot from cell_start[ncells] to
 * Nprime; sorted_row (Nprime capacity) = the row each entry's features are read from: the pixel
 * q(p) when dims is given (fused lift), p itself when dims is NULL (per-point rows); defined for
 * the first cell_start[ncells] entries. scratch: lss_csr_scratch_bytes bytes.
 * Replaces: ranks = ...; sorts = ranks.argsort(); x, geom_feats, ranks = x[sorts], ... (src/models.py:225-231). */
size_t lss_csr_scratch_bytes(int32_t ncells, int32_t nprime);
int lss_csr_build(const int32_t* cell_of, const int32_t* slot_of, int32_t nprime,
                  const int32_t* cell_count, int32_t ncells, const lss_dims_t* dims,
                  int32_t* cell_start, long long* sorted_key, int32_t* sorted_row,
                  void* scratch, lss_stream_t stream);

/* lss_csr_build with a persistent workspace: the same outputs, bit for bit, in three kernels
 * instead of four and no count memset -- a single-pass scan (decoupled look-back between blocks,
 * bounded spins) and a scatter that also re-zeroes the scan's state and cell_count for the next
 * call. Contract: `workspace` (lss_csr_workspace_bytes(ncells)) is zero-filled before its first
 * use; cell_count is zero-filled before the first lss_geometry_cells / lss_cells_from_geom that
 * counts into it; every call leaves both zero-filled again. One call at a time per workspace (the
 * caller orders calls that share one: ops.py records the stream and event of its last use).
 * Workspace header, 4 uint32: [0] overflow-record counter of the ordered plans (below; 0 between
 * calls), [1] sticky count of look-back timeouts (a block that
 * waited its spin limit for a predecessor sums that predecessor's counts itself: the output is exact
 * either way), [2] spin-limit override (0: the built-in limit; s > 0: s - 1 polls -- tests of the
 * timeout path), [3] unused. */
size_t lss_csr_workspace_bytes(int32_t ncells);
int lss_csr_build_ws(const int32_t* cell_of, const int32_t* slot_of, int32_t nprime,
                     int32_t* cell_count, int32_t ncells, const lss_dims_t* dims,
                     int32_t* cell_start, long long* sorted_key, int32_t* sorted_row,
                     void* scratch, void* workspace, lss_stream_t stream);

/* Ordered plans (ABI 22): the same CSR as lss_csr_build, bit for bit, in three kernels (geometry,
 * look-back scan, scatter) -- no sort pass after the scatter. The geometry kernel gives every kept
 * point its rank among the points of its cell in its own 256-point block (lower point ids first)
 * and appends one record (block, points) per distinct (block, cell) to the cell's list in `lists`;
 * the scatter places point p at cell_start[cell] + (the cell's points in lower blocks) + rank.
 * cell_word (ncells int32) packs the cell's point count (low 20 bits) and its record count (high
 * bits): zero-filled before the first call, as cell_count is for lss_csr_build_ws, and left
 * zero-filled by every lss_csr_build_ordered. `lists`: lss_csr_lists_bytes(ncells, nprime) bytes,
 * 16-B aligned, no initialisation. `workspace`: as lss_csr_build_ws's (its word 0 counts overflow
 * records: cells shared by more than 8 blocks). A sample may hold fewer than 2^20 - 512 points
 * (N*D*H*W, or points_per_batch); larger returns LSS_EUNSUPPORTED (use lss_geometry_cells +
 * lss_csr_build_ws). One plan at a time per (cell_word, lists, workspace).
 * Replaces: ranks = ...; sorts = ranks.argsort(); x, geom_feats, ranks = x[sorts], ... (src/models.py:225-231). */
size_t lss_csr_lists_bytes(int32_t ncells, int32_t nprime);
int lss_geometry_cells_ordered(const float* frustum, const float* rots, const float* trans,
                               const float* kinv, const float* pinv, const float* post_trans,
                               const lss_dims_t* dims, const lss_grid_t* grid,
                               float* out_geom, int32_t* cell_of, int32_t* cell_word, int32_t* rank_of,
                               void* lists, void* workspace, lss_stream_t stream);
int lss_cells_from_geom_ordered(const float* geom, int32_t nprime, int32_t points_per_batch,
                                const lss_grid_t* grid, int32_t* cell_of, int32_t* cell_word,
                                int32_t* rank_of, void* lists, void* workspace, lss_stream_t stream);
int lss_csr_build_ordered(const int32_t* cell_of, const int32_t* rank_of, int32_t nprime,
                          int32_t* cell_word, int32_t ncells, const lss_dims_t* dims, const void* lists,
                          int32_t* cell_start, long long* sorted_key, int32_t* sorted_row,
                          void* workspace, lss_stream_t stream);

/* Lift, part 1 (CamEncode.get_depth_dist + layout, src/models.py:49-59, 192-202):
 * depth (B*N, D, H, W) fp32 = softmax over D of depthnet_out[:, :D];
 * ctx_t (B*N*H*W, C), element type ctx_dtype = depthnet_out[:, D:D+C] moved to pixel-major rows
 * (bf16 rows are exact when depthnet_out is bf16, as under autocast).
 * depthnet_out is (B*N, D+C, H, W) contiguous, element type in_dtype. */
int lss_lift_prep(const void* depthnet_out, int32_t in_dtype, const lss_dims_t* dims,
                  float* depth, void* ctx_t, int32_t ctx_dtype, lss_stream_t stream);

/* Depthnet + lift, part 1, fused (CamEncode.depthnet 1x1 conv + get_depth_dist + layout,
 * src/models.py:47, 55-59, 192-202): logits = weight . feat + bias on MFMA (bf16 in, fp32
 * accumulate, rounded to bf16 like the autocast conv output), depth (B*N, D, H, W) fp32 = softmax
 * over the first D logits, ctx_t (B*N*H*W, C) bf16 = the last C logits as pixel-major rows. The
 * depthnet output (B*N, D+C, H, W) is never written. feat (B*N, K, H, W) contiguous, weight
 * (D+C, K) row-major, bias (D+C); dtype and ctx_dtype must be LSS_BF16; K % 16 == 0, K <= 512,
 * D + C <= 128 (else LSS_EUNSUPPORTED). The backward stays the conv's: d(logits) from
 * lss_splat_bwd feeds the 1x1 conv's weight / input gradients. */
int lss_depthnet_lift(const void* feat, const void* weight, const void* bias, int32_t dtype, int32_t K,
                      const lss_dims_t* dims, float* depth, void* ctx_t, int32_t ctx_dtype, lss_stream_t stream);

/* As lss_depthnet_lift, with feat channels-last: (B*N, H, W, K) = pixel-major rows of K bf16 (the
 * memory of a torch.channels_last (B*N, K, H, W) tensor, as a channels-last Up stage produces it).
 * K must be 512; feat and weight 16-B aligned (else LSS_EINVAL). One block per compute unit, each
 * on one contiguous run of pixel rows; identical results to lss_depthnet_lift on the same values. */
int lss_depthnet_lift_nhwc(const void* feat, const void* weight, const void* bias, int32_t dtype, int32_t K,
                           const lss_dims_t* dims, float* depth, void* ctx_t, int32_t ctx_dtype, lss_stream_t stream);

/* The depthnet weights for lss_depthnet_lift_nhwc_packed (CamEncode.depthnet.weight / .bias,
 * src/models.py:47, as the autocast conv would see them): weight (O, K) row-major and bias (O) of
 * `dtype` (LSS_F32 or LSS_BF16) rounded to bf16 (nearest even, as torch's .to(torch.bfloat16)) into
 * `packed` (LSS_DN_PACKED_BYTES(K) bytes, 16-B aligned: the lift kernel's MFMA A fragments in the
 * order one wave-instruction reads them), and, when non-NULL, `plain` (O*K bf16 row-major, 16-B
 * aligned) and `bias_out` (O bf16). K % 32 == 0, K <= 512, O <= 128 (else LSS_EUNSUPPORTED). */
#define LSS_DN_PACKED_BYTES(K) ((size_t)(K) * 256)
int lss_depthnet_pack(const void* weight, const void* bias, int32_t dtype, int32_t O, int32_t K, void* packed,
                      void* plain, void* bias_out, lss_stream_t stream);

/* Mixed-precision working copy of flat fp32 master parameters (lss_carla_amd.flat_params): dst[i] =
 * bf16(src[i]) for i < n (nearest even, as torch's .to(torch.bfloat16)); with `packed` non-NULL the
 * same launch also writes the depthnet weight (O, K) fp32 at dn_weight (a range of src) as
 * lss_depthnet_pack does -- the plain bf16 copy and the bias are ranges of dst. src, dst, packed
 * 16-B aligned. */
int lss_flat_cast_bf16(const float* src, void* dst, int64_t n, const float* dn_weight, int32_t O, int32_t K,
                       void* packed, lss_stream_t stream);

/* lss_depthnet_lift_nhwc with the weights as lss_depthnet_pack wrote them (bias: O bf16);
 * identical results. */
int lss_depthnet_lift_nhwc_packed(const void* feat, const void* packed, const void* bias, int32_t K,
                                  const lss_dims_t* dims, float* depth, void* ctx_t, int32_t ctx_dtype,
                                  lss_stream_t stream);

/* Splat forward: segmented per-cell sum written as the dense (B, Z*C, X, Y) BEV
 * (voxel_pooling + QuickCumsum.forward + griddify, src/models.py:233-246,
 * src/tools.py:195-209). Fused mode (x_rows == NULL): contribution of point p to
 * channel c is depth[p] * ctx_t[q(p), c] (the lift's outer product, never
 * materialised; ctx_t of element type ctx_dtype). Lifted mode (depth == ctx_t == NULL):
 * x_rows is (Nprime, C) fp32. Points of a cell are summed in ascending point id, in fp32, one
 * rounded multiply and add per point (deterministic; both layouts give identical bits). Empty
 * cells are written as zeros; every element of out is written once. LSS_NHWC: one wave per
 * 64-entry chunk of the CSR (one gather round trip, LDS-staged ordered sums, rows stored
 * directly) plus zero-fill waves; LSS_NCHW: a BEV-row tile kernel (<= 128 cells per tile along Y)
 * with an LDS transpose. sorted_key / sorted_row as lss_csr_build wrote them (sorted_row is
 * unused in lifted mode, where the rows are the point ids).
 * ev_start / ev_stop (nullable) are stamped with the kernel's own start / end
 * (hipExtLaunchKernel), so their elapsed time is the kernel alone, never launch latency. */
int lss_splat_fwd(const float* depth, const void* ctx_t, int32_t ctx_dtype, const float* x_rows,
                  const int32_t* cell_start, const long long* sorted_key, const int32_t* sorted_row,
                  const lss_dims_t* dims, const lss_grid_t* grid, void* out, int32_t out_dtype,
                  int32_t out_layout, lss_stream_t stream, lss_event_t ev_start, lss_event_t ev_stop);

/* Backward helpers. A "row" is the C gradient values of one cell.
 * lss_bev_rows: NCHW dbev -> rows[cell*C + c] for every occupied cell (others untouched). */
int lss_bev_rows(const void* dbev, int32_t g_dtype, const int32_t* cell_start,
                 const lss_dims_t* dims, const lss_grid_t* grid, void* rows, lss_stream_t stream);

/* Fused splat + lift backward (QuickCumsum.backward gather, src/tools.py:212-219,
 * then the outer-product and softmax backward of src/models.py:58-59):
 * d_depthnet_out (B*N, D+C, H, W), element type d_dtype. rows_layout LSS_NHWC means
 * g is the channels-last dbev itself; LSS_NCHW means g is the rows buffer of lss_bev_rows. */
int lss_splat_bwd(const void* g, int32_t g_dtype, int32_t rows_layout, const int32_t* cell_of,
                  const float* depth, const void* ctx_t, int32_t ctx_dtype, const lss_dims_t* dims,
                  const lss_grid_t* grid, void* d_depthnet_out, int32_t d_dtype,
                  lss_stream_t stream);

/* Lifted-mode backward: dx[p, c] = g_row(cell_of[p])[c], 0 for dropped points (Nprime, C) fp32. */
int lss_splat_bwd_lifted(const void* g, int32_t g_dtype, int32_t rows_layout, const int32_t* cell_of,
                         int32_t nprime, const lss_dims_t* dims, const lss_grid_t* grid,
                         float* dx, lss_stream_t stream);

/* ---- The reference's op-level boundary: QuickCumsum / cumsum_trick (src/tools.py:182-219).
 * Rows x (n, C) fp32 sorted by an int64 rank (src/models.py:226-231); one output row per run of
 * equal ranks.
 * lss_segment_build: seg_of[i] (n) = run index of row i; seg_start (n + 1 capacity) = first row of
 *   each run, seg_start[nseg] = n; nseg (1 int, device) = number of runs. Replaces
 *   `kept[:-1] = ranks[1:] != ranks[:-1]` and QuickCumsum.backward's `cumsum(kept) - 1`
 *   (src/tools.py:197-198, 214-215). scratch: lss_segment_scratch_bytes(n) bytes. n > 0.
 * lss_segment_sum: out[j] (nseg, C) = sum of the rows of run j in row order (fp32);
 *   key_out[j] (nseg, key_width) = keys row of the run's last row -- geom_feats[kept]
 *   (src/tools.py:200); keys may be NULL. Replaces QuickCumsum.forward / cumsum_trick
 *   (src/tools.py:182-209).
 * lss_segment_gather: dx[i] = g[seg_of[i]] (n, C) -- QuickCumsum.backward (src/tools.py:212-219). */
size_t lss_segment_scratch_bytes(int32_t n);
int lss_segment_build(const long long* ranks, int32_t n, int32_t* seg_of, int32_t* seg_start, int32_t* nseg,
                      void* scratch, lss_stream_t stream);
int lss_segment_sum(const float* x, int32_t C, const int32_t* seg_start, int32_t nseg, const long long* keys,
                    int32_t key_width, long long* key_out, float* out, lss_stream_t stream);
int lss_segment_gather(const float* g, int32_t C, const int32_t* seg_of, int32_t n, float* dx,
                       lss_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* LSS_HIP_H */

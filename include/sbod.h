/*
 * sbod.h — C ABI of libsbod_hip.so, the gfx950 (MI355X) implementation of the
 * shape_based_object_detection hot path: anchor matching, detection losses, box decode + NMS
 * and DeformConv2d.
 *
 * Conventions:
 *   - every pointer is a DEVICE pointer unless documented otherwise; the caller owns all memory
 *     (outputs and workspaces are allocated by the caller, e.g. from torch's caching allocator);
 *   - every call is asynchronous on `stream` (a hipStream_t passed as void*); nothing here
 *     allocates, frees or synchronises, so every call is hipGraph-capturable;
 *   - return SBOD_OK (0) or a negative sbod_status; sbod_last_error() then holds a message
 *     (thread-local).  Nothing throws across the ABI;
 *   - ragged per-image ground truth is packed as gt_boxes [sum(G_i), 4] float32 xyxy,
 *     gt_labels [sum(G_i)] int64 and gt_offsets [B + 1] int32 (image b owns rows
 *     gt_offsets[b] .. gt_offsets[b+1]-1) — the collate_fn list-of-tensors batch of
 *     dataset/Datasets.py:58-86, concatenated once per step;
 *   - load after `import torch` so SONAME libamdhip64.so.7 binds to torch's HIP runtime.
 *
 * Each entry point cites the reference Python interface it replaces (file:line in the
 * upstream repository).
 */
#ifndef SBOD_H
#define SBOD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SBOD_ABI_VERSION 4

typedef enum sbod_status {
  SBOD_OK = 0,
  SBOD_E_INVALID = -1,      /* bad argument / shape */
  SBOD_E_HIP = -2,          /* HIP runtime error (launch failure) */
  SBOD_E_WORKSPACE = -3,    /* workspace too small */
  SBOD_E_UNSUPPORTED = -4   /* size beyond what this build supports (message says which) */
} sbod_status;

/* ---------------------------------------------------------------- library */
const char *sbod_version(void);
int sbod_abi_version(void);
const char *sbod_last_error(void);
/* Compile-time variants built into this library (bit mask): SBOD_VARIANT_ONE_LAUNCH_CRITERION =
 * the one-launch focal criterion of sbod_criterion_focal (A/B builds only,
 * scripts/build_variant_lib.sh; the product library has none and always runs two launches). */
enum { SBOD_VARIANT_ONE_LAUNCH_CRITERION = 1 };
int sbod_build_variants(void);

/* Kernel timing for benchmarks: kernel_filter = a kernel name ("k_det_prepare"), "*" for every
 * instrumented kernel, or NULL / "" to stop.  Each call clears previous records.  Matching
 * launches are bracketed by HIP events on their own stream; sbod_timing_query() waits for them
 * and returns the number of timed launches and their summed duration in milliseconds. */
int sbod_timing_enable(const char *kernel_filter);
int sbod_timing_query(const char *kernel, int *launches, double *total_ms);
/* Time only one launch in n of each selected kernel (n >= 1, default 1; resets the per-kernel
 * launch counts).  Timed launches carry their events on the dispatch itself
 * (hipExtLaunchKernelGGL), which costs host time per timed launch; sampling keeps that out of
 * most steps of a benchmark. */
int sbod_timing_every(int n);
/* Under hipGraph stream capture a dispatch cannot carry events (and this runtime refuses
 * external event nodes): a selected HBM-bound kernel (k_match_tile, k_multibox, k_det_prepare)
 * is instead captured with a device span record that the kernel itself overwrites on every
 * replay — each workgroup's start, and its end after its stores are acknowledged, in
 * s_memrealtime ticks (plain per-workgroup stores: no atomics, no host writes between
 * replays).  sbod_timing_query() then reports the latest completed replay's first-start to
 * last-end span.  The capture records survive sbod_timing_enable();
 * sbod_timing_reset_graphs() releases (and clears) them once the graphs holding them are gone. */
double sbod_timing_clock_hz(void);   /* the span clock (hipDeviceAttributeWallClockRate) */
int sbod_timing_reset_graphs(void);

/* An empty kernel of `blocks` 64-thread workgroups (profiling calibration: the per-dispatch
 * cost a profiler adds to every kernel it traces). */
int sbod_null_kernel(int blocks, void *stream);

/* Asynchronous device -> host copy on `stream` (hipMemcpyAsync; dst_host should be pinned, e.g.
 * torch's pin_memory buffers).  Used for detect's per-image counts (the one value the host needs
 * from a detect call, models/utils.py:274-290); the caller orders its host read after an event
 * recorded behind it.  Cheaper on the host than a framework-level non_blocking copy. */
int sbod_memcpy_d2h_async(void *dst_host, const void *src_dev, size_t bytes, void *stream);

/* Replay of a captured step without a framework round trip per call: launch an instantiated
 * hipGraphExec_t on `stream` (torch: CUDAGraph.raw_cuda_graph_exec()), and record a hipEvent_t
 * (torch: Event.cuda_event) on `stream`.  Used by the host extension's one-call step submit
 * (GT packing + the criterion and detect graphs on their streams + the detect event). */
int sbod_graph_launch(void *graph_exec, void *stream);
int sbod_event_record(void *event, void *stream);

/* Stream ordering for work handed between streams (no host sync): everything queued on
 * `on_stream` so far completes before anything queued on `waiting_stream` after this call.
 * A no-op when both are the same stream. */
int sbod_stream_wait(void *waiting_stream, void *on_stream);

/* End a stream capture that a failed capture left open (an error inside the captured region can
 * leave the stream capturing, and then every later call on it fails): ends it if `stream` is
 * capturing and discards the graph; a no-op otherwise.  Returns SBOD_OK, or SBOD_E_HIP when the
 * status cannot be read or the stream is still capturing afterwards (ROCm 7.2 keeps an
 * INVALIDATED capture open: such a stream cannot be reused; the caller moves to a fresh one). */
int sbod_stream_abort_capture(void *stream);

/* ---------------------------------------------------------------- f1: ground-truth packing
 * Replaces the per-step GT handling of every criterion: the collate_fn list-of-tensors batch
 * (dataset/Datasets.py:58-86), moved to the device image by image (train_anchor.py:266-268) and
 * indexed per image in the matching loop (models/SSD512.py:525-572).  One launch copies image
 * i's `counts[i]` rows from the DEVICE pointers box_ptrs[i] ([G_i,4] f32) / label_ptrs[i]
 * ([G_i] int64) into gt_boxes / gt_labels back to back and writes gt_offsets [B+1].
 * box_ptrs, label_ptrs and counts are HOST arrays of B entries (they travel in the kernel
 * arguments: no device pointer table, no host->device copy).  `capacity` = rows available in
 * gt_boxes / gt_labels (a fixed-capacity destination can be read by a captured hipGraph). */
int sbod_gt_pack(const void *const *box_ptrs, const void *const *label_ptrs,
                 const int32_t *counts, int B, int64_t capacity, float *gt_boxes,
                 int64_t *gt_labels, int32_t *gt_offsets, void *stream);

/* ---------------------------------------------------------------- a1 / a4: pairwise IoU
 * Replaces metrics.find_jaccard_overlap (metrics.py:208-252; mode SBOD_IOU_METRICS: +1e-5
 * denominator, zero-GT -> 0, zero-anchor -> -1) and iou_utils.jaccard (iou_utils.py:215-233;
 * mode SBOD_IOU_PLAIN).  out[b, g, p] for g < G_b; rows g >= G_b are left untouched.
 * anchors: [P,4] xyxy shared when anchor_batch_stride == 0, else image b reads
 * anchors + b * anchor_batch_stride (elements). */
enum { SBOD_IOU_METRICS = 0, SBOD_IOU_PLAIN = 1, SBOD_IOU_INTER = 2 /* intersection areas */ };
int sbod_iou_pairwise_f32(const float *gt_boxes, const int32_t *gt_offsets, int B, int Gmax,
                          const float *anchors, int64_t anchor_batch_stride, int P, int mode,
                          float *out, void *stream);

/* ---------------------------------------------------------------- a2 / a3: anchor matching
 * Replaces the per-image matching block of every criterion
 * (models/SSD512.py:532-572, SSD300.py:501-542, RetinaNet.py:409-449,
 *  RefineDet512.py:745-785 (ARM, SBOD_MATCH_BINARY) and :846-886 (ODM, SBOD_MATCH_ODM)):
 * find_jaccard_overlap -> max(dim 0) / max(dim 1) (first index on ties) -> forced match with the
 * FILTERED j, last writer wins -> label / negative thresholds.
 *   anchors: xyxy [P,4] (shared priors_xy); for SBOD_MATCH_ODM `anchors` are the ARM locs
 *            [B,P,4] (gcxgcy) decoded on the fly against priors_cxcy, exactly
 *            cxcy_to_xy(gcxgcy_to_cxcy(arm_locs[i], priors_cxcy)) (RefineDet512.py:850).
 *   arm_scores: [B,P,2] logits, only for SBOD_MATCH_ODM (easy negatives softmax[...,1] < theta).
 *   gt_boxes / gt_labels must hold at least one row even when every image is empty (the
 *   matcher's prologue reads row 0 unconditionally; sbod_gt_pack's callers size them max(n, 1)).
 *   Outputs [B,P]: obj (object per prior, int32), ovl (overlap per prior after the forced match).
 *   n_pos [B+1] int32: positives per image (+ the batch total at n_pos[B]).  Labels and the
 *   negative mask are derived from (obj, ovl, gt_labels) by the loss kernels.
 * Workspace: sbod_match_workspace_bytes(B, Gmax): per-(image, object) best-prior keys and
 * per-wave positive counts, which must be zero on entry.  Every successful call leaves the
 * whole workspace zero, so a caller that knows it is clean (a previous successful call on it,
 * of any shape, or its own memset) passes SBOD_MATCH_WS_ZEROED and the call issues no memset
 * (hipGraph capture); without the flag the call zeroes it first (hipMemsetAsync). */
enum { SBOD_MATCH_BINARY = 1, SBOD_MATCH_ODM = 2, SBOD_MATCH_WS_ZEROED = 256 };
size_t sbod_match_workspace_bytes(int B, int Gmax);          /* enough for P <= 2^20 */
size_t sbod_match_workspace_bytes_p(int B, int Gmax, int P);  /* exact for this P */
int sbod_match_f32(const float *gt_boxes, const int64_t *gt_labels, const int32_t *gt_offsets,
                   int B, int Gmax, const float *anchors, const float *priors_cxcy,
                   const float *arm_scores, int P, float threshold, float theta, int flags,
                   int32_t *obj, float *ovl, int32_t *n_pos, void *workspace,
                   size_t workspace_bytes, void *stream);
/* The list form: sbod_gt_pack + sbod_match_f32 in the matcher's two launches.  The first launch
 * reads each image's rows in place from the collate_fn lists (box_ptrs / label_ptrs / counts as
 * for sbod_gt_pack: HOST arrays of device pointers, carried in the kernel arguments) and also
 * writes them packed into gt_boxes / gt_labels / gt_offsets (capacity rows) for the loss pass
 * that follows.  B <= 64; every image has 1..Gmax objects; boxes 16-B and labels 8-B aligned
 * (what torch's allocator gives).  Callers with other batches use the two calls. */
int sbod_match_lists_f32(const void *const *box_ptrs, const void *const *label_ptrs, const int32_t *counts,
                         int64_t capacity, float *gt_boxes, int64_t *gt_labels, int32_t *gt_offsets, int B,
                         int Gmax, const float *anchors, const float *priors_cxcy, const float *arm_scores, int P,
                         float threshold, float theta, int flags, int32_t *obj, float *ovl, int32_t *n_pos,
                         void *workspace, size_t workspace_bytes, void *stream);

/* Expand matcher outputs to the reference's tensors (for parity tests and the iou_utils API):
 * cls [B,P] int64 (labels[obj], 0 where ovl < threshold; binary -> 0/1),
 * neg [B,P] int64 (labels[obj], -1 where ovl < neg_threshold),
 * true_xy [B,P,4] (gt_boxes[obj]) and enc [B,P,4] (cxcy_to_gcxgcy(xy_to_cxcy(gt[obj]), prior)).
 * Any output pointer may be NULL. */
int sbod_match_expand_f32(const float *gt_boxes, const int64_t *gt_labels,
                          const int32_t *gt_offsets, int B, const int32_t *obj, const float *ovl,
                          const float *priors_cxcy, const float *odm_arm_locs, int P,
                          float threshold, float neg_threshold, int flags, int64_t *cls,
                          int64_t *neg, float *true_xy, float *enc, void *stream);

/* iou_utils.match / match_ious (iou_utils.py:236-321): plain jaccard vs point_form(priors),
 * best-prior fill 2.0, UNFILTERED j, conf = labels + 1.  Writes loc_t[idx] / conf_t[idx]
 * rows (caller passes the row pointers).  encode != 0 -> encode(variances) else raw matches.
 * Workspace: sbod_match_ssd_workspace_bytes(G, P) (0 for non-positive sizes). */
size_t sbod_match_ssd_workspace_bytes(int G, int P);
int sbod_match_ssd_f32(const float *truths, const int64_t *labels, int G,
                       const float *priors_cxcy, int P, float threshold, float var0, float var1,
                       int encode, float *loc_t_row, int64_t *conf_t_row, void *workspace,
                       size_t workspace_bytes, void *stream);

/* ---------------------------------------------------------------- a3: box codecs
 * dataset/transforms.py:26-83 and iou_utils.py:167-177, 324-368.  n rows of 4 floats.
 * priors may be [n,4] or broadcast [P,4] with rows = n (prior_rows > 0 -> row i uses
 * prior i % prior_rows). */
enum { SBOD_CODEC_XY_TO_CXCY = 0, SBOD_CODEC_CXCY_TO_XY = 1, SBOD_CODEC_ENCODE_TENFIVE = 2,
       SBOD_CODEC_DECODE_TENFIVE = 3, SBOD_CODEC_ENCODE_VAR = 4, SBOD_CODEC_DECODE_VAR = 5,
       SBOD_CODEC_DECODE_TENFIVE_XY = 6 };
int sbod_codec_f32(int op, const float *in, const float *priors, int64_t n, int64_t prior_rows,
                   float var0, float var1, float *out, void *stream);

/* ---------------------------------------------------------------- a5-a10: fused criterion
 * One pass over the predictions of every criterion in models/ (*.py): per prior the label is
 * derived from the matcher, the box loss (a5/a6) and class loss (a7/a10) and their gradients
 * are produced together (one read of locs/scores, one write of their gradients).
 *   reg:  SBOD_REG_SMOOTHL1 (Loss.py:203-226, beta 1/9, mean over positive rows),
 *         SBOD_REG_L1 (nn.L1Loss, SSD300.py:465, mean over elements),
 *         SBOD_REG_DIOU (IouLoss 'Corner' Diou on decoded boxes, Loss.py:164-200).
 *   cls:  SBOD_CLS_FOCAL (softmax focal_loss, Loss.py:9-38, rows = positives + negatives),
 *         SBOD_CLS_CE (CrossEntropy + hard-negative mining, a10).
 *   flags: SBOD_LOSS_FOCAL_NORM (divide focal by total positives, RetinaNet.py:471-472),
 *          pool for CE mining: SBOD_POOL_NONPOS (SSD512.py:601-623), SBOD_POOL_NEG
 *          (RetinaNet.py:478-503), SBOD_POOL_GLOBAL_NEG (SSD300.py:567-591),
 *          SBOD_POOL_NONPOS_NOT_EASY (RefineDet512.py:910-936); SBOD_MATCH_BINARY / _ODM as
 *          for the matcher.
 *   locs/scores: [B,P,4] / [B,P,C], dtype float32 (SBOD_DT_F32) or bfloat16 (SBOD_DT_BF16);
 *   grad_locs/grad_scores: same shape and dtype; may be NULL (forward only).
 *   loss_out: device float[4] = {total, conf, loc, n_pos_total}.
 *   npos_total: device int32 pointer to the normaliser (the matcher's n_pos[B], or a
 *   cross-rank all-reduced copy for data parallelism).
 * Workspace: sbod_loss_workspace_bytes(B, P). */
enum { SBOD_REG_SMOOTHL1 = 0, SBOD_REG_L1 = 1, SBOD_REG_DIOU = 2 };
enum { SBOD_CLS_FOCAL = 0, SBOD_CLS_CE = 1 };
enum { SBOD_DT_F32 = 0, SBOD_DT_BF16 = 1 };
enum { SBOD_LOSS_FOCAL_NORM = 4, SBOD_POOL_NONPOS = 0, SBOD_POOL_NEG = 8,
       SBOD_POOL_GLOBAL_NEG = 16, SBOD_POOL_NONPOS_NOT_EASY = 32 };
size_t sbod_loss_workspace_bytes(int B, int P);

/* Data-parallel global mining — the one exchange step of the data-parallel path (SURVEY
 * §8(e)): MultiBoxLoss300's CE mines its hard negatives over the WHOLE batch
 * (models/SSD300.py:580-588), so with the batch sharded over ranks the top-k must see every
 * rank's pool.  Call sbod_multibox_loss with flags | SBOD_LOSS_DEFER_MINING (CE +
 * SBOD_POOL_GLOBAL_NEG only): it runs the fused pass and leaves this rank's pool [B*P] f32
 * (CE of pool members, -1 otherwise) at workspace + sbod_loss_pool_offset(B, P).  The caller
 * all-gathers the pools rank-major (equal B on every rank) and calls
 * sbod_multibox_mine_global with the gathered pool and this rank's offset in it: threshold,
 * tie order (lowest global index first) and k = ratio * npos_total are those of one device
 * holding the whole batch; the hard-negative gradients and the loss cover this rank's rows
 * (the sum over ranks is the single-device loss).  Same workspace as the deferred call. */
enum { SBOD_LOSS_DEFER_MINING = 64 };
/* Focal criteria (no mining pass) finish the loss inside the fused pass: every workgroup
 * publishes its fp32 partials as one tagged 16-byte record and the grid's last workgroup sums
 * all of them exactly, as 128-bit fixed-point integers (2^-64 resolution; a partial that is
 * non-finite or >= 2^40 in magnitude switches the finish to a double sum of the fp32 partials in
 * record order, as the separate finaliser computes it).  The finish's state — a few words and the
 * records — is the workspace's first sbod_loss_zero_bytes(B, P) bytes: zero on entry, and left
 * zero by every successful call (so any smaller prefix stays zero too).  A caller that knows that
 * passes SBOD_LOSS_WS_ZEROED and the call issues no memset (hipGraph capture); without it the
 * call zeroes them first (one hipMemsetAsync).  A finish whose wait for the records timed out
 * (2 s: a hardware fault) makes this and every later loss on the workspace NaN until it is zeroed.
 * SBOD_LOSS_UNFUSED_FINISH finishes a focal criterion with the separate one-block finaliser
 * launch instead (the same exact sum: the same loss bit for bit). */
enum { SBOD_LOSS_WS_ZEROED = 128, SBOD_LOSS_UNFUSED_FINISH = 512 };
size_t sbod_loss_zero_bytes(int B, int P);
size_t sbod_loss_pool_offset(int B, int P);
int sbod_multibox_mine_global(const void *scores, int dtype, int B, int P, int C,
                              const int32_t *npos_total, int reg, int cls, int flags,
                              int neg_pos_ratio, float reg_weight, const float *pool_all,
                              int64_t n_all, int64_t local_off, void *grad_scores,
                              float *loss_out, void *workspace, size_t workspace_bytes,
                              void *stream);
int sbod_multibox_loss(const void *locs, const void *scores, int dtype, int B, int P, int C,
                       const float *priors_cxcy, const float *odm_arm_locs,
                       const float *arm_scores, const float *gt_boxes, const int64_t *gt_labels,
                       const int32_t *gt_offsets, const int32_t *obj, const float *ovl,
                       const int32_t *n_pos, const int32_t *npos_total, float threshold,
                       float neg_threshold, float theta, int reg, int cls, int flags,
                       int neg_pos_ratio, float reg_weight, float focal_alpha, float focal_gamma,
                       void *grad_locs, void *grad_scores, float *loss_out, void *workspace,
                       size_t workspace_bytes, void *stream);

/* One-launch focal criterion: the matcher (sbod_match_f32 with shared priors) and the fused
 * focal pass (sbod_multibox_loss, cls = SBOD_CLS_FOCAL) in ONE launch — MultiBoxLoss512 /
 * MultiBoxLoss300 / RetinaFocalLoss with cls_loss 'focal' on one device
 * (models/SSD512.py:508-626, SSD300.py:477-594, RetinaNet.py:385-506).  Every workgroup matches
 * its 256 priors, the last tile of each image runs that image's forced match, and every
 * workgroup waits (in the launch) until all images are counted in before it applies its priors'
 * forced rewrites and computes its rows' losses and gradients scaled by the batch's positives.
 * Same outputs as the two calls: obj / ovl [B,P], n_pos [B+1] (n_pos[B] = the batch total),
 * grad_locs / grad_scores (may be NULL), loss_out {total, conf, loc, n_pos}.
 * The grid (B * ceil(P/256) workgroups) must be resident at once; when the occupancy query says
 * it is not (or with SBOD_CRIT_TWO_LAUNCH / SBOD_LOSS_UNFUSED_FINISH) the call runs the two
 * launches instead, on the same workspace, with the same results.  The one-launch form exists
 * only in a variant library (sbod_build_variants() & SBOD_VARIANT_ONE_LAUNCH_CRITERION): its
 * workgroups wait for each other, which stalls when other streams' kernels hold CUs (measured,
 * DESIGN.md round 4); the product library always runs the two launches.  Data parallelism (a
 * normaliser all-reduced between the matcher and the loss) uses the two calls.
 * Workspace: sbod_criterion_workspace_bytes(B, Gmax, P); its first
 * sbod_criterion_zero_bytes(B, Gmax, P) bytes must be zero on entry and are left zero by every
 * successful call: pass SBOD_CRIT_WS_ZEROED when they are (else the call zeroes them, one
 * hipMemsetAsync).  flags: SBOD_LOSS_FOCAL_NORM, SBOD_CRIT_WS_ZEROED, SBOD_CRIT_TWO_LAUNCH,
 * SBOD_LOSS_UNFUSED_FINISH.  sbod_criterion_status() (diagnostics, synchronises the stream) reads
 * the sticky word the one-launch form sets if a bounded in-launch wait ever gave up (that call's
 * loss and its waiting workgroups' gradients are NaN; the next call starts clean). */
enum { SBOD_CRIT_WS_ZEROED = 128, SBOD_CRIT_TWO_LAUNCH = 1024 };
size_t sbod_criterion_workspace_bytes(int B, int Gmax, int P);
size_t sbod_criterion_zero_bytes(int B, int Gmax, int P);
int sbod_criterion_focal(const void *locs, const void *scores, int dtype, int B, int P, int C,
                         const float *priors_cxcy, const float *priors_xy, const float *gt_boxes,
                         const int64_t *gt_labels, const int32_t *gt_offsets, int Gmax, float threshold,
                         float neg_threshold, int reg, int flags, float reg_weight, float focal_alpha,
                         float focal_gamma, int32_t *obj, float *ovl, int32_t *n_pos, void *grad_locs,
                         void *grad_scores, float *loss_out, void *workspace, size_t workspace_bytes,
                         void *stream);
/* The focal criterion reading the collate_fn lists: sbod_gt_pack + sbod_criterion_focal's
 * two-launch form (sbod_match_lists_f32, then the fused focal pass) — one launch fewer per step.
 * List arguments and limits as sbod_match_lists_f32; gt_boxes / gt_labels / gt_offsets are the
 * packed OUTPUT (capacity rows); the rest as sbod_criterion_focal (SBOD_CRIT_TWO_LAUNCH implied). */
int sbod_criterion_focal_lists(const void *const *box_ptrs, const void *const *label_ptrs, const int32_t *counts,
                               int64_t capacity, const void *locs, const void *scores, int dtype, int B, int P,
                               int C, const float *priors_cxcy, const float *priors_xy, float *gt_boxes,
                               int64_t *gt_labels, int32_t *gt_offsets, int Gmax, float threshold,
                               float neg_threshold, int reg, int flags, float reg_weight, float focal_alpha,
                               float focal_gamma, int32_t *obj, float *ovl, int32_t *n_pos, void *grad_locs,
                               void *grad_scores, float *loss_out, void *workspace, size_t workspace_bytes,
                               void *stream);
int sbod_criterion_status(const void *workspace, void *stream);
/* The fused loss finish's sticky word (diagnostics, synchronises the stream): 1 if a bounded gather
 * wait ever gave up on this workspace (every later loss from it is NaN until its zero-on-entry
 * prefix is zeroed again: one call without SBOD_LOSS_WS_ZEROED / SBOD_CRIT_WS_ZEROED), else 0.
 * Gmax == 0: a sbod_multibox_loss workspace; Gmax > 0: a sbod_criterion_focal one of (B, Gmax, P). */
int sbod_loss_finish_status(const void *workspace, int B, int Gmax, int P, void *stream);

/* grad *= (*scale) in place unless *scale == 1 (decided on the device: no host sync).
 * Used by backward to apply the upstream gradient to gradients produced by the fused
 * forward. */
int sbod_scale_inplace(void *grad, int dtype, int64_t n, const float *scale, void *stream);
int sbod_scale2_inplace(void *a, int64_t na, void *b, int64_t nb, int dtype, const float *scale,
                        void *stream);  /* both buffers, one launch */

/* ---------------------------------------------------------------- a5/a6/a7/a8/a9 standalone
 * The operators.Loss / iou_utils API on already-selected rows.  Each call writes the per-row
 * (or per-element) values and their local derivatives; the Python layer applies the
 * reference's own reductions (Loss.py:192-200, 219-226, 38, 80, 103) through autograd.
 *   aligned overlap (iou_utils.py:6-164): overlap [n], d overlap / d b1 [n,4] and d overlap /
 *     d b2 [n,4] (either gradient may be NULL; autograd reaches both box sets in the reference);
 *     the reference's clamp masks and its min/max tie rule (gradient split in half).
 *   smooth L1 (Loss.py:213-217): loss [n] and d loss / d pred [n] per element.
 *   focal (Loss.py:9-38 softmax, :41-80 sigmoid, :83-103 bce): loss [rows] and
 *     d loss / d logits [rows, C]. */
enum { SBOD_OV_IOU = 0, SBOD_OV_GIOU = 1, SBOD_OV_DIOU = 2, SBOD_OV_CIOU = 3 };
int sbod_aligned_overlap_f32(int kind, const float *b1, const float *b2, int64_t n,
                             float *overlap, float *grad_b1, float *grad_b2, void *stream);
int sbod_smooth_l1_f32(const float *pred, const float *target, int64_t n, float beta,
                       float *loss, float *grad, void *stream);
enum { SBOD_FOCAL_SOFTMAX = 0, SBOD_FOCAL_SIGMOID = 1, SBOD_FOCAL_BCE = 2 };
int sbod_focal_f32(int kind, const float *logits, const int64_t *target, int64_t rows, int C,
                   float alpha_fg, float alpha_bg, float gamma, float *row_loss, float *grad,
                   void *stream);

/* ---------------------------------------------------------------- a11-a13: decode + NMS
 * Replaces models/utils.py:181-297 (detect), detect_scripts/detect_tools.py:100-341
 * (detect / detect_refine, final class-agnostic NMS) and the torchvision.ops.nms it calls
 * (torchvision semantics: descending stable order, suppress IoU > thr).
 *   box_type: SBOD_BOX_OFFSET (gcxgcy vs priors), SBOD_BOX_CENTER (cxcy), SBOD_BOX_CORNER
 *             (xyxy; clamped IN PLACE into `locs`, the reference's clamp_ quirk).
 *   act: SBOD_ACT_SOFTMAX | SBOD_ACT_SIGMOID.
 *   pos_mask: [B,P] uint8 (prior_positives_idx) or NULL.
 *   Outputs: det_boxes [B,top_k,4], det_labels [B,top_k] int64, det_scores [B,top_k],
 *            det_count [B] int32 (rows beyond count are unspecified);
 *            det_count_host: NULL, or a device-accessible PINNED host buffer [B] int32 (e.g. torch
 *            pin_memory / hipHostMalloc) that the last kernel also writes det_count into — the
 *            caller reads it after an event recorded behind the call, with no copy launch;
 *            debug_probs [B,P,C] / debug_boxes [B,P,4] may be NULL.
 *   final_nms < 0 disables the detect_tools final class-agnostic NMS.
 *   window: per-class candidate window (0 = auto: next_pow2(top_k + 1)).  Only the first top_k
 *   outputs are observable, so NMS runs on each class's best `window` candidates; when a
 *   candidate outside a truncated window could still reach the output, det_count[b] = -1 and the
 *   caller re-runs with a larger window (results never depend on the window size).
 *   flags: SBOD_DETECT_COUNTERS_ZEROED — the caller guarantees that the workspace's first
 *   sbod_detect_counter_bytes(B, C) bytes are zero on entry (e.g. the workspace was allocated
 *   zeroed); every call leaves them zero again, so repeated calls (and a captured hipGraph)
 *   need no memset.  Without the flag the call zeroes them itself (one memset).
 *   SBOD_DETECT_INPUT_BF16 — locs and scores hold bf16 (C <= 32): each value is widened to fp32
 *   exactly on load, so the results equal those of the fp32 call on the widened tensors (no
 *   widened copies in HBM).  Without it both are fp32.
 *   The per-class NMS and the per-image merge run as two launches, the merge running a wider
 *   second window inline for a class whose first window was truncated.  SBOD_DETECT_FUSED (ABI 4;
 *   opt-in) runs them as ONE launch when there is no final NMS (window 0, C <= 64): the image's
 *   last class merges, and an image its first window of 64 candidates per class cannot decide
 *   reports det_count -1 (the caller re-runs it with a wider window).
 *   Every kernel after k_det_prepare decodes prior indices from candidate keys; an index >= P
 *   (a corrupted or stale candidate region) is never dereferenced: the image reports
 *   det_count -2 (SBOD_DETECT_CORRUPT) and its outputs are unspecified.
 * Workspace: sbod_detect_workspace_bytes(B, P, C). */
enum { SBOD_BOX_OFFSET = 0, SBOD_BOX_CENTER = 1, SBOD_BOX_CORNER = 2 };
enum { SBOD_DETECT_COUNTERS_ZEROED = 1, SBOD_DETECT_INPUT_BF16 = 2, SBOD_DETECT_FUSED = 8 };
enum { SBOD_DETECT_CORRUPT = -2 };
size_t sbod_detect_counter_bytes(int B, int C);
enum { SBOD_ACT_SOFTMAX = 0, SBOD_ACT_SIGMOID = 1 };
size_t sbod_detect_workspace_bytes(int B, int P, int C);
int sbod_detect_f32(void *locs, const void *scores, int B, int P, int C,
                    const float *priors_cxcy, const uint8_t *pos_mask, int box_type, int act,
                    float min_score, float max_overlap, int top_k, float final_nms, int window,
                    int flags, float *det_boxes, int64_t *det_labels, float *det_scores,
                    int32_t *det_count, int32_t *det_count_host, float *debug_probs,
                    float *debug_boxes, void *workspace, size_t workspace_bytes, void *stream);

/* Single-segment greedy NMS (iou_utils.nms / diounms, iou_utils.py:385-530; torchvision.ops.nms).
 *   variant: SBOD_NMS_TV (union (a_i + a_j) - inter, suppress iff IoU > thr),
 *            SBOD_NMS_REF (iou_utils.nms: union (a_j - inter) + a_i, keep iff IoU <= thr,
 *                          the top_k highest kept BEFORE suppression),
 *            SBOD_NMS_DIOU (iou_utils.diounms incl. its center_y2 quirk, beta1 exponent).
 *   keep [n] int64 (indices, descending score), count [1] int32. top_k <= 0: no truncation. */
enum { SBOD_NMS_TV = 0, SBOD_NMS_REF = 1, SBOD_NMS_DIOU = 2 };
size_t sbod_nms_workspace_bytes(int64_t n);
int sbod_nms_f32(const float *boxes, const float *scores, int64_t n, float overlap, int top_k,
                 int variant, float beta1, int64_t *keep, int32_t *count, void *workspace,
                 size_t workspace_bytes, void *stream);

/* ---------------------------------------------------------------- a14: DeformConv2d
 * operators/Deformable_convolution.py:33-146 (modulated DCNv2, rows|cols offset layout,
 * p_0 starting at 1, floor-before-clamp, border clamp, k x k stride-k bias-free conv).
 *   x [B,C,H,W], offset [B,2k²,Ho,Wo] (p_conv output), mask_logits [B,k²,Ho,Wo] (m_conv
 *   output BEFORE sigmoid, or NULL for modulation=False), weight [O,C,k,k] -> out [B,O,Ho,Wo].
 *   Backward: grad_out -> grad_x, grad_offset, grad_mask_logits, grad_weight (any may be NULL).
 *   The backward writes dcols rows [B*Ho*Wo][k²][C] and gathers dx per input pixel (no float
 *   atomics on dx); the weight gradient is summed from per-pixel-slice partial planes in a fixed
 *   order (bit-reproducible run to run); grad_out and weight must each stay below 2 GiB
 *   (buffer-descriptor range).
 * Workspace: sbod_dcn_workspace_bytes(...) for the backward (it includes the dcols rows,
 * B*Ho*Wo*k²*C*4 bytes); the forward needs only sbod_dcn_fwd_workspace_bytes(...) (coefficients,
 * channels-last x and the transposed weights — a prefix of the backward's layout, so one
 * workspace sized for the backward serves both).
 * Streams: all work is ordered on `stream` as for any entry point.  An eager (not capturing)
 * call with B*Ho*Wo*O >= 2^24 runs its independent branches on an internal side stream of the
 * calling host thread, forked from and joined back into `stream` with events before it returns;
 * a call under hipGraph capture stays on `stream`. */
size_t sbod_dcn_workspace_bytes(int B, int C, int H, int W, int O, int k, int stride, int pad);
size_t sbod_dcn_fwd_workspace_bytes(int B, int C, int H, int W, int O, int k, int stride, int pad);
int sbod_dcn_fwd_f32(const float *x, const float *offset, const float *mask_logits,
                     const float *weight, int B, int C, int H, int W, int O, int k, int stride,
                     int pad, float *out, void *workspace, size_t workspace_bytes, void *stream);
int sbod_dcn_bwd_f32(const float *x, const float *offset, const float *mask_logits,
                     const float *weight, const float *grad_out, int B, int C, int H, int W,
                     int O, int k, int stride, int pad, float *grad_x, float *grad_offset,
                     float *grad_mask_logits, float *grad_weight, void *workspace,
                     size_t workspace_bytes, void *stream);
/* Training form (what an autograd Function binds; Deformable_convolution.py:33-91 forward and its
 * autograd backward).  The forward derives, once, everything the backward re-uses — per-(pixel,
 * kernel point) coefficients, channels-last x, both weight layouts, per-input-pixel sample counts —
 * into a caller-owned STATE buffer (sbod_dcn_state_bytes) that must stay unchanged until the
 * backward; the backward reads it (never writes it: a retained graph may run it twice) and
 * works in SCRATCH (sbod_dcn_scratch_bytes, reusable across calls in stream order).
 * grad_mask_logits must be NULL when the forward had no mask.  The stateless
 * sbod_dcn_bwd_f32 above re-derives the state in its own workspace (state + scratch). */
size_t sbod_dcn_state_bytes(int B, int C, int H, int W, int O, int k, int stride, int pad);
size_t sbod_dcn_scratch_bytes(int B, int C, int H, int W, int O, int k, int stride, int pad);
int sbod_dcn_fwd_train_f32(const float *x, const float *offset, const float *mask_logits,
                           const float *weight, int B, int C, int H, int W, int O, int k, int stride,
                           int pad, float *out, void *state, size_t state_bytes, void *stream);
int sbod_dcn_bwd_state_f32(const float *grad_out, int B, int C, int H, int W, int O, int k, int stride,
                           int pad, float *grad_x, float *grad_offset, float *grad_mask_logits,
                           float *grad_weight, const void *state, size_t state_bytes, void *scratch,
                           size_t scratch_bytes, void *stream);

/* ---------------------------------------------------------------- f2: VOC 11-point mAP
 * metrics.calculate_mAP (metrics.py:8-145).  Detections and ground truth are the concatenated
 * per-image lists: det_offsets / true_offsets [B+1] int32 give each image's row range.
 *   det_boxes [D,4] f32 xyxy, det_labels [D] int64, det_scores [D] f32;
 *   true_boxes [T,4] f32, true_labels [T] int64, true_difficulties [T] uint8 (0/1);
 *   threshold: IoU threshold, compared against the float32 IoU promoted to double (:108);
 *   recall_thresholds: device float[11] = torch.arange(0, 1.1, 0.1) (float32, :128).
 * Output: ap [C-1] f32 (class 1..C-1; 0 for classes without detections) and mean_ap [1].
 * Score ties between detections of one class keep input order (the reference's sort is not
 * stable: tie order is unspecified there).  Workspace: sbod_map_workspace_bytes(D, T). */
size_t sbod_map_workspace_bytes(int64_t n_det, int64_t n_true);
int sbod_map_f32(const float *det_boxes, const int64_t *det_labels, const float *det_scores,
                 const int32_t *det_offsets, const float *true_boxes, const int64_t *true_labels,
                 const uint8_t *true_difficulties, const int32_t *true_offsets, int B, int C,
                 int64_t n_det, int64_t n_true, double threshold, const float *recall_thresholds,
                 float *ap, float *mean_ap, void *workspace, size_t workspace_bytes, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* SBOD_H */

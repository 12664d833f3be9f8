// Anchor matching: pairwise IoU (metrics.find_jaccard_overlap / iou_utils.jaccard), the
// criteria's argmax + forced-match + threshold block, and iou_utils.match.
//
// Data layout in HBM: priors are one shared [P,4] xyxy table (read once per tile, L2-resident
// across images); ground truth is ragged [sum G, 4] + offsets; per-prior results are [B,P]
// int32/float32 planes (coalesced).  A tile = 256 priors of ONE image, so every workgroup stages
// its image's G boxes in LDS once and streams its priors.
//
// Roofline: HBM-bound.  Algorithmic bytes per launch (matcher alone) = 16*P (priors once) +
// B*P*8 (obj + ovl written); ~17*G flops per prior-image.
#include "sbod_common.h"

namespace sbod {

SBOD_STAMP_DECL

// Diagnostic build only (-DSBOD_BLOCK_STAMPS, scripts/build_stamps_lib.sh): wave 0 of each
// k_match_tile workgroup records four wall-clock marks while its stamps are armed — 0 the anchors
// reduced to the wave's bounding box, 1 the first object chunk's hit ballot taken (its loads
// landed), 2 the object loop done, 3 the keys flushed — read by sbod_debug_match_marks
// (scripts/match_stamps.py).  Compiles to nothing otherwise.
#ifdef SBOD_BLOCK_STAMPS
static __device__ unsigned long long g_match_marks[SBOD_STAMP_REGION * 4];
#define MATCH_WAVE_MARK(slot, dep)                                                                  \
  do {                                                                                              \
    asm volatile("" ::"v"(dep)); /* the mark follows the value it times */                          \
    if ((g_stamp_armed & (1 << 5)) && threadIdx.x == 0) {                                           \
      const unsigned _b = blockIdx.x + gridDim.x * blockIdx.y;                                      \
      if (_b < SBOD_STAMP_REGION) g_match_marks[_b * 4 + (slot)] = __builtin_amdgcn_s_memrealtime(); \
    }                                                                                               \
  } while (0)
#endif

}  // namespace sbod

#include "match_dev.h"

namespace sbod {

constexpr int kTile = 256;

struct GtTile {
  float x1, y1, x2, y2, area;
  int zero;
};

// metrics.py:224-250 — evaluation order of the reference, one (gt, anchor) pair.
__device__ __forceinline__ float iou_metrics(const GtTile &g, float ax1, float ay1, float ax2,
                                             float ay2, float aarea, bool azero) {
  float iw = fminf(g.x2, ax2) - fmaxf(g.x1, ax1);
  if (iw < 0.f) iw = 0.f;
  float ih = fminf(g.y2, ay2) - fmaxf(g.y1, ay1);
  if (ih < 0.f) ih = 0.f;
  float inner = iw * ih;
  float ov = inner / (((g.area + aarea) - inner) + kIouEps);
  if (g.zero) ov = 0.f;
  if (azero) ov = -1.f;
  return ov;
}

// iou_utils.py:192-233 — plain IoU.
__device__ __forceinline__ float iou_plain(const GtTile &g, float ax1, float ay1, float ax2,
                                           float ay2, float aarea) {
  float w = fmaxf(fminf(g.x2, ax2) - fmaxf(g.x1, ax1), 0.f);
  float h = fmaxf(fminf(g.y2, ay2) - fmaxf(g.y1, ay1), 0.f);
  float inter = w * h;
  return inter / ((g.area + aarea) - inter);
}

__device__ __forceinline__ void load_gt_tile(GtTile *s, const float *gt, int g0, int G) {
  for (int i = threadIdx.x; i < G; i += blockDim.x) {
    Box4 b = ld4(gt + 4 * static_cast<int64_t>(g0 + i));
    float gx = b.c - b.a, gy = b.d - b.b;
    s[i] = GtTile{b.a, b.b, b.c, b.d, gx * gy, (fabsf(gx) < kIouEps) && (fabsf(gy) < kIouEps)};
  }
}

// Matching in two launches.
//
// k_match_tile (B x ceil(P / 256) workgroups of four INDEPENDENT waves, one prior per lane: no
// barrier and no LDS anywhere in the kernel):
//   per prior: the best object (first index on ties) -> obj / ovl;
//   per object: the image's best prior as a packed (ord(overlap) << 32 | ~prior) key (the lowest
//     prior on ties), for overlaps > 0 only (an object whose best overlap is <= 0 is never
//     forced): each wave reduces its 64 lanes (u32 DPP max of the ord, then the lowest lane
//     holding it) and one lane folds the result into best[b][shard][g] with a no-return
//     agent-scope 64-bit atomic max (executed at the memory side, so waves on different XCDs
//     meet in one word; kKeyShards words per object, by workgroup, keep the queue per word short);
//   lane j holds object j of the current 64-object chunk (box, area, zero flag, label): object g
//     reaches the wave's scalar registers by readlane, so there is no per-object memory access;
//   a wave skips every object whose box misses the bounding box of the wave's priors (the common
//     case: a wave's priors are one small patch of one feature map): every overlap there is <= 0,
//     which can neither raise a prior's best (>= 0 from object 0 on) nor make a key.  The test
//     runs once per chunk as a ballot over the object lanes; the wave walks the set bits;
//   the wave's positive count before the forced match -> wcnt[b][wave] (a plain store: one
//     counter per image took ~2 µs of queued atomics at the end of the launch).
// k_match_final (one workgroup per image): the max over each object's key shards and the sum of
// the image's wave counts, then the forced match of
// models/SSD512.py:546-553 (filter objects whose best overlap > 0, overlap 1.0 and object j = the
// FILTERED position, last writer wins) against the phase-1 (obj, ovl) of each forced prior, the
// positive count adjusted for exactly the priors it rewrites -> n_pos[b], n_pos[B].  Up to 64
// objects it is ONE wave, lane = object, everything in registers (ballots, readlanes, bpermutes);
// more objects take the LDS form.  It leaves best[b][*][*] zero again: the workspace's keys are
// zero on entry to every call after the first (SBOD_MATCH_WS_ZEROED).
// (Round 2's form — a per-tile LDS table of overlaps reduced per (tile, object) into 16-byte
// records, block barriers around it — spent ≈10-12 µs per launch at SSD512 B=32, most of it in
// the barriers and the LDS table)
template <bool kOdm, int kFlags>
__device__ __forceinline__ void match_tile_body(
    const float *__restrict__ gt, const int64_t *__restrict__ labels, const int32_t *__restrict__ off, int g0_in,
    int G_in, const float *__restrict__ anchors, const float *__restrict__ priors,
    const float *__restrict__ arm_scores, int P, int Gmax, float thr, float theta, int32_t *__restrict__ obj,
    float *__restrict__ ovl, unsigned long long *__restrict__ best_key, int32_t *__restrict__ wcnt,
    int32_t *__restrict__ npos, int B, SpanRing *span) {
  __shared__ __attribute__((aligned(16))) uint32_t s_od[kMThreads / 64][kSlots][64 * SBOD_MATCH_PPL];   // per wave
  __shared__ int s_slot[kMThreads / 64][kSlots];
  STAMP_BEGIN();
  span_begin(span);
  const int b = blockIdx.y, tid = threadIdx.x, lane = tid & 63;
  if (blockIdx.x == 0 && b == 0 && tid == 0) npos[B] = 0;   // k_match_final accumulates
  const int wbase = blockIdx.x * kMPriors + SBOD_MATCH_PPL * (tid & ~63), wv = tid >> 6;
  // this workgroup's shard of the image's keys (kKeyShards copies: the waves of one image spread
  // their atomics over kKeyShards words per object instead of queueing on one)
  unsigned long long *brow = best_key + (static_cast<int64_t>(b) * kKeyShards + (blockIdx.x & (kKeyShards - 1))) * Gmax;
  // the wave's positive count per 64 priors, one plain store each (summed by k_match_final)
  int32_t *wc = wcnt + static_cast<int64_t>(b) * (gridDim.x * (kMPriors / 64)) + (wbase >> 6);
#if SBOD_MATCH_PPL == 2
  MatchLane ma, mb;
  match_wave2<kOdm, kFlags>(gt, labels, off, anchors, priors, arm_scores, P, b, wbase, brow, s_od[wv], s_slot[wv],
                            g0_in, G_in, ma, mb);
  if (ma.valid) {
    const int64_t i = static_cast<int64_t>(b) * P + ma.p;
    obj[i] = ma.bi;
    ovl[i] = ma.best;
  }
  if (mb.valid) {
    const int64_t i = static_cast<int64_t>(b) * P + mb.p;
    obj[i] = mb.bi;
    ovl[i] = mb.best;
  }
  const int na = __popcll(__ballot(phase1_positive<kOdm>(ma, thr, theta)));
  const int nb = __popcll(__ballot(phase1_positive<kOdm>(mb, thr, theta)));
  if (lane == 0) {
    wc[0] = na;
    wc[1] = nb;
  }
#else
  const MatchLane m = match_wave<kOdm, kFlags>(gt, labels, off, anchors, priors, arm_scores, P, b, wbase, brow,
                                               s_od[wv], s_slot[wv], g0_in, G_in);
  if (m.valid) {
    const int64_t i = static_cast<int64_t>(b) * P + m.p;
    obj[i] = m.bi;
    ovl[i] = m.best;
  }
  const bool pos = phase1_positive<kOdm>(m, thr, theta);
  const int n = __popcll(__ballot(pos));
  if (lane == 0) wc[0] = n;
#endif
  span_end(span);
  STAMP_END(5, 1);
}

// The matcher's launches take one by-value argument struct (the host cost of a launch grows with
// the argument count on this runtime: scripts/micro/launch_cost.hip).
struct MatchArgs {
  const float *anchors, *priors, *arm_scores;
  int P, Gmax;
  float thr, theta;
  int32_t *obj;
  float *ovl;
  unsigned long long *best_key;
  int32_t *wcnt, *npos;
  int B;
};

template <bool kOdm, int kFlags>
__global__ __launch_bounds__(kMThreads) void k_match_tile(const float *__restrict__ gt, const int64_t *__restrict__ labels,
                                                          const int32_t *__restrict__ off, const MatchArgs m,
                                                          SpanRing *span) {
  match_tile_body<kOdm, kFlags>(gt, labels, off, -1, 0, m.anchors, m.priors, m.arm_scores, m.P, m.Gmax, m.thr, m.theta,
                                m.obj, m.ovl, m.best_key, m.wcnt, m.npos, m.B, span);
}

// The list form (B <= kPackImgs): each image's rows are read in place from the collate_fn lists
// (pointers and row offsets in the kernel arguments), and the image's first workgroup also writes
// them packed (gt_boxes / gt_labels / gt_offsets) for k_match_final and the loss pass after this
// launch — the separate sbod_gt_pack launch folded in.  Every image has >= 1 row, 16-B aligned.
struct MatchListsArgs {
  float *out_boxes;
  int64_t *out_labels;
  int32_t *out_off;
  MatchArgs m;
};
template <bool kOdm, int kFlags>
__global__ __launch_bounds__(kMThreads) void k_match_tile_lists(const GtPackArgs lists, const MatchListsArgs la) {
  float *__restrict__ out_boxes = la.out_boxes;
  int64_t *__restrict__ out_labels = la.out_labels;
  int32_t *__restrict__ out_off = la.out_off;
  const MatchArgs &m = la.m;
  const int B = m.B;
  const int b = blockIdx.y;
  const int r0 = lists.off[b], G = lists.off[b + 1] - r0;
  const float *gtb = lists.boxes[b];
  const int64_t *lab = lists.labels[b];
  if (blockIdx.x == 0) {   // the packed copy of this image's rows
    const float4 *src = reinterpret_cast<const float4 *>(gtb);
    float4 *dst = reinterpret_cast<float4 *>(out_boxes) + r0;
    for (int g = threadIdx.x; g < G; g += kMThreads) {
      dst[g] = src[g];
      out_labels[r0 + g] = lab[g];
    }
    if (threadIdx.x == 0) {
      out_off[b] = r0;
      if (b == B - 1) out_off[B] = r0 + G;
    }
  }
  match_tile_body<kOdm, kFlags>(gtb, lab, nullptr, 0, G, m.anchors, m.priors, m.arm_scores, m.P, m.Gmax, m.thr, m.theta,
                                m.obj, m.ovl, m.best_key, m.wcnt, m.npos, B, nullptr);
}

// k_match_final: one workgroup per image; 64 threads when Gmax <= 64 (the register form),
// else kFThreads (the LDS form).
constexpr int kFThreads = 256;

template <int kFlags>
__global__ __launch_bounds__(kFThreads) void k_match_final(const int64_t *__restrict__ labels,
                                                           const int32_t *__restrict__ off, const MatchArgs m,
                                                           int nw) {
  extern __shared__ __attribute__((aligned(16))) unsigned char s_dyn[];
  __shared__ int s_red[16];
  STAMP_BEGIN();
  match_final_image<kFlags, false>(blockIdx.x, labels, off, m.best_key, m.wcnt, nw, m.Gmax, m.P, m.thr, m.arm_scores,
                                   m.theta, m.obj, m.ovl, m.npos, m.B, 0, ForcedOut{nullptr, nullptr, nullptr}, s_dyn,
                                   s_red);
  STAMP_END(7, 0);
}

// Pairwise IoU matrix out[b, g, p].
__global__ __launch_bounds__(kTile) void k_iou_pairwise(const float *__restrict__ gt,
                                                        const int32_t *__restrict__ off, int Gmax,
                                                        const float *__restrict__ anchors,
                                                        int64_t astride, int P, int mode,
                                                        float *__restrict__ out) {
  extern __shared__ GtTile s_gt[];
  const int b = blockIdx.y;
  const int g0 = off[b], G = off[b + 1] - g0;
  load_gt_tile(s_gt, gt, g0, G);
  __syncthreads();
  const int p = blockIdx.x * kTile + threadIdx.x;
  if (p >= P) return;
  Box4 q = ld4(anchors + astride * b + 4 * static_cast<int64_t>(p));
  float ax = q.c - q.a, ay = q.d - q.b;
  float aarea = ax * ay;
  bool azero = (ax < kIouEps) && (ay < kIouEps);
  float *o = out + (static_cast<int64_t>(b) * Gmax) * P + p;
  for (int g = 0; g < G; ++g) {
    float v;
    if (mode == SBOD_IOU_METRICS) {
      v = iou_metrics(s_gt[g], q.a, q.b, q.c, q.d, aarea, azero);
    } else if (mode == SBOD_IOU_PLAIN) {
      v = iou_plain(s_gt[g], q.a, q.b, q.c, q.d, aarea);
    } else {  // metrics.py:192-205 / iou_utils.py:192-212 intersect
      const GtTile &t = s_gt[g];
      v = fmaxf(fminf(t.x2, q.c) - fmaxf(t.x1, q.a), 0.f) * fmaxf(fminf(t.y2, q.d) - fmaxf(t.y1, q.b), 0.f);
    }
    o[static_cast<int64_t>(g) * P] = v;
  }
}

// Matcher outputs -> the reference's per-prior tensors (parity tests / iou_utils API).
template <bool kOdm>
__global__ __launch_bounds__(kTile) void k_match_expand(
    const float *__restrict__ gt, const int64_t *__restrict__ labels,
    const int32_t *__restrict__ off, const int32_t *__restrict__ obj, const float *__restrict__ ovl,
    const float *__restrict__ priors, const float *__restrict__ arm_locs, int P, float thr,
    float nthr, int flags, int64_t *cls, int64_t *neg, float *txy, float *enc) {
  const int b = blockIdx.y;
  const int p = blockIdx.x * kTile + threadIdx.x;
  if (p >= P) return;
  const int64_t i = static_cast<int64_t>(b) * P + p;
  const int g = off[b] + obj[i];
  const float v = ovl[i];
  const int64_t lab = labels[g];
  if (cls) {
    int64_t c = v < thr ? 0 : lab;
    if (flags & SBOD_MATCH_BINARY) c = c > 0 ? 1 : 0;
    cls[i] = c;
  }
  if (neg) neg[i] = v < nthr ? -1 : lab;
  Box4 t = ld4(gt + 4 * static_cast<int64_t>(g));
  if (txy) st4(txy + 4 * i, t);
  if (enc) {
    Box4 pr;
    if constexpr (kOdm)
      pr = xy_to_cxcy(decode_tenfive_xy(ld4(arm_locs + 4 * i), ld4(priors + 4 * p)));
    else
      pr = ld4(priors + 4 * p);
    st4(enc + 4 * i, encode_tenfive(xy_to_cxcy(t), pr));
  }
}

// iou_utils.match / match_ious, one image: phase A = plain IoU argmaxes.
__global__ __launch_bounds__(kTile) void k_ssd_match_tile(const float *__restrict__ truths, int G,
                                                          const float *__restrict__ priors, int P,
                                                          int32_t *__restrict__ bti,
                                                          float *__restrict__ bto,
                                                          unsigned long long *__restrict__ best) {
  extern __shared__ GtTile s_gt[];
  for (int i = threadIdx.x; i < G; i += blockDim.x) {
    Box4 t = ld4(truths + 4 * i);
    s_gt[i] = GtTile{t.a, t.b, t.c, t.d, (t.c - t.a) * (t.d - t.b), 0};
  }
  __syncthreads();
  const int p = blockIdx.x * kTile + threadIdx.x;
  const bool valid = p < P;
  float x1 = 0.f, y1 = 0.f, x2 = 0.f, y2 = 0.f, area = 0.f;
  if (valid) {  // point_form (iou_utils.py:176-177)
    Box4 q = ld4(priors + 4 * p);
    x1 = q.a - q.c / 2.f;
    y1 = q.b - q.d / 2.f;
    x2 = q.a + q.c / 2.f;
    y2 = q.b + q.d / 2.f;
    area = (x2 - x1) * (y2 - y1);
  }
  float bv = 0.f;
  int bg = 0;
  const unsigned long long low = 0xffffffffull - static_cast<uint32_t>(p);
  for (int g = 0; g < G; ++g) {
    float ov = iou_plain(s_gt[g], x1, y1, x2, y2, area);
    if (g == 0 || ov > bv) {
      bv = ov;
      bg = g;
    }
    unsigned long long key = valid ? ((static_cast<unsigned long long>(f2ord(ov)) << 32) | low) : 0ull;
    key = wave_max_u64(key);
    if ((threadIdx.x & 63) == 0 && key) atomicMax(best + g, key);
  }
  if (valid) {
    bti[p] = bg;
    bto[p] = bv;
  }
}

// phase B: fill 2 at each object's best prior (UNFILTERED j, last writer wins), conf / loc.
__global__ __launch_bounds__(1024) void k_ssd_match_final(
    const float *__restrict__ truths, const int64_t *__restrict__ labels, int G,
    const float *__restrict__ priors, int P, const unsigned long long *__restrict__ best,
    const int32_t *__restrict__ bti, const float *__restrict__ bto, float thr, float v0, float v1,
    int encode, float *__restrict__ loc, int64_t *__restrict__ conf) {
  extern __shared__ int32_t s_bp[];
  for (int g = threadIdx.x; g < G; g += blockDim.x)
    s_bp[g] = static_cast<int32_t>(0xffffffffu - static_cast<uint32_t>(best[g]));
  __syncthreads();
  for (int p = threadIdx.x; p < P; p += blockDim.x) {
    int o = bti[p];
    float v = bto[p];
    for (int g = 0; g < G; ++g)
      if (s_bp[g] == p) {
        o = g;
        v = 2.0f;
      }
    int64_t c = labels[o] + 1;
    if (v < thr) c = 0;
    conf[p] = c;
    Box4 m = ld4(truths + 4 * o);
    if (encode) {  // iou_utils.py:338-345
      Box4 q = ld4(priors + 4 * p);
      float gx = (m.a + m.c) / 2.f - q.a, gy = (m.b + m.d) / 2.f - q.b;
      gx = gx / (v0 * q.c);
      gy = gy / (v0 * q.d);
      float gw = logf((m.c - m.a) / q.c) / v1;
      float gh = logf((m.d - m.b) / q.d) / v1;
      st4(loc + 4 * p, Box4{gx, gy, gw, gh});
    } else {
      st4(loc + 4 * p, m);
    }
  }
}

}  // namespace sbod

using namespace sbod;

namespace {
// Matcher workspace: the per-(image, shard, object) best-prior keys [B][kKeyShards][Gmax] u64
// (zero on entry), then the per-(image, wave) positive counts [B][waves] i32 (written by every
// wave of k_match_tile).  k_match_final leaves ALL of it zero, so a workspace known clean stays
// clean for a later call of any shape that fits in it (SBOD_MATCH_WS_ZEROED).
struct MatchWs {
  unsigned long long *best;
  int32_t *wcnt;
  int nw;
  size_t bytes;
};
MatchWs carve_match(void *w, int B, int Gmax, int P) {
  MatchWs r;
  r.nw = ((P + kMPriors - 1) / kMPriors) * (kMPriors / 64);
  size_t o = 0;
  r.best = ws_at<unsigned long long>(w, o);
  o += align_up(static_cast<size_t>(B) * kKeyShards * Gmax * 8);
  r.wcnt = ws_at<int32_t>(w, o);
  o += align_up(static_cast<size_t>(B) * r.nw * 4);
  r.bytes = o;
  return r;
}
}  // namespace

extern "C" {

size_t sbod_match_workspace_bytes_p(int B, int Gmax, int P) {
  return carve_match(nullptr, B > 0 ? B : 1, Gmax > 0 ? Gmax : 1, P > 0 ? P : 1).bytes;
}

size_t sbod_match_workspace_bytes(int B, int Gmax) {
  return sbod_match_workspace_bytes_p(B, Gmax, 1 << 20);
}

int sbod_iou_pairwise_f32(const float *gt_boxes, const int32_t *gt_offsets, int B, int Gmax,
                          const float *anchors, int64_t anchor_batch_stride, int P, int mode,
                          float *out, void *stream) {
  SBOD_REQUIRE(B > 0 && Gmax >= 0 && P >= 0 && gt_boxes && gt_offsets && anchors && out,
               "sbod_iou_pairwise_f32: bad arguments");
  SBOD_REQUIRE(Gmax <= 4096, "sbod_iou_pairwise_f32: Gmax %d > 4096 unsupported", Gmax);
  if (P == 0 || Gmax == 0) return SBOD_OK;
  dim3 grid((P + kTile - 1) / kTile, B);
  hipLaunchKernelGGL(k_iou_pairwise, grid, dim3(kTile), Gmax * sizeof(GtTile), as_stream(stream),
                     gt_boxes, gt_offsets, Gmax, anchors, anchor_batch_stride, P, mode, out);
  SBOD_LAUNCHED("k_iou_pairwise");
  return SBOD_OK;
}

}  // extern "C"

namespace {
// The matcher's two launches; `lists` non-null = the list form (k_match_tile_lists, which also
// writes gt_boxes / gt_labels / gt_offsets).
int match_run(const float *gt_boxes, const int64_t *gt_labels, const int32_t *gt_offsets, int B, int Gmax,
              const float *anchors, const float *priors_cxcy, const float *arm_scores, int P, float threshold,
              float theta, int flags, int32_t *obj, float *ovl, int32_t *n_pos, void *workspace,
              size_t workspace_bytes, hipStream_t s, const GtPackArgs *lists, const char *who) {
  SBOD_REQUIRE(B > 0 && Gmax > 0 && P > 0 && gt_boxes && gt_labels && gt_offsets && anchors &&
                   obj && ovl && n_pos,
               "%s: bad arguments (B=%d Gmax=%d P=%d)", who, B, Gmax, P);
  SBOD_REQUIRE(Gmax <= 4096, "%s: Gmax %d > 4096 unsupported", who, Gmax);
  SBOD_REQUIRE((flags & ~(SBOD_MATCH_BINARY | SBOD_MATCH_ODM | SBOD_MATCH_WS_ZEROED)) == 0,
               "%s: unknown flags 0x%x", who, flags);
  const bool odm = (flags & SBOD_MATCH_ODM) != 0;
  SBOD_REQUIRE(!odm || (priors_cxcy && arm_scores), "%s: ODM needs priors and arm_scores", who);
  const size_t need = sbod_match_workspace_bytes_p(B, Gmax, P);
  if (workspace_bytes < need) {
    set_error("%s: workspace %zu < %zu", who, workspace_bytes, need);
    return SBOD_E_WORKSPACE;
  }
  const int ntile = (P + kMPriors - 1) / kMPriors;
  MatchWs w = carve_match(workspace, B, Gmax, P);
  // the keys and counts must be zero on entry: every call leaves them so (k_match_final), so
  // only a workspace the caller does not know to be clean is zeroed here (not capturable)
  if ((flags & SBOD_MATCH_WS_ZEROED) == 0 && hipMemsetAsync(workspace, 0, w.bytes, s) != hipSuccess)
    return launch_status("hipMemsetAsync");
  dim3 grid(ntile, B);
  const int fthreads = Gmax <= 64 ? 64 : kFThreads;
  const MatchArgs ma{anchors, priors_cxcy, arm_scores, P, Gmax, threshold, theta, obj, ovl, w.best, w.wcnt, n_pos, B};
#define SBOD_MATCH(ODM, FL)                                                                          \
  do {                                                                                               \
    if (lists) {                                                                                     \
      KernelTimer kt("k_match_tile_lists", s, true);                                                 \
      tlaunch(kt, (k_match_tile_lists<ODM, FL>), grid, dim3(kMThreads), 0, s, *lists,                \
              MatchListsArgs{const_cast<float *>(gt_boxes), const_cast<int64_t *>(gt_labels),        \
                             const_cast<int32_t *>(gt_offsets), ma});                                \
      SBOD_LAUNCHED("k_match_tile_lists");                                                           \
    } else {                                                                                         \
      KernelTimer kt("k_match_tile", s, true);                                                       \
      tlaunch(kt, (k_match_tile<ODM, FL>), grid, dim3(kMThreads), 0, s, gt_boxes, gt_labels,          \
              gt_offsets, ma, kt.span());                                                             \
      SBOD_LAUNCHED("k_match_tile");                                                                 \
    }                                                                                                \
    KernelTimer kt("k_match_final", s, true);                                                        \
    tlaunch(kt, (k_match_final<FL>), dim3(B), dim3(fthreads),                                        \
            Gmax <= 64 ? 0 : static_cast<size_t>(Gmax) * 24, s, gt_labels, gt_offsets, ma, w.nw);   \
  } while (0)
  if (odm)
    SBOD_MATCH(true, SBOD_MATCH_ODM);
  else if (flags & SBOD_MATCH_BINARY)
    SBOD_MATCH(false, SBOD_MATCH_BINARY);
  else
    SBOD_MATCH(false, 0);
#undef SBOD_MATCH
  SBOD_LAUNCHED("k_match_final");
  return SBOD_OK;
}
}  // namespace

extern "C" {

int sbod_match_f32(const float *gt_boxes, const int64_t *gt_labels, const int32_t *gt_offsets,
                   int B, int Gmax, const float *anchors, const float *priors_cxcy,
                   const float *arm_scores, int P, float threshold, float theta, int flags,
                   int32_t *obj, float *ovl, int32_t *n_pos, void *workspace,
                   size_t workspace_bytes, void *stream) {
  return match_run(gt_boxes, gt_labels, gt_offsets, B, Gmax, anchors, priors_cxcy, arm_scores, P, threshold,
                   theta, flags, obj, ovl, n_pos, workspace, workspace_bytes, as_stream(stream), nullptr,
                   "sbod_match_f32");
}

int sbod_match_lists_f32(const void *const *box_ptrs, const void *const *label_ptrs, const int32_t *counts,
                         int64_t capacity, float *gt_boxes, int64_t *gt_labels, int32_t *gt_offsets, int B,
                         int Gmax, const float *anchors, const float *priors_cxcy, const float *arm_scores, int P,
                         float threshold, float theta, int flags, int32_t *obj, float *ovl, int32_t *n_pos,
                         void *workspace, size_t workspace_bytes, void *stream) {
  SBOD_REQUIRE(B > 0 && B <= kPackImgs && box_ptrs && label_ptrs && counts,
               "sbod_match_lists_f32: bad arguments (B=%d, at most %d images)", B, kPackImgs);
  GtPackArgs a;
  int64_t row = 0;
  for (int i = 0; i < B; ++i) {
    SBOD_REQUIRE(counts[i] >= 1 && counts[i] <= Gmax,
                 "sbod_match_lists_f32: image %d has %d objects (1..Gmax=%d)", i, counts[i], Gmax);
    SBOD_REQUIRE(box_ptrs[i] && label_ptrs[i] && (reinterpret_cast<uintptr_t>(box_ptrs[i]) & 15) == 0 &&
                     (reinterpret_cast<uintptr_t>(label_ptrs[i]) & 7) == 0,
                 "sbod_match_lists_f32: image %d: null or misaligned rows", i);
    a.boxes[i] = static_cast<const float *>(box_ptrs[i]);
    a.labels[i] = static_cast<const int64_t *>(label_ptrs[i]);
    a.off[i] = static_cast<int32_t>(row);
    row += counts[i];
  }
  a.off[B] = static_cast<int32_t>(row);
  SBOD_REQUIRE(row <= capacity, "sbod_match_lists_f32: %lld objects exceed the capacity %lld",
               static_cast<long long>(row), static_cast<long long>(capacity));
  SBOD_REQUIRE(reinterpret_cast<uintptr_t>(gt_boxes) % 16 == 0, "sbod_match_lists_f32: gt_boxes not 16-B aligned");
  return match_run(gt_boxes, gt_labels, gt_offsets, B, Gmax, anchors, priors_cxcy, arm_scores, P, threshold,
                   theta, flags, obj, ovl, n_pos, workspace, workspace_bytes, as_stream(stream), &a,
                   "sbod_match_lists_f32");
}

int sbod_match_expand_f32(const float *gt_boxes, const int64_t *gt_labels,
                          const int32_t *gt_offsets, int B, const int32_t *obj, const float *ovl,
                          const float *priors_cxcy, const float *odm_arm_locs, int P,
                          float threshold, float neg_threshold, int flags, int64_t *cls,
                          int64_t *neg, float *true_xy, float *enc, void *stream) {
  SBOD_REQUIRE(B > 0 && P > 0 && gt_boxes && gt_labels && gt_offsets && obj && ovl,
               "sbod_match_expand_f32: bad arguments");
  SBOD_REQUIRE(!enc || priors_cxcy, "sbod_match_expand_f32: enc needs priors_cxcy");
  const bool odm = (flags & SBOD_MATCH_ODM) != 0;
  SBOD_REQUIRE(!(odm && enc) || odm_arm_locs, "sbod_match_expand_f32: ODM enc needs arm locs");
  dim3 grid((P + kTile - 1) / kTile, B);
  if (odm)
    hipLaunchKernelGGL(k_match_expand<true>, grid, dim3(kTile), 0, as_stream(stream), gt_boxes,
                       gt_labels, gt_offsets, obj, ovl, priors_cxcy, odm_arm_locs, P, threshold,
                       neg_threshold, flags, cls, neg, true_xy, enc);
  else
    hipLaunchKernelGGL(k_match_expand<false>, grid, dim3(kTile), 0, as_stream(stream), gt_boxes,
                       gt_labels, gt_offsets, obj, ovl, priors_cxcy, odm_arm_locs, P, threshold,
                       neg_threshold, flags, cls, neg, true_xy, enc);
  SBOD_LAUNCHED("k_match_expand");
  return SBOD_OK;
}

size_t sbod_match_ssd_workspace_bytes(int G, int P) {
  // per object: the best prior key (8 B); per prior: best object and its overlap (4 + 4 B)
  if (G <= 0 || P <= 0) return 0;
  return align_up(G * 8ull) + align_up(P * 4ull) * 2;
}

int sbod_match_ssd_f32(const float *truths, const int64_t *labels, int G,
                       const float *priors_cxcy, int P, float threshold, float var0, float var1,
                       int encode, float *loc_t_row, int64_t *conf_t_row, void *workspace,
                       size_t workspace_bytes, void *stream) {
  SBOD_REQUIRE(G > 0 && P > 0 && truths && labels && priors_cxcy && loc_t_row && conf_t_row,
               "sbod_match_ssd_f32: bad arguments (G=%d P=%d)", G, P);
  SBOD_REQUIRE(G <= 4096, "sbod_match_ssd_f32: G %d > 4096 unsupported", G);
  const size_t need = sbod_match_ssd_workspace_bytes(G, P);
  if (workspace_bytes < need) {
    set_error("sbod_match_ssd_f32: workspace %zu < %zu", workspace_bytes, need);
    return SBOD_E_WORKSPACE;
  }
  char *w = static_cast<char *>(workspace);
  auto *best = reinterpret_cast<unsigned long long *>(w);
  auto *bti = reinterpret_cast<int32_t *>(w + align_up(G * 8ull));
  auto *bto = reinterpret_cast<float *>(w + align_up(G * 8ull) + align_up(P * 4ull));
  hipStream_t s = as_stream(stream);
  if (hipMemsetAsync(best, 0, G * 8ull, s) != hipSuccess) return launch_status("hipMemsetAsync");
  hipLaunchKernelGGL(k_ssd_match_tile, dim3((P + kTile - 1) / kTile), dim3(kTile),
                     G * sizeof(GtTile), s, truths, G, priors_cxcy, P, bti, bto, best);
  SBOD_LAUNCHED("k_ssd_match_tile");
  hipLaunchKernelGGL(k_ssd_match_final, dim3(1), dim3(1024), G * sizeof(int32_t), s, truths,
                     labels, G, priors_cxcy, P, best, bti, bto, threshold, var0, var1, encode,
                     loc_t_row, conf_t_row);
  SBOD_LAUNCHED("k_ssd_match_final");
  return SBOD_OK;
}

}  // extern "C"

SBOD_STAMP_EXPORT(match)

#ifdef SBOD_BLOCK_STAMPS
// k_match_tile's per-workgroup marks (diagnostic build): copies the first n workgroups' 4 marks out,
// then clears them.
extern "C" int sbod_debug_match_marks(unsigned long long *host, int n) {
  const int cap = static_cast<int>(SBOD_STAMP_REGION);
  if (host && n > 0)
    hipMemcpyFromSymbol(host, HIP_SYMBOL(sbod::g_match_marks), sizeof(unsigned long long) * 4 * (n < cap ? n : cap));
  void *sym = nullptr;
  if (hipGetSymbolAddress(&sym, HIP_SYMBOL(sbod::g_match_marks)) == hipSuccess)
    hipMemset(sym, 0, sizeof(unsigned long long) * 4 * cap);
  return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}
#endif

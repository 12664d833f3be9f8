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

struct Anchor {
  float x1, y1, x2, y2, area;
  bool zero;
};

template <bool kOdm>
__device__ __forceinline__ Anchor load_anchor(const float *anchors, const float *priors, int b,
                                              int P, int p) {
  Box4 a;
  if constexpr (kOdm) {
    a = decode_tenfive_xy(ld4(anchors + 4 * (static_cast<int64_t>(b) * P + p)), ld4(priors + 4 * p));
  } else {
    a = ld4(anchors + 4 * static_cast<int64_t>(p));
  }
  float ax = a.c - a.a, ay = a.d - a.b;
  return Anchor{a.a, a.b, a.c, a.d, ax * ay, (ax < kIouEps) && (ay < kIouEps)};
}

// Phase 1: per prior the best object (first index on ties); per object the best prior as a
// packed (ord(overlap) << 32 | ~prior) key reduced with atomicMax (max is order independent, so
// the result is deterministic and equals torch's first-index argmax).
template <bool kOdm>
__global__ __launch_bounds__(kTile) void k_match_tile(
    const float *__restrict__ gt, const int32_t *__restrict__ off, const float *__restrict__ anchors,
    const float *__restrict__ priors, int P, int Gmax, int32_t *__restrict__ obj,
    float *__restrict__ ovl, unsigned long long *__restrict__ objbest, int32_t *__restrict__ npos,
    int B) {
  extern __shared__ GtTile s_gt[];
  const int b = blockIdx.y;
  const int g0 = off[b], G = off[b + 1] - g0;
  if (blockIdx.x == 0 && b == 0 && threadIdx.x == 0) npos[B] = 0;
  load_gt_tile(s_gt, gt, g0, G);
  __syncthreads();
  const int p = blockIdx.x * kTile + threadIdx.x;
  const bool valid = p < P;
  Anchor a{0.f, 0.f, 0.f, 0.f, 0.f, false};
  if (valid) a = load_anchor<kOdm>(anchors, priors, b, P, p);
  float best = 0.f;
  int bi = 0;
  const unsigned long long low = 0xffffffffull - static_cast<uint32_t>(p);
  for (int g = 0; g < G; ++g) {
    float ov = iou_metrics(s_gt[g], a.x1, a.y1, a.x2, a.y2, a.area, a.zero);
    if (g == 0 || ov > best) {
      best = ov;
      bi = g;
    }
    unsigned long long key =
        valid ? ((static_cast<unsigned long long>(f2ord(ov)) << 32) | low) : 0ull;
    key = wave_max_u64(key);
    if ((threadIdx.x & 63) == 0 && key) atomicMax(objbest + static_cast<int64_t>(b) * Gmax + g, key);
  }
  if (valid) {
    obj[static_cast<int64_t>(b) * P + p] = bi;
    ovl[static_cast<int64_t>(b) * P + p] = best;
  }
}

// Phase 2 (one workgroup per image): the forced match of models/SSD512.py:546-553 —
// filter objects whose best overlap > 0, set overlap 1.0 and object j (the FILTERED position,
// last writer wins) — then count positives for the loss normalisers.
template <int kFlags>
__global__ __launch_bounds__(1024) void k_match_final(
    const int64_t *__restrict__ labels, const int32_t *__restrict__ off,
    const unsigned long long *__restrict__ objbest, int Gmax, int P, float thr,
    const float *__restrict__ arm_scores, float theta, int32_t *__restrict__ obj,
    float *__restrict__ ovl, int32_t *__restrict__ npos, int B) {
  extern __shared__ int32_t s_i[];
  int32_t *s_fp = s_i;             // forced prior per filtered j
  int32_t *s_lab = s_i + Gmax;     // labels
  __shared__ int s_nf;
  __shared__ int s_red[16];
  const int b = blockIdx.x;
  const int g0 = off[b], G = off[b + 1] - g0;
  for (int i = threadIdx.x; i < G; i += blockDim.x) s_lab[i] = static_cast<int32_t>(labels[g0 + i]);
  if (threadIdx.x == 0) {
    int nf = 0;
    for (int g = 0; g < G; ++g) {
      unsigned long long k = objbest[static_cast<int64_t>(b) * Gmax + g];
      if (ord2f(static_cast<uint32_t>(k >> 32)) > 0.f)
        s_fp[nf++] = static_cast<int32_t>(0xffffffffu - static_cast<uint32_t>(k));
    }
    s_nf = nf;
  }
  __syncthreads();
  const int nf = s_nf;
  int cnt = 0;
  for (int p = threadIdx.x; p < P; p += blockDim.x) {
    const int64_t i = static_cast<int64_t>(b) * P + p;
    int o = obj[i];
    float v = ovl[i];
    bool hit = false;
    for (int f = 0; f < nf; ++f)
      if (s_fp[f] == p) {
        o = f;
        hit = true;
      }
    if (hit) {
      v = 1.0f;
      obj[i] = o;
      ovl[i] = v;
    }
    int c = v < thr ? 0 : s_lab[o];
    bool pos = c > 0;
    if constexpr ((kFlags & SBOD_MATCH_ODM) != 0) {
      float z0 = arm_scores[2 * i], z1 = arm_scores[2 * i + 1];
      float m = fmaxf(z0, z1);
      float e0 = expf(z0 - m), e1 = expf(z1 - m);
      if (e1 / (e0 + e1) < theta) pos = false;
    }
    cnt += pos ? 1 : 0;
  }
  cnt = block_sum(cnt, s_red);
  if (threadIdx.x == 0) {
    npos[b] = cnt;
    atomicAdd(npos + B, cnt);
  }
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

extern "C" {

size_t sbod_match_workspace_bytes(int B, int Gmax) {
  return align_up(static_cast<size_t>(B) * (Gmax > 0 ? Gmax : 1) * sizeof(unsigned long long));
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

int sbod_match_f32(const float *gt_boxes, const int64_t *gt_labels, const int32_t *gt_offsets,
                   int B, int Gmax, const float *anchors, const float *priors_cxcy,
                   const float *arm_scores, int P, float threshold, float theta, int flags,
                   int32_t *obj, float *ovl, int32_t *n_pos, void *workspace,
                   size_t workspace_bytes, void *stream) {
  SBOD_REQUIRE(B > 0 && Gmax > 0 && P > 0 && gt_boxes && gt_labels && gt_offsets && anchors &&
                   obj && ovl && n_pos,
               "sbod_match_f32: bad arguments (B=%d Gmax=%d P=%d)", B, Gmax, P);
  SBOD_REQUIRE(Gmax <= 4096, "sbod_match_f32: Gmax %d > 4096 unsupported", Gmax);
  const bool odm = (flags & SBOD_MATCH_ODM) != 0;
  SBOD_REQUIRE(!odm || (priors_cxcy && arm_scores), "sbod_match_f32: ODM needs priors and arm_scores");
  if (workspace_bytes < sbod_match_workspace_bytes(B, Gmax)) {
    set_error("sbod_match_f32: workspace %zu < %zu", workspace_bytes, sbod_match_workspace_bytes(B, Gmax));
    return SBOD_E_WORKSPACE;
  }
  hipStream_t s = as_stream(stream);
  auto *objbest = static_cast<unsigned long long *>(workspace);
  if (hipMemsetAsync(objbest, 0, static_cast<size_t>(B) * Gmax * 8, s) != hipSuccess)
    return launch_status("hipMemsetAsync(match)");
  dim3 grid((P + kTile - 1) / kTile, B);
  const size_t lds = Gmax * sizeof(GtTile);
  if (odm)
    hipLaunchKernelGGL(k_match_tile<true>, grid, dim3(kTile), lds, s, gt_boxes, gt_offsets,
                       anchors, priors_cxcy, P, Gmax, obj, ovl, objbest, n_pos, B);
  else
    hipLaunchKernelGGL(k_match_tile<false>, grid, dim3(kTile), lds, s, gt_boxes, gt_offsets,
                       anchors, priors_cxcy, P, Gmax, obj, ovl, objbest, n_pos, B);
  SBOD_LAUNCHED("k_match_tile");
  const size_t lds2 = 2 * Gmax * sizeof(int32_t);
  if (odm)
    hipLaunchKernelGGL(k_match_final<SBOD_MATCH_ODM>, dim3(B), dim3(1024), lds2, s, gt_labels,
                       gt_offsets, objbest, Gmax, P, threshold, arm_scores, theta, obj, ovl, n_pos, B);
  else if (flags & SBOD_MATCH_BINARY)
    hipLaunchKernelGGL(k_match_final<SBOD_MATCH_BINARY>, dim3(B), dim3(1024), lds2, s, gt_labels,
                       gt_offsets, objbest, Gmax, P, threshold, arm_scores, theta, obj, ovl, n_pos, B);
  else
    hipLaunchKernelGGL(k_match_final<0>, dim3(B), dim3(1024), lds2, s, gt_labels, gt_offsets,
                       objbest, Gmax, P, threshold, arm_scores, theta, obj, ovl, n_pos, B);
  SBOD_LAUNCHED("k_match_final");
  return SBOD_OK;
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

int sbod_match_ssd_f32(const float *truths, const int64_t *labels, int G,
                       const float *priors_cxcy, int P, float threshold, float var0, float var1,
                       int encode, float *loc_t_row, int64_t *conf_t_row, void *workspace,
                       size_t workspace_bytes, void *stream) {
  SBOD_REQUIRE(G > 0 && P > 0 && truths && labels && priors_cxcy && loc_t_row && conf_t_row,
               "sbod_match_ssd_f32: bad arguments (G=%d P=%d)", G, P);
  SBOD_REQUIRE(G <= 4096, "sbod_match_ssd_f32: G %d > 4096 unsupported", G);
  const size_t need = align_up(G * 8ull) + align_up(P * 4ull) * 2;
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

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

// Phase 1 (B x P/256 workgroups): per prior the best object (first index on ties) and the
// tile's positive count before the forced match; per object the tile's best prior as a packed
// (ord(overlap) << 32 | ~prior) key — waves reduce through LDS and each tile writes its own
// partial row (no global atomics: the per-object argmax is finished deterministically by
// phase 2, equal to torch's first-index argmax because max is order independent).
constexpr int kMaxGLds = 256;   // objects per image whose per-wave partials stay in LDS

template <bool kOdm, int kFlags>
__global__ __launch_bounds__(kTile) void k_match_tile(
    const float *__restrict__ gt, const int64_t *__restrict__ labels,
    const int32_t *__restrict__ off, const float *__restrict__ anchors,
    const float *__restrict__ priors, const float *__restrict__ arm_scores, int P, int Gmax,
    float thr, float theta, int32_t *__restrict__ obj, float *__restrict__ ovl,
    unsigned long long *__restrict__ part, int32_t *__restrict__ tcount, int32_t *__restrict__ npos,
    int B, SpanRing *span) {
  extern __shared__ GtTile s_gt[];
  __shared__ unsigned long long s_key[kTile / 64][kMaxGLds];
  STAMP_BEGIN();
  span_begin(span);
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) npos[B] = 0;  // phase 2 accumulates
  __shared__ int32_t s_lab[kMaxGLds];
  __shared__ int s_red[16];
  PHASE_DECL;
  SEG_PHASE(0);
  const int b = blockIdx.y, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int ntile = gridDim.x;
  // the prior's own load goes out first: it does not wait on the ground-truth chain
  const int p = blockIdx.x * kTile + threadIdx.x;
  const bool valid = p < P;
  Anchor a{0.f, 0.f, 0.f, 0.f, 0.f, false};
  if (valid) a = load_anchor<kOdm>(anchors, priors, b, P, p);
  const int g0 = off[b], G = off[b + 1] - g0;
  load_gt_tile(s_gt, gt, g0, G);
  for (int i = threadIdx.x; i < G && i < kMaxGLds; i += blockDim.x)
    s_lab[i] = static_cast<int32_t>(labels[g0 + i]);
  __syncthreads();
  SEG_PHASE(1);
  float best = 0.f;
  int bi = 0;
  const int pw = blockIdx.x * kTile + wv * 64;   // prior of lane 0 of this wave
  unsigned long long *prow = part + (static_cast<int64_t>(b) * ntile + blockIdx.x) * Gmax;
  for (int g = 0; g < G; ++g) {
    const float ov = iou_metrics(s_gt[g], a.x1, a.y1, a.x2, a.y2, a.area, a.zero);
    if (g == 0 || ov > best) {
      best = ov;
      bi = g;
    }
    // the wave's best (ord(overlap), lowest prior) — torch's first-index argmax over priors:
    // max of the 32-bit ord over the wave (DPP), then the lowest lane holding it (ballot)
    const uint32_t ko = valid ? f2ord(ov) : 0u;   // f2ord of any real overlap is > 0
    const uint32_t mx = wave_max_u32(ko);
    const unsigned long long hit = __ballot(valid && ko == mx);
    if (lane == 0) {
      const unsigned long long key =
          hit ? ((static_cast<unsigned long long>(mx) << 32) |
                 (0xffffffffull - static_cast<uint32_t>(pw + __builtin_ctzll(hit))))
              : 0ull;
      if (G <= kMaxGLds) s_key[wv][g] = key;
      else if (key) atomicMax(prow + g, key);   // very large G: partial row via atomics
    }
  }
  SEG_PHASE(2);
  int pos = 0;
  if (valid) {
    obj[static_cast<int64_t>(b) * P + p] = bi;
    ovl[static_cast<int64_t>(b) * P + p] = best;
    const int lab = G <= kMaxGLds ? s_lab[bi] : static_cast<int>(labels[g0 + bi]);
    int c = best < thr ? 0 : lab;
    if ((kFlags & SBOD_MATCH_BINARY) != 0) c = c > 0;
    pos = c > 0;
    if constexpr (kOdm) {
      const int64_t i = static_cast<int64_t>(b) * P + p;
      const float z0 = arm_scores[2 * i], z1 = arm_scores[2 * i + 1];
      const float m = fmaxf(z0, z1);
      const float e0 = expf(z0 - m), e1 = expf(z1 - m);
      if (e1 / (e0 + e1) < theta) pos = 0;
    }
  }
  pos = block_sum(pos, s_red);  // contains __syncthreads: s_key complete after it
  if (G <= kMaxGLds) {
    for (int g = threadIdx.x; g < G; g += blockDim.x) {
      unsigned long long k = s_key[0][g];
      for (int w = 1; w < kTile / 64; ++w) k = s_key[w][g] > k ? s_key[w][g] : k;
      prow[g] = k;
    }
  }
  if (threadIdx.x == 0) tcount[b * ntile + blockIdx.x] = pos;
  span_end(span);
  SEG_PHASE(3);
#ifdef SBOD_PHASE_CLOCKS
  if (PHASE_PRINT_SEL)
    printf("match x%d b%d G=%d: gt %lld iou+argmax %lld store+sum %lld total %lld\n", blockIdx.x, b, G,
           ph[1] - ph[0], ph[2] - ph[1], ph[3] - ph[2], ph[3] - ph[0]);
#endif
  STAMP_END(5, 1);
}

// Phase 2 (one wave per image): finish the per-object argmax over the tiles, then the forced
// match of models/SSD512.py:546-553 applied serially — filter objects whose best overlap > 0,
// overlap 1.0 and object j (the FILTERED position, last writer wins) — adjusting the positive
// count for exactly the priors it rewrites.
template <int kFlags>
__global__ __launch_bounds__(256) void k_match_final(
    const int64_t *__restrict__ labels, const int32_t *__restrict__ off,
    const unsigned long long *__restrict__ part, const int32_t *__restrict__ tcount, int ntile,
    int Gmax, int P, float thr, const float *__restrict__ arm_scores, float theta,
    int32_t *__restrict__ obj, float *__restrict__ ovl, int32_t *__restrict__ npos, int B) {
  // LDS per object g: best key, its prior, the prior's phase-1 (obj, ovl), easy flag, label
  extern __shared__ unsigned long long s_best[];
  int32_t *s_pr = reinterpret_cast<int32_t *>(s_best + Gmax);
  int32_t *s_o0 = s_pr + Gmax;
  float *s_v0 = reinterpret_cast<float *>(s_o0 + Gmax);
  int32_t *s_lab = reinterpret_cast<int32_t *>(s_v0 + Gmax);
  int32_t *s_easy = s_lab + Gmax;
  int32_t *s_new = s_easy + Gmax;     // final object written for this g's prior, -1 = superseded
  __shared__ int s_red[16];
  const int b = blockIdx.x, tid = threadIdx.x;
  const int g0 = off[b], G = off[b + 1] - g0;
  const unsigned long long *pb = part + static_cast<int64_t>(b) * ntile * Gmax;
  for (int g = tid; g < G; g += blockDim.x) {
    s_best[g] = 0ull;
    s_lab[g] = static_cast<int32_t>(labels[g0 + g]);
  }
  __syncthreads();
  for (int it = tid; it < G * ntile; it += blockDim.x) {   // all tile partials in flight at once
    const int g = it / ntile, t = it - g * ntile;
    atomicMax(&s_best[g], pb[static_cast<int64_t>(t) * Gmax + g]);
  }
  int cnt = 0;
  for (int t = tid; t < ntile; t += blockDim.x) cnt += tcount[b * ntile + t];
  cnt = block_sum(cnt, s_red);
  for (int g = tid; g < G; g += blockDim.x) {
    const unsigned long long k = s_best[g];
    int p = -1;
    if (ord2f(static_cast<uint32_t>(k >> 32)) > 0.f) {
      p = static_cast<int>(0xffffffffu - static_cast<uint32_t>(k));
      const int64_t i = static_cast<int64_t>(b) * P + p;
      s_o0[g] = obj[i];
      s_v0[g] = ovl[i];
      int easy = 0;
      if constexpr ((kFlags & SBOD_MATCH_ODM) != 0) {
        const float z0 = arm_scores[2 * i], z1 = arm_scores[2 * i + 1];
        const float m = fmaxf(z0, z1);
        const float e0 = expf(z0 - m), e1 = expf(z1 - m);
        easy = e1 / (e0 + e1) < theta;
      }
      s_easy[g] = easy;
    }
    s_pr[g] = p;
  }
  __syncthreads();
  // The forced match (SSD512.py:546-553) without a serial loop: object g's filtered position j_g
  // is the number of valid objects before it; a prior forced more than once keeps its LAST
  // writer, and each writer's "old" state is the previous writer's (or the phase-1 state).
  for (int g = tid; g < G; g += blockDim.x) {
    int j = 0, prev = -1;
    const int p = s_pr[g];
    for (int h = 0; h < g; ++h) {
      const int ph = s_pr[h];
      if (ph >= 0) {
        ++j;
        if (ph == p) prev = h;
      }
    }
    s_o0[g] = p >= 0 ? s_o0[g] : 0;
    s_new[g] = p >= 0 ? j : -1;
    s_easy[g] = (s_easy[g] & 1) | (prev >= 0 ? ((prev + 1) << 1) : 0);  // pack prev into easy
  }
  __syncthreads();
  auto is_pos = [&](int o, float v, int easy) {
    int c = v < thr ? 0 : s_lab[o];
    if ((kFlags & SBOD_MATCH_BINARY) != 0) c = c > 0;
    return c > 0 && !easy;
  };
  int delta = 0;
  for (int g = tid; g < G; g += blockDim.x) {
    if (s_pr[g] < 0) continue;
    const int easy = s_easy[g] & 1, prev = (s_easy[g] >> 1) - 1;
    const int o_old = prev >= 0 ? s_new[prev] : s_o0[g];
    const float v_old = prev >= 0 ? 1.0f : s_v0[g];
    delta += (is_pos(s_new[g], 1.0f, easy) ? 1 : 0) - (is_pos(o_old, v_old, easy) ? 1 : 0);
  }
  delta = block_sum(delta, s_red);
  for (int g = tid; g < G; g += blockDim.x) {
    const int p = s_pr[g];
    if (p < 0) continue;
    bool last = true;                                  // superseded by a later writer?
    for (int h = g + 1; h < G && last; ++h)
      if (s_pr[h] == p) last = false;
    if (!last) continue;
    const int64_t i = static_cast<int64_t>(b) * P + p;
    obj[i] = s_new[g];
    ovl[i] = 1.0f;
  }
  if (tid == 0) {
    npos[b] = cnt + delta;
    atomicAdd(npos + B, cnt + delta);
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

namespace {
struct MatchWs {
  unsigned long long *part, *best;
  int32_t *tcount;
  size_t bytes;
};
MatchWs carve_match(void *w, int B, int Gmax, int P) {
  const size_t ntile = (P + kTile - 1) / kTile;
  char *c = static_cast<char *>(w);
  MatchWs r;
  size_t o = 0;
  r.part = reinterpret_cast<unsigned long long *>(c + o);
  o += align_up(static_cast<size_t>(B) * ntile * Gmax * 8);
  r.best = reinterpret_cast<unsigned long long *>(c + o);
  o += align_up(static_cast<size_t>(B) * Gmax * 8);
  r.tcount = reinterpret_cast<int32_t *>(c + o);
  o += align_up(static_cast<size_t>(B) * ntile * 4);
  r.bytes = o;
  return r;
}
}  // namespace

extern "C" {

size_t sbod_match_workspace_bytes_p(int B, int Gmax, int P) {
  return carve_match(nullptr, B, Gmax > 0 ? Gmax : 1, P > 0 ? P : 1).bytes;
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
  const size_t need = sbod_match_workspace_bytes_p(B, Gmax, P);
  if (workspace_bytes < need) {
    set_error("sbod_match_f32: workspace %zu < %zu", workspace_bytes, need);
    return SBOD_E_WORKSPACE;
  }
  hipStream_t s = as_stream(stream);
  const int ntile = (P + kTile - 1) / kTile;
  MatchWs w = carve_match(workspace, B, Gmax, P);
  if (Gmax > kMaxGLds &&
      hipMemsetAsync(w.part, 0, static_cast<size_t>(B) * ntile * Gmax * 8, s) != hipSuccess)
    return launch_status("hipMemsetAsync(match)");
  dim3 grid(ntile, B);
  const size_t lds = Gmax * sizeof(GtTile);
#define SBOD_TILE(ODM, FL)                                                                      \
  do {                                                                                          \
    KernelTimer kt("k_match_tile", s, true);                                                          \
    tlaunch(kt, (k_match_tile<ODM, FL>), grid, dim3(kTile), lds, s, gt_boxes, gt_labels,   \
                       gt_offsets, anchors, priors_cxcy, arm_scores, P, Gmax, threshold, theta, obj, \
                       ovl, w.part, w.tcount, n_pos, B, kt.span());                              \
  } while (0)
#define SBOD_FINAL(FL)                                                                          \
  do {                                                                                          \
    KernelTimer kt("k_match_final", s, true);                                                         \
    tlaunch(kt, (k_match_final<FL>), dim3(B), dim3(256), Gmax * 32, s, gt_labels, gt_offsets, \
                       w.part, w.tcount, ntile, Gmax, P, threshold, arm_scores, theta, obj, ovl, n_pos, B); \
  } while (0)
  if (odm) {
    SBOD_TILE(true, SBOD_MATCH_ODM);
    SBOD_LAUNCHED("k_match_tile");
    SBOD_FINAL(SBOD_MATCH_ODM);
  } else if (flags & SBOD_MATCH_BINARY) {
    SBOD_TILE(false, SBOD_MATCH_BINARY);
    SBOD_LAUNCHED("k_match_tile");
    SBOD_FINAL(SBOD_MATCH_BINARY);
  } else {
    SBOD_TILE(false, 0);
    SBOD_LAUNCHED("k_match_tile");
    SBOD_FINAL(0);
  }
#undef SBOD_TILE
#undef SBOD_FINAL
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

SBOD_STAMP_EXPORT(match)

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
constexpr int kMThreads = 256;   // k_match_tile: one prior per thread

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
__device__ __forceinline__ Anchor make_anchor(Box4 raw, Box4 prior) {
  Box4 a = raw;
  if constexpr (kOdm) a = decode_tenfive_xy(raw, prior);
  float ax = a.c - a.a, ay = a.d - a.b;
  return Anchor{a.a, a.b, a.c, a.d, ax * ay, (ax < kIouEps) && (ay < kIouEps)};
}

template <bool kOdm>
__device__ __forceinline__ Anchor load_anchor(const float *anchors, const float *priors, int b,
                                              int P, int p) {
  if constexpr (kOdm)
    return make_anchor<true>(ld4(anchors + 4 * (static_cast<int64_t>(b) * P + p)), ld4(priors + 4 * p));
  return make_anchor<false>(ld4(anchors + 4 * static_cast<int64_t>(p)), Box4{0.f, 0.f, 0.f, 0.f});
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
constexpr int kKeyShards = 8;   // copies of the per-object key words (one per XCD-sized group of tiles)
constexpr int kSlots = 16;      // per-wave LDS rows of pending per-object ords

// Max of a u64 over each quad of lanes, valid in every lane of the quad (DPP quad swaps; keys are
// unique, so the max is the quad's best).
template <int kCtrl>
__device__ __forceinline__ unsigned long long dpp_max_u64(unsigned long long v) {
  const uint32_t lo = dpp_u32<kCtrl, 0xf>(static_cast<uint32_t>(v));
  const uint32_t hi = dpp_u32<kCtrl, 0xf>(static_cast<uint32_t>(v >> 32));
  const unsigned long long o = (static_cast<unsigned long long>(hi) << 32) | lo;
  return o > v ? o : v;
}
__device__ __forceinline__ unsigned long long quad_max_u64(unsigned long long v) {
  v = dpp_max_u64<0xB1>(v);        // quad_perm [1,0,3,2]
  return dpp_max_u64<0x4E>(v);     // quad_perm [2,3,0,1]
}

struct GtLane {   // lane j of a chunk: object j
  float x1, y1, x2, y2, area;
  int zero, lab;
};

template <int kFlags>
__device__ __forceinline__ GtLane load_gt_lane(const float *__restrict__ gt, const int64_t *__restrict__ labels,
                                               int g0, int gc, int gn, int lane) {
  const int j = g0 + gc + min(lane, max(gn - 1, 0));
  const Box4 bx = ld4(gt + 4 * static_cast<int64_t>(j));
  const float gx = bx.c - bx.a, gy = bx.d - bx.b;
  int lab = static_cast<int32_t>(labels[j]);
  if ((kFlags & SBOD_MATCH_BINARY) != 0) lab = lab > 0;
  return GtLane{bx.a, bx.b, bx.c, bx.d, gx * gy, (fabsf(gx) < kIouEps) && (fabsf(gy) < kIouEps), lab};
}

__device__ __forceinline__ float rl_f(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

template <bool kOdm, int kFlags>
__global__ __launch_bounds__(kMThreads) void k_match_tile(
    const float *__restrict__ gt, const int64_t *__restrict__ labels,
    const int32_t *__restrict__ off, const float *__restrict__ anchors,
    const float *__restrict__ priors, const float *__restrict__ arm_scores, int P, int Gmax,
    float thr, float theta, int32_t *__restrict__ obj, float *__restrict__ ovl,
    unsigned long long *__restrict__ best_key, int32_t *__restrict__ wcnt, int32_t *__restrict__ npos,
    int B, SpanRing *span) {
  __shared__ __attribute__((aligned(16))) uint32_t s_od[kMThreads / 64][kSlots][64];   // per wave
  __shared__ int s_slot[kMThreads / 64][kSlots];
  STAMP_BEGIN();
  span_begin(span);
  const int b = blockIdx.y, tid = threadIdx.x, lane = tid & 63;
  if (blockIdx.x == 0 && b == 0 && tid == 0) npos[B] = 0;   // k_match_final accumulates
  const int wbase = blockIdx.x * kMThreads + (tid & ~63);
  const int p = wbase + lane;
  const bool valid = p < P;
  // one memory round trip before the object loop: the anchor and the first chunk's objects
  // (unconditional, clamped loads; an image without objects reads element 0 — the GT buffers
  // hold at least one)
  const int pc = min(p, P - 1);
  const Box4 araw = ld4(kOdm ? anchors + 4 * (static_cast<int64_t>(b) * P + pc) : anchors + 4 * static_cast<int64_t>(pc));
  const Box4 apri = kOdm ? ld4(priors + 4 * pc) : Box4{0.f, 0.f, 0.f, 0.f};
  const int g0 = ld_i32_uniform(off + b), G = ld_i32_uniform(off + b + 1) - g0;
  const bool has = G > 0;
  GtLane o = load_gt_lane<kFlags>(gt, labels, has ? g0 : 0, 0, has ? min(G, 64) : 1, lane);
  float eas0 = 0.f, eas1 = 0.f;
  if constexpr (kOdm) {
    const int64_t ic = static_cast<int64_t>(b) * P + pc;
    eas0 = arm_scores[2 * ic];
    eas1 = arm_scores[2 * ic + 1];
  }
  const Anchor a = make_anchor<kOdm>(araw, apri);
  // the wave's prior bounding box as monotone integer keys
  const bool live = valid && !a.zero;
  const uint32_t wx1 = ~wave_max_u32(live ? ~f2ord(a.x1) : 0u), wy1 = ~wave_max_u32(live ? ~f2ord(a.y1) : 0u);
  const uint32_t wx2 = wave_max_u32(live ? f2ord(a.x2) : 0u), wy2 = wave_max_u32(live ? f2ord(a.y2) : 0u);
  const bool wlive = __ballot(live) != 0ull;
  float best = 0.f;
  int bi = 0, blab = 0;
  // this workgroup's shard of the image's keys (kKeyShards copies: the waves of one image spread
  // their atomics over kKeyShards words per object instead of queueing on one)
  unsigned long long *brow = best_key + (static_cast<int64_t>(b) * kKeyShards + (blockIdx.x & (kKeyShards - 1))) * Gmax;
  // metrics.py:224-250, in the reference's order: this lane's overlap with chunk object j
  auto iou_of = [&](int j, int &glab) {
    const float tx1 = rl_f(o.x1, j), ty1 = rl_f(o.y1, j), tx2 = rl_f(o.x2, j), ty2 = rl_f(o.y2, j);
    const float garea = rl_f(o.area, j);
    const int gzero = __builtin_amdgcn_readlane(o.zero, j);
    glab = __builtin_amdgcn_readlane(o.lab, j);
    float iw = fminf(tx2, a.x2) - fmaxf(tx1, a.x1);
    if (iw < 0.f) iw = 0.f;
    float ih = fminf(ty2, a.y2) - fmaxf(ty1, a.y1);
    if (ih < 0.f) ih = 0.f;
    const float inner = iw * ih;
    float ov = inner / (((garea + a.area) - inner) + kIouEps);
    if (gzero) ov = 0.f;
    if (a.zero) ov = -1.f;
    return ov;
  };
  // Per-object keys: an object with a positive overlap in this wave leaves its lanes' ords in
  // one of the wave's kSlots LDS rows (one ds_write, no cross-lane work in the object loop);
  // flush_keys reduces all filled rows at once — lane = (row, 16-lane segment): the segment's
  // max ord and lowest lane holding it, then the max over the row's 4 segments (DPP) — and
  // folds each row's key into the object's word with one atomic.  Rows are wave-private: no
  // block barrier, only the wave's own LDS order.
  const int wv = tid >> 6;
  int nslot = 0;
  auto flush_keys = [&]() {
    if (nslot == 0) return;
    __builtin_amdgcn_wave_barrier();
    const int j = lane >> 2, q = lane & 3;
    unsigned long long key = 0ull;
    if (j < nslot) {
      const uint4 *row = reinterpret_cast<const uint4 *>(&s_od[wv][j][16 * q]);
      uint32_t v[16];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint4 x = row[r];
        v[4 * r] = x.x;
        v[4 * r + 1] = x.y;
        v[4 * r + 2] = x.z;
        v[4 * r + 3] = x.w;
      }
      uint32_t mx = v[0];
#pragma unroll
      for (int c = 1; c < 16; ++c) mx = max(mx, v[c]);
      int c0 = 15;
#pragma unroll
      for (int c = 14; c >= 0; --c) c0 = v[c] == mx ? c : c0;
      key = mx ? ((static_cast<unsigned long long>(mx) << 32) |
                  (0xffffffffull - static_cast<uint32_t>(wbase + 16 * q + c0)))
               : 0ull;
    }
    key = quad_max_u64(key);
    if (q == 0 && j < nslot && key)
      __hip_atomic_fetch_max(brow + s_slot[wv][j], key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_wave_barrier();
    nslot = 0;
  };
  auto note_key = [&](int g, float ov) {
    const uint32_t od = (valid && ov > 0.f) ? f2ord(ov) : 0u;
    if (__ballot(od != 0u) == 0ull) return;   // no positive overlap here: never this wave's key
    s_od[wv][nslot][lane] = od;
    if (lane == 0) s_slot[wv][nslot] = g;
    if (++nslot == kSlots) flush_keys();
  };
  for (int gc = 0; gc < G; gc += 64) {
    const int gn = min(G - gc, 64);
    if (gc > 0) o = load_gt_lane<kFlags>(gt, labels, g0, gc, gn, lane);
    // objects of this chunk whose box meets the wave's prior box (object 0 always: it sets
    // every prior's first best, ties included)
    const bool hit = wlive && lane < gn && f2ord(o.x2) > wx1 && f2ord(o.x1) < wx2 && f2ord(o.y2) > wy1 &&
                     f2ord(o.y1) < wy2;
    unsigned long long todo = __ballot(hit) | (gc == 0 ? 1ull : 0ull);
    // two objects per step (independent IoU chains), applied in object order
    while (todo) {
      const int j1 = __builtin_ctzll(todo);
      todo &= todo - 1ull;
      const bool two = todo != 0ull;
      const int j2 = two ? __builtin_ctzll(todo) : j1;
      if (two) todo &= todo - 1ull;
      int lab1, lab2;
      const float ov1 = iou_of(j1, lab1), ov2 = iou_of(j2, lab2);
      if (gc + j1 == 0 || ov1 > best) {
        best = ov1;
        bi = gc + j1;
        blab = lab1;
      }
      if (two && ov2 > best) {
        best = ov2;
        bi = gc + j2;
        blab = lab2;
      }
      note_key(gc + j1, ov1);
      if (two) note_key(gc + j2, ov2);
    }
  }
  flush_keys();
  bool pos = false;
  if (valid) {
    const int64_t i = static_cast<int64_t>(b) * P + p;
    obj[i] = bi;
    ovl[i] = best;
    pos = !(best < thr) && blab > 0;
    if constexpr (kOdm) {
      const float m = fmaxf(eas0, eas1);
      const float e0 = expf(eas0 - m), e1 = expf(eas1 - m);
      if (e1 / (e0 + e1) < theta) pos = false;
    }
  }
  // the wave's positive count, one plain store per wave (summed by k_match_final)
  const int n = __popcll(__ballot(pos));
  if (lane == 0) wcnt[static_cast<int64_t>(b) * (gridDim.x * (kMThreads / 64)) + (wbase >> 6)] = n;
  span_end(span);
  STAMP_END(5, 1);
}

// k_match_final: one workgroup per image; 64 threads when Gmax <= 64 (the register form),
// else kFThreads (the LDS form).
constexpr int kFThreads = 256;

template <int kFlags>
__global__ __launch_bounds__(kFThreads) void k_match_final(
    const int64_t *__restrict__ labels, const int32_t *__restrict__ off,
    unsigned long long *__restrict__ best_key, int32_t *__restrict__ wcnt, int nw, int Gmax,
    int P, float thr, const float *__restrict__ arm_scores, float theta, int32_t *__restrict__ obj,
    float *__restrict__ ovl, int32_t *__restrict__ npos, int B) {
  extern __shared__ __attribute__((aligned(16))) unsigned char s_dyn[];
  __shared__ int s_red[16];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  STAMP_BEGIN();
  const int g0 = off[b], G = off[b + 1] - g0;
  unsigned long long *brow = best_key + static_cast<int64_t>(b) * kKeyShards * Gmax;
  // the phase-1 positive count: the image's per-wave counts (first wave only; the LDS form
  // shares it through s_red)
  int cnt1 = 0;
  if (tid < 64) {
    for (int w = lane; w < nw; w += 64) {
      int32_t *c = wcnt + static_cast<int64_t>(b) * nw + w;
      cnt1 += *c;
      *c = 0;   // the whole workspace is zero again after a call (any B, Gmax, P next time)
    }
    cnt1 = wave_sum_i32(cnt1);
  }
  // an object's key: the max over its shards, which return to zero
  auto take_key = [&](int g) {
    unsigned long long k = 0ull;
#pragma unroll
    for (int s = 0; s < kKeyShards; ++s) {
      const unsigned long long v = brow[s * Gmax + g];
      k = v > k ? v : k;
    }
#pragma unroll
    for (int s = 0; s < kKeyShards; ++s) brow[s * Gmax + g] = 0ull;
    return k;
  };
  auto lab_of = [&](int g) {
    int l = static_cast<int32_t>(labels[g0 + g]);
    if ((kFlags & SBOD_MATCH_BINARY) != 0) l = l > 0;
    return l;
  };
  auto easy_of = [&](int p) {
    int easy = 0;
    if constexpr ((kFlags & SBOD_MATCH_ODM) != 0) {
      const int64_t i = static_cast<int64_t>(b) * P + p;
      const float z0 = arm_scores[2 * i], z1 = arm_scores[2 * i + 1];
      const float m = fmaxf(z0, z1);
      const float e0 = expf(z0 - m), e1 = expf(z1 - m);
      easy = e1 / (e0 + e1) < theta;
    }
    return easy;
  };
  // is_pos(label, overlap, easy): the positive rule of the criteria
  auto is_pos = [&](int lab, float v, int easy) { return !(v < thr) && lab > 0 && !easy; };
  auto publish = [&](int delta) {   // one lane
    const int nb = cnt1 + delta;
    npos[b] = nb;
    atomicAdd(npos + B, nb);
  };
  if (G <= 64) {
    if (tid >= 64) return;
    // lane = object: its best key, the key's prior and that prior's phase-1 (obj, ovl)
    const unsigned long long k = lane < G ? take_key(lane) : 0ull;
    const int lab = lane < G ? lab_of(lane) : 0;
    const int p = k ? static_cast<int>(0xffffffffu - static_cast<uint32_t>(k)) : -1;
    const int64_t ip = static_cast<int64_t>(b) * P + (p >= 0 ? p : 0);
    const int o_ph1 = obj[ip];
    const float v_ph1 = ovl[ip];
    const int easy = p >= 0 ? easy_of(p) : 0;
    const unsigned long long valid = __ballot(p >= 0);
    const int j = __popcll(valid & ((1ull << lane) - 1ull));   // filtered position
    int prev = -1;      // the previous writer of the same prior
    bool lastw = true;  // no later writer of the same prior
    for (int h = 0; h < G; ++h) {
      const int ph = __builtin_amdgcn_readlane(p, h);
      if (p >= 0 && ph == p) {
        if (h < lane) prev = h;
        if (h > lane) lastw = false;
      }
    }
    const int jprev = __shfl(j, prev < 0 ? lane : prev, 64);
    const int o_old = prev >= 0 ? jprev : o_ph1;
    const float v_old = prev >= 0 ? 1.0f : v_ph1;
    // labels of the new object j and the old object, read from the lanes that hold them
    const int lab_new = __shfl(lab, j & 63, 64), lab_old = __shfl(lab, o_old & 63, 64);
    int d = 0;
    if (p >= 0) {
      d = (is_pos(lab_new, 1.0f, easy) ? 1 : 0) - (is_pos(lab_old, v_old, easy) ? 1 : 0);
      if (lastw) {
        obj[ip] = j;
        ovl[ip] = 1.0f;
      }
    }
    const int delta = wave_sum_i32(d);
    if (lane == 0) publish(delta);
    STAMP_END(7, 0);
    return;
  }
  // more objects: the LDS form of the same rules.  LDS per object: prior, easy | previous writer,
  // label, final object, phase-1 (obj, ovl)
  int32_t *s_pr = reinterpret_cast<int32_t *>(s_dyn);
  int32_t *s_easy = s_pr + Gmax;
  int32_t *s_lab = s_easy + Gmax;
  int32_t *s_new = s_lab + Gmax;
  int32_t *s_o0 = s_new + Gmax;
  float *s_v0 = reinterpret_cast<float *>(s_o0 + Gmax);
  if (tid == 0) s_red[15] = cnt1;
  for (int g = tid; g < G; g += blockDim.x) {
    const unsigned long long k = take_key(g);
    const int p = k ? static_cast<int>(0xffffffffu - static_cast<uint32_t>(k)) : -1;
    s_pr[g] = p;
    s_lab[g] = lab_of(g);
    if (p >= 0) {
      const int64_t i = static_cast<int64_t>(b) * P + p;
      s_o0[g] = obj[i];
      s_v0[g] = ovl[i];
    }
    s_easy[g] = p >= 0 ? easy_of(p) : 0;
  }
  __syncthreads();
  cnt1 = s_red[15];
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
    s_new[g] = p >= 0 ? j : -1;
    s_easy[g] = p >= 0 ? ((s_easy[g] & 1) | (prev >= 0 ? ((prev + 1) << 1) : 0)) : 0;
  }
  __syncthreads();
  int delta = 0;
  for (int g = tid; g < G; g += blockDim.x) {
    if (s_pr[g] < 0) continue;
    const int easy = s_easy[g] & 1, prev = (s_easy[g] >> 1) - 1;
    const int o_old = prev >= 0 ? s_new[prev] : s_o0[g];
    const float v_old = prev >= 0 ? 1.0f : s_v0[g];
    delta += (is_pos(s_lab[s_new[g]], 1.0f, easy) ? 1 : 0) - (is_pos(s_lab[o_old], v_old, easy) ? 1 : 0);
  }
  delta = block_sum(delta, s_red);
  for (int g = tid; g < G; g += blockDim.x) {
    const int p = s_pr[g];
    if (p < 0) continue;
    bool lastw = true;   // superseded by a later writer?
    for (int h = g + 1; h < G && lastw; ++h)
      if (s_pr[h] == p) lastw = false;
    if (!lastw) continue;
    const int64_t i = static_cast<int64_t>(b) * P + p;
    obj[i] = s_new[g];
    ovl[i] = 1.0f;
  }
  if (tid == 0) publish(delta);
  STAMP_END(7, 1);
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
  r.nw = ((P + kMThreads - 1) / kMThreads) * (kMThreads / 64);
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

int sbod_match_f32(const float *gt_boxes, const int64_t *gt_labels, const int32_t *gt_offsets,
                   int B, int Gmax, const float *anchors, const float *priors_cxcy,
                   const float *arm_scores, int P, float threshold, float theta, int flags,
                   int32_t *obj, float *ovl, int32_t *n_pos, void *workspace,
                   size_t workspace_bytes, void *stream) {
  SBOD_REQUIRE(B > 0 && Gmax > 0 && P > 0 && gt_boxes && gt_labels && gt_offsets && anchors &&
                   obj && ovl && n_pos,
               "sbod_match_f32: bad arguments (B=%d Gmax=%d P=%d)", B, Gmax, P);
  SBOD_REQUIRE(Gmax <= 4096, "sbod_match_f32: Gmax %d > 4096 unsupported", Gmax);
  SBOD_REQUIRE((flags & ~(SBOD_MATCH_BINARY | SBOD_MATCH_ODM | SBOD_MATCH_WS_ZEROED)) == 0,
               "sbod_match_f32: unknown flags 0x%x", flags);
  const bool odm = (flags & SBOD_MATCH_ODM) != 0;
  SBOD_REQUIRE(!odm || (priors_cxcy && arm_scores), "sbod_match_f32: ODM needs priors and arm_scores");
  const size_t need = sbod_match_workspace_bytes_p(B, Gmax, P);
  if (workspace_bytes < need) {
    set_error("sbod_match_f32: workspace %zu < %zu", workspace_bytes, need);
    return SBOD_E_WORKSPACE;
  }
  hipStream_t s = as_stream(stream);
  const int ntile = (P + kMThreads - 1) / kMThreads;
  MatchWs w = carve_match(workspace, B, Gmax, P);
  // the keys and counts must be zero on entry: every call leaves them so (k_match_final), so
  // only a workspace the caller does not know to be clean is zeroed here (not capturable)
  if ((flags & SBOD_MATCH_WS_ZEROED) == 0 && hipMemsetAsync(workspace, 0, w.bytes, s) != hipSuccess)
    return launch_status("hipMemsetAsync");
  dim3 grid(ntile, B);
  const int fthreads = Gmax <= 64 ? 64 : kFThreads;
#define SBOD_MATCH(ODM, FL)                                                                     \
  do {                                                                                          \
    {                                                                                           \
      KernelTimer kt("k_match_tile", s, true);                                                  \
      tlaunch(kt, (k_match_tile<ODM, FL>), grid, dim3(kMThreads), 0, s, gt_boxes, gt_labels,     \
              gt_offsets, anchors, priors_cxcy, arm_scores, P, Gmax, threshold, theta, obj, ovl, \
              w.best, w.wcnt, n_pos, B, kt.span());                                              \
    }                                                                                           \
    SBOD_LAUNCHED("k_match_tile");                                                              \
    KernelTimer kt("k_match_final", s, true);                                                   \
    tlaunch(kt, (k_match_final<FL>), dim3(B), dim3(fthreads),                                   \
            Gmax <= 64 ? 0 : static_cast<size_t>(Gmax) * 24, s, gt_labels, gt_offsets, w.best,  \
            w.wcnt, w.nw, Gmax, P, threshold, arm_scores, theta, obj, ovl, n_pos, B);           \
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

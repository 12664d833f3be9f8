// Device pieces of the anchor matcher (models/SSD512.py:535-572 and its siblings) shared by the
// two-launch matcher (match.hip: k_match_tile + k_match_final) and the one-launch focal
// criterion (loss.hip: k_multibox<..., kFused>), so both run the same arithmetic:
//   match_wave   — one wave's 64 priors against every object of the image: the best object per
//                  prior (first index on ties) and the per-object best-prior keys folded into
//                  the key shards by agent-scope 64-bit atomic max;
//   match_final_image — the forced match of one image (filtered j, last writer wins) and its
//                  positive count, from the key shards and the phase-1 (obj, ovl).
#pragma once

#include "sbod_common.h"

// per-wave phase marks of the diagnostic stamps build (match.hip defines them there)
#ifndef MATCH_WAVE_MARK
#define MATCH_WAVE_MARK(slot, dep) \
  do {                             \
  } while (0)
#endif

namespace sbod {

constexpr int kMThreads = 256;  // matcher tile: one prior per thread
#ifndef SBOD_MATCH_PPL
#define SBOD_MATCH_PPL 1           // priors per lane in k_match_tile (A/B builds: 2, match_wave2)
#endif
constexpr int kMPriors = kMThreads * SBOD_MATCH_PPL;   // priors per k_match_tile workgroup
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

// One lane's phase-1 result: the best object of its prior and that object's label.
struct MatchLane {
  int p, bi, blab;
  float best;
  bool valid;
  float eas0, eas1;   // ODM: the prior's ARM logits (easy-negative test)
};

// match_wave: the calling wave's 64 priors [wbase, wbase + 64) of image b against all its objects.
// No barrier and no block-shared LDS: every wave is independent.
//   lane j holds object j of the current 64-object chunk (box, area, zero flag, label): object g
//     reaches the wave's scalar registers by readlane, so there is no per-object memory access;
//   the wave skips every object whose box misses the bounding box of the wave's priors (the common
//     case: a wave's priors are one small patch of one feature map): every overlap there is <= 0,
//     which can neither raise a prior's best (>= 0 from object 0 on) nor make a key.  The test
//     runs once per chunk as a ballot over the object lanes; the wave walks the set bits;
//   per object: the image's best prior as a packed (ord(overlap) << 32 | ~prior) key (the lowest
//     prior on ties), for overlaps > 0 only (an object whose best overlap is <= 0 is never forced):
//     an object with a positive overlap in this wave leaves its lanes' ords in one of the wave's
//     kSlots LDS rows (s_od, wave-private); flush_keys reduces all filled rows at once — lane =
//     (row, 16-lane segment): the segment's max ord and lowest lane holding it, then the max over
//     the row's 4 segments (DPP) — and folds each row's key into brow[object] with ONE no-return
//     agent-scope 64-bit atomic max (executed at the memory side, so waves on different XCDs meet in
//     one word; kKeyShards words per object, by workgroup, keep the queue per word short).
template <bool kOdm, int kFlags>
__device__ __forceinline__ MatchLane match_wave(const float *__restrict__ gt, const int64_t *__restrict__ labels,
                                                const int32_t *__restrict__ off, const float *__restrict__ anchors,
                                                const float *__restrict__ priors,
                                                const float *__restrict__ arm_scores, int P, int b, int wbase,
                                                unsigned long long *brow, uint32_t (*s_od)[64], int *s_slot,
                                                int g0_in = -1, int G_in = 0) {
  const int lane = threadIdx.x & 63;
  const int p = wbase + lane;
  const bool valid = p < P;
  // one memory round trip before the object loop: the anchor and the first chunk's objects
  // (unconditional, clamped loads; an image without objects reads element 0 — the GT buffers
  // hold at least one, include/sbod.h)
  const int pc = min(p, P - 1);
  const Box4 araw = ld4(kOdm ? anchors + 4 * (static_cast<int64_t>(b) * P + pc) : anchors + 4 * static_cast<int64_t>(pc));
  const Box4 apri = kOdm ? ld4(priors + 4 * pc) : Box4{0.f, 0.f, 0.f, 0.f};
  // the image's object rows: [off[b], off[b+1]) of the packed buffers, or (g0_in >= 0) the
  // G_in rows the caller points gt / labels at (an image's own list, read in place)
  const int g0 = g0_in >= 0 ? g0_in : ld_i32_uniform(off + b);
  const int G = g0_in >= 0 ? G_in : ld_i32_uniform(off + b + 1) - g0;
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
  MATCH_WAVE_MARK(0, wx1 ^ wy2);
  float best = 0.f;
  int bi = 0, blab = 0;
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
  int nslot = 0;
  auto flush_keys = [&]() {
    if (nslot == 0) return;
    __builtin_amdgcn_wave_barrier();
    const int j = lane >> 2, q = lane & 3;
    unsigned long long key = 0ull;
    if (j < nslot) {
      const uint4 *row = reinterpret_cast<const uint4 *>(&s_od[j][16 * q]);
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
      __hip_atomic_fetch_max(brow + s_slot[j], key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_wave_barrier();
    nslot = 0;
  };
  auto note_key = [&](int g, float ov) {
    const uint32_t od = (valid && ov > 0.f) ? f2ord(ov) : 0u;
    if (__ballot(od != 0u) == 0ull) return;   // no positive overlap here: never this wave's key
    s_od[nslot][lane] = od;
    if (lane == 0) s_slot[nslot] = g;
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
    if (gc == 0) MATCH_WAVE_MARK(1, static_cast<uint32_t>(todo));
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
  MATCH_WAVE_MARK(2, __float_as_uint(best) ^ static_cast<uint32_t>(nslot));
  flush_keys();
  MATCH_WAVE_MARK(3, static_cast<uint32_t>(nslot));
  return MatchLane{p, bi, blab, best, valid, eas0, eas1};
}

#if SBOD_MATCH_PPL == 2
// match_wave2 (A/B build -DSBOD_MATCH_PPL=2): match_wave with TWO priors per lane — the wave's
// 128 priors [wbase, wbase + 128), lane l holding wbase + l and wbase + 64 + l — so the tile
// covers 512 priors and the grid is half as large; the object's readlanes are shared by the two
// IoUs and the two chains are independent.  Per prior the same arithmetic in the same object
// order (first index on ties); the per-object key row holds the wave's 128 ords (s_od[slot][128]).
template <bool kOdm, int kFlags>
__device__ __forceinline__ void match_wave2(const float *__restrict__ gt, const int64_t *__restrict__ labels,
                                            const int32_t *__restrict__ off, const float *__restrict__ anchors,
                                            const float *__restrict__ priors, const float *__restrict__ arm_scores,
                                            int P, int b, int wbase, unsigned long long *brow, uint32_t (*s_od)[128],
                                            int *s_slot, int g0_in, int G_in, MatchLane &ra, MatchLane &rb) {
  const int lane = threadIdx.x & 63;
  const int pA = wbase + lane, pB = wbase + 64 + lane;
  const bool validA = pA < P, validB = pB < P;
  const int pcA = min(pA, P - 1), pcB = min(pB, P - 1);
  const Box4 arA = ld4(kOdm ? anchors + 4 * (static_cast<int64_t>(b) * P + pcA) : anchors + 4 * static_cast<int64_t>(pcA));
  const Box4 arB = ld4(kOdm ? anchors + 4 * (static_cast<int64_t>(b) * P + pcB) : anchors + 4 * static_cast<int64_t>(pcB));
  const Box4 apA = kOdm ? ld4(priors + 4 * pcA) : Box4{0.f, 0.f, 0.f, 0.f};
  const Box4 apB = kOdm ? ld4(priors + 4 * pcB) : Box4{0.f, 0.f, 0.f, 0.f};
  const int g0 = g0_in >= 0 ? g0_in : ld_i32_uniform(off + b);
  const int G = g0_in >= 0 ? G_in : ld_i32_uniform(off + b + 1) - g0;
  const bool has = G > 0;
  GtLane o = load_gt_lane<kFlags>(gt, labels, has ? g0 : 0, 0, has ? min(G, 64) : 1, lane);
  float eA0 = 0.f, eA1 = 0.f, eB0 = 0.f, eB1 = 0.f;
  if constexpr (kOdm) {
    const int64_t icA = static_cast<int64_t>(b) * P + pcA, icB = static_cast<int64_t>(b) * P + pcB;
    eA0 = arm_scores[2 * icA];
    eA1 = arm_scores[2 * icA + 1];
    eB0 = arm_scores[2 * icB];
    eB1 = arm_scores[2 * icB + 1];
  }
  const Anchor aA = make_anchor<kOdm>(arA, apA), aB = make_anchor<kOdm>(arB, apB);
  const bool liveA = validA && !aA.zero, liveB = validB && !aB.zero;
  const uint32_t wx1 = ~wave_max_u32(max(liveA ? ~f2ord(aA.x1) : 0u, liveB ? ~f2ord(aB.x1) : 0u));
  const uint32_t wy1 = ~wave_max_u32(max(liveA ? ~f2ord(aA.y1) : 0u, liveB ? ~f2ord(aB.y1) : 0u));
  const uint32_t wx2 = wave_max_u32(max(liveA ? f2ord(aA.x2) : 0u, liveB ? f2ord(aB.x2) : 0u));
  const uint32_t wy2 = wave_max_u32(max(liveA ? f2ord(aA.y2) : 0u, liveB ? f2ord(aB.y2) : 0u));
  const bool wlive = __ballot(liveA || liveB) != 0ull;
  float bestA = 0.f, bestB = 0.f;
  int biA = 0, blabA = 0, biB = 0, blabB = 0;
  // metrics.py:224-250, in the reference's order (as match_wave's iou_of), for both priors
  auto iou2 = [&](int j, int &glab, float &ovA, float &ovB) {
    const float tx1 = rl_f(o.x1, j), ty1 = rl_f(o.y1, j), tx2 = rl_f(o.x2, j), ty2 = rl_f(o.y2, j);
    const float garea = rl_f(o.area, j);
    const int gzero = __builtin_amdgcn_readlane(o.zero, j);
    glab = __builtin_amdgcn_readlane(o.lab, j);
    auto one = [&](const Anchor &a) {
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
    ovA = one(aA);
    ovB = one(aB);
  };
  int nslot = 0;
  auto flush_keys = [&]() {
    if (nslot == 0) return;
    __builtin_amdgcn_wave_barrier();
    const int j = lane >> 2, q = lane & 3;   // row j, 32-prior segment q
    unsigned long long key = 0ull;
    if (j < nslot) {
      const uint4 *row = reinterpret_cast<const uint4 *>(&s_od[j][32 * q]);
      uint32_t v[32];
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const uint4 x = row[r];
        v[4 * r] = x.x;
        v[4 * r + 1] = x.y;
        v[4 * r + 2] = x.z;
        v[4 * r + 3] = x.w;
      }
      uint32_t mx = v[0];
#pragma unroll
      for (int c = 1; c < 32; ++c) mx = max(mx, v[c]);
      int c0 = 31;
#pragma unroll
      for (int c = 30; c >= 0; --c) c0 = v[c] == mx ? c : c0;
      key = mx ? ((static_cast<unsigned long long>(mx) << 32) |
                  (0xffffffffull - static_cast<uint32_t>(wbase + 32 * q + c0)))
               : 0ull;
    }
    key = quad_max_u64(key);
    if (q == 0 && j < nslot && key)
      __hip_atomic_fetch_max(brow + s_slot[j], key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_wave_barrier();
    nslot = 0;
  };
  auto note_key = [&](int g, float ovA, float ovB) {
    const uint32_t odA = (validA && ovA > 0.f) ? f2ord(ovA) : 0u;
    const uint32_t odB = (validB && ovB > 0.f) ? f2ord(ovB) : 0u;
    if (__ballot((odA | odB) != 0u) == 0ull) return;
    s_od[nslot][lane] = odA;
    s_od[nslot][64 + lane] = odB;
    if (lane == 0) s_slot[nslot] = g;
    if (++nslot == kSlots) flush_keys();
  };
  for (int gc = 0; gc < G; gc += 64) {
    const int gn = min(G - gc, 64);
    if (gc > 0) o = load_gt_lane<kFlags>(gt, labels, g0, gc, gn, lane);
    const bool hit = wlive && lane < gn && f2ord(o.x2) > wx1 && f2ord(o.x1) < wx2 && f2ord(o.y2) > wy1 &&
                     f2ord(o.y1) < wy2;
    unsigned long long todo = __ballot(hit) | (gc == 0 ? 1ull : 0ull);
    while (todo) {
      const int j = __builtin_ctzll(todo);
      todo &= todo - 1ull;
      int lab;
      float ovA, ovB;
      iou2(j, lab, ovA, ovB);
      if (gc + j == 0 || ovA > bestA) {
        bestA = ovA;
        biA = gc + j;
        blabA = lab;
      }
      if (gc + j == 0 || ovB > bestB) {
        bestB = ovB;
        biB = gc + j;
        blabB = lab;
      }
      note_key(gc + j, ovA, ovB);
    }
  }
  flush_keys();
  ra = MatchLane{pA, biA, blabA, bestA, validA, eA0, eA1};
  rb = MatchLane{pB, biB, blabB, bestB, validB, eB0, eB1};
}
#endif

// The positive rule of the criteria before the forced match (label of the best object, overlap
// threshold; ODM: easy negatives excluded, RefineDet512.py:894-899).
template <bool kOdm>
__device__ __forceinline__ bool phase1_positive(const MatchLane &m, float thr, float theta) {
  bool pos = m.valid && !(m.best < thr) && m.blab > 0;
  if constexpr (kOdm) {
    const float mx = fmaxf(m.eas0, m.eas1);
    const float e0 = expf(m.eas0 - mx), e1 = expf(m.eas1 - mx);
    if (e1 / (e0 + e1) < theta) pos = false;
  }
  return pos;
}

// In-launch outputs of the forced match (one-launch criterion only).
struct ForcedOut {
  unsigned long long *list;   // [B][Gmax] (prior << 32 | object j) of the priors the forced match rewrites
  int32_t *count;             // [B] entries of each image's list
  unsigned long long *done;   // (images finished << 32) | their positives, agent-scope atomic adds
};

// match_final_image: the forced match of models/SSD512.py:546-553 for image b (filter objects
// whose best overlap > 0, overlap 1.0 and object j = the FILTERED position, last writer wins)
// against the phase-1 (obj, ovl) of each forced prior, and the image's positive count adjusted for
// exactly the priors it rewrites.  Up to 64 objects it is ONE wave (wave 0), lane = object,
// everything in registers (ballots, readlanes, bpermutes); more objects take the LDS form over
// the whole workgroup (s_dyn: 24 * Gmax bytes; s_red: 16 ints).  The image's keys are left zero.
// Must be reached by every thread of the workgroup (barriers inside).
//   kFused = false (k_match_final): cnt1 is summed from the per-wave counts `wcnt` (left zero),
//     keys / (obj, ovl) are plain loads of the previous launch's stores, the results are plain
//     stores and the count goes to npos[b] and npos[B] (atomic);
//   kFused = true (one-launch criterion, k_multibox): cnt1 comes from the image's arrival word;
//     the keys are taken by agent-scope exchanges, the phase-1 (obj, ovl) read with sc1 loads (their
//     writers stored them write-through and drained before arriving), the rewrites stored
//     write-through and listed in fo.list, and fo.done counts the image in once every list entry
//     is drained.
template <int kFlags, bool kFused>
__device__ __forceinline__ void match_final_image(
    int b, const int64_t *__restrict__ labels, const int32_t *__restrict__ off, unsigned long long *best_key,
    int32_t *wcnt, int nw, int Gmax, int P, float thr, const float *__restrict__ arm_scores, float theta,
    int32_t *obj, float *ovl, int32_t *npos, int B, int cnt1_fused, const ForcedOut &fo, unsigned char *s_dyn,
    int *s_red) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int g0 = off[b], G = off[b + 1] - g0;
  unsigned long long *brow = best_key + static_cast<int64_t>(b) * kKeyShards * Gmax;
  // the phase-1 positive count: the image's per-wave counts (first wave only; the LDS form
  // shares it through s_red)
  int cnt1 = 0;
  if constexpr (kFused) {
    cnt1 = cnt1_fused;
  } else if (tid < 64) {
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
    if constexpr (kFused) {
#pragma unroll
      for (int s = 0; s < kKeyShards; ++s) {
        const unsigned long long v =
            __hip_atomic_exchange(brow + s * Gmax + g, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        k = v > k ? v : k;
      }
    } else {
#pragma unroll
      for (int s = 0; s < kKeyShards; ++s) {
        const unsigned long long v = brow[s * Gmax + g];
        k = v > k ? v : k;
      }
#pragma unroll
      for (int s = 0; s < kKeyShards; ++s) brow[s * Gmax + g] = 0ull;
    }
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
  auto ld_obj = [&](int64_t i) { return kFused ? static_cast<int>(ld_wt_u32(obj + i)) : obj[i]; };
  auto ld_ovl = [&](int64_t i) {
    return kFused ? __uint_as_float(ld_wt_u32(reinterpret_cast<const int32_t *>(ovl) + i)) : ovl[i];
  };
  auto write_forced = [&](int p, int j, int slot) {
    const int64_t i = static_cast<int64_t>(b) * P + p;
    if constexpr (kFused) {
      st_wt_u32(obj + i, static_cast<uint32_t>(j));
      st_wt_u32(reinterpret_cast<int32_t *>(ovl) + i, __float_as_uint(1.0f));
      st_wt_u64(fo.list + static_cast<int64_t>(b) * Gmax + slot,
                (static_cast<unsigned long long>(p) << 32) | static_cast<uint32_t>(j));
    } else {
      obj[i] = j;
      ovl[i] = 1.0f;
    }
  };
  // is_pos(label, overlap, easy): the positive rule of the criteria
  auto is_pos = [&](int lab, float v, int easy) { return !(v < thr) && lab > 0 && !easy; };
  auto publish = [&](int delta, int nforced) {   // one lane, after the workgroup's stores are drained
    const int nb = cnt1 + delta;
    npos[b] = nb;
    if constexpr (kFused) {
      st_wt_u32(fo.count + b, static_cast<uint32_t>(nforced));
      drain_vm();
      __hip_atomic_fetch_add(fo.done, (1ull << 32) | static_cast<uint32_t>(nb), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    } else {
      atomicAdd(npos + B, nb);
    }
  };
  if (G <= 64) {
    if (tid < 64) {
      // lane = object: its best key, the key's prior and that prior's phase-1 (obj, ovl)
      const unsigned long long k = lane < G ? take_key(lane) : 0ull;
      const int lab = lane < G ? lab_of(lane) : 0;
      const int p = k ? static_cast<int>(0xffffffffu - static_cast<uint32_t>(k)) : -1;
      const int64_t ip = static_cast<int64_t>(b) * P + (p >= 0 ? p : 0);
      const int o_ph1 = ld_obj(ip);
      const float v_ph1 = ld_ovl(ip);
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
      const unsigned long long wl = __ballot(p >= 0 && lastw);
      if (p >= 0) {
        d = (is_pos(lab_new, 1.0f, easy) ? 1 : 0) - (is_pos(lab_old, v_old, easy) ? 1 : 0);
        if (lastw) write_forced(p, j, __popcll(wl & ((1ull << lane) - 1ull)));
      }
      const int delta = wave_sum_i32(d);
      if (kFused) drain_vm();
      if (lane == 0) publish(delta, __popcll(wl));
    }
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
  if (tid == 0) {
    s_red[15] = cnt1;
    s_red[14] = 0;   // forced-list slots taken
  }
  for (int g = tid; g < G; g += blockDim.x) {
    const unsigned long long k = take_key(g);
    const int p = k ? static_cast<int>(0xffffffffu - static_cast<uint32_t>(k)) : -1;
    s_pr[g] = p;
    s_lab[g] = lab_of(g);
    if (p >= 0) {
      const int64_t i = static_cast<int64_t>(b) * P + p;
      s_o0[g] = ld_obj(i);
      s_v0[g] = ld_ovl(i);
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
    write_forced(p, s_new[g], kFused ? atomicAdd(&s_red[14], 1) : 0);
  }
  if (kFused) drain_vm();
  __syncthreads();
  if (tid == 0) publish(delta, kFused ? s_red[14] : 0);
}

}  // namespace sbod

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
// k_match_tile (B x ceil(P / 256) workgroups, one prior per thread; 2 and 4 consecutive priors
// per thread measured slower: fewer waves to hide the per-object latency chain):
//   per prior: the best object (first index on ties) -> obj / ovl;
//   per object: this tile's best prior as a packed (ord(overlap) << 32 | ~prior) key (the lowest
//     prior on ties), for overlaps > 0 only (an object whose best overlap is <= 0 is never
//     forced, so every such key may read 0).  No cross-lane work in the object loop: each thread
//     leaves its overlap's ord per object in LDS, and after the loop one pass reduces the
//     [objects x priors] table (a thread per (object, 16-prior segment), then a DPP max over the
//     16 lanes holding one object) -> one 16-byte record per (tile, object) {key, obj and ovl of
//     the key's prior (-1 when not known: objects beyond one LDS chunk)};
//   a wave whose priors overlap none of an object (the common case: a wave's priors are one
//     small patch of one feature map) skips that object's divisions: every overlap there is
//     <= 0, which can neither raise a prior's best (>= 0 from object 0 on) nor make a key;
//   the tile's positive count before the forced match -> tcount.
// k_match_final (one workgroup per image): every record of the image in flight at once, the max
// key per object through LDS, then the forced match of models/SSD512.py:546-553 (filter objects
// whose best overlap > 0, overlap 1.0 and object j = the FILTERED position, last writer wins),
// the positive count adjusted for exactly the priors it rewrites -> n_pos[b], n_pos[B].  Up to 64
// objects the forced match runs in wave 0's registers (lane = object: ballots, readlanes and one
// permute, no barrier); more objects take the LDS form.
// (An in-launch finish by each image's last-arriving tile, with write-through records and
// arrival counters, measured slower: the write-through drain, the counter round trip and the
// fabric-latency record loads cost more than this launch boundary — DESIGN.md §9.)
constexpr int kGc = 16;       // objects per chunk of the per-thread best table in LDS
constexpr int kSegCols = 16;  // threads (columns) per first-pass reduction segment
constexpr int kNSeg = kMThreads / kSegCols;

struct MRec {   // 16-byte (tile, object) record
  unsigned long long key;
  int32_t obj;
  float ovl;
};

// Max of a u64 over each row of 16 lanes, valid in every lane of the row (DPP quad swaps and
// mirrors; keys are unique, so the max is the row's best).
template <int kCtrl>
__device__ __forceinline__ unsigned long long dpp_max_u64(unsigned long long v) {
  const uint32_t lo = dpp_u32<kCtrl, 0xf>(static_cast<uint32_t>(v));
  const uint32_t hi = dpp_u32<kCtrl, 0xf>(static_cast<uint32_t>(v >> 32));
  const unsigned long long o = (static_cast<unsigned long long>(hi) << 32) | lo;
  return o > v ? o : v;
}
__device__ __forceinline__ unsigned long long row16_max_u64(unsigned long long v) {
  v = dpp_max_u64<0xB1>(v);    // quad_perm [1,0,3,2]
  v = dpp_max_u64<0x4E>(v);    // quad_perm [2,3,0,1]
  v = dpp_max_u64<0x141>(v);   // row_half_mirror
  return dpp_max_u64<0x140>(v);   // row_mirror
}

template <bool kOdm, int kFlags>
__global__ __launch_bounds__(kMThreads) void k_match_tile(
    const float *__restrict__ gt, const int64_t *__restrict__ labels,
    const int32_t *__restrict__ off, const float *__restrict__ anchors,
    const float *__restrict__ priors, const float *__restrict__ arm_scores, int P, int Gmax,
    float thr, float theta, int32_t *__restrict__ obj, float *__restrict__ ovl,
    MRec *__restrict__ rec, int32_t *__restrict__ tcount, int32_t *__restrict__ npos, int B,
    SpanRing *span) {
  // dynamic LDS: [4 * max(Gmax, kMThreads) labels]
  extern __shared__ __attribute__((aligned(16))) unsigned char s_dyn[];
  __shared__ __attribute__((aligned(16))) uint32_t s_ord[kGc][kMThreads];  // per object, per prior: ord
  __shared__ uint32_t s_ev[kMThreads / 64];                                 // per wave: objects evaluated
  __shared__ int32_t s_fo[kMThreads];                                       // final (obj, ovl) per prior
  __shared__ float s_fv[kMThreads];
  __shared__ int s_red[16];
  __shared__ float4 s_gt[kMThreads];   // this chunk's GT boxes: slot j < 16 = object gc + j
  STAMP_BEGIN();
  span_begin(span);
  PHASE_DECL;
  SEG_PHASE(0);
  int32_t *s_lab = reinterpret_cast<int32_t *>(s_dyn);
  const int b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int ntile = gridDim.x;
  if (blockIdx.x == 0 && b == 0 && tid == 0) npos[B] = 0;   // k_match_final accumulates
  const int tbase = blockIdx.x * kMThreads;
  const int p = tbase + tid;
  const bool valid = p < P;
  // ONE memory round trip before the object loop: the anchor, the first chunk's GT boxes and the
  // labels are loaded together (unconditional, clamped) and committed to LDS by unconditional
  // stores before the first barrier, so no load sits under a branch where the compiler would
  // sink it behind the anchor's wait; the object loop then reads the boxes from LDS instead of a
  // scalar load round trip per group of objects.  An image without objects reads element 0 (the
  // GT buffers hold at least one); s_lab has room for max(Gmax, kMThreads) labels.
  const int pc = min(p, P - 1);
  const Box4 araw = ld4(kOdm ? anchors + 4 * (static_cast<int64_t>(b) * P + pc) : anchors + 4 * static_cast<int64_t>(pc));
  const Box4 apri = kOdm ? ld4(priors + 4 * pc) : Box4{0.f, 0.f, 0.f, 0.f};
  const int g0 = ld_i32_uniform(off + b), G = ld_i32_uniform(off + b + 1) - g0;
  const Box4 gt0 = ld4(gt + 4 * static_cast<int64_t>(G > 0 ? g0 + min(tid & (kGc - 1), G - 1) : 0));
  const int32_t lab0 = static_cast<int32_t>(labels[G > 0 ? g0 + min(tid, G - 1) : 0]);
  const Anchor a = make_anchor<kOdm>(araw, apri);
  s_gt[tid] = make_float4(gt0.a, gt0.b, gt0.c, gt0.d);
  s_lab[tid] = lab0;
  for (int i = tid + kMThreads; i < G; i += kMThreads) s_lab[i] = static_cast<int32_t>(labels[g0 + i]);
  // the wave's prior bounding box as monotone integer keys, so each object's "does any prior of
  // this wave overlap it" test runs on the scalar unit: an object outside the box has
  // iw <= 0 or ih <= 0 for every prior of the wave (overlap 0 or -1, never a key, never a new
  // best after object 0), so its divisions are skipped exactly
  const bool live = valid && !a.zero;
  const uint32_t wx1 = ~wave_max_u32(live ? ~f2ord(a.x1) : 0u), wy1 = ~wave_max_u32(live ? ~f2ord(a.y1) : 0u);
  const uint32_t wx2 = wave_max_u32(live ? f2ord(a.x2) : 0u), wy2 = wave_max_u32(live ? f2ord(a.y2) : 0u);
  const bool wlive = __ballot(live) != 0ull;
  SEG_PHASE(1);
  float best = 0.f;
  int bi = 0;
  const bool one_chunk = G <= kGc;
  MRec *rrow = rec + (static_cast<int64_t>(b) * ntile + blockIdx.x) * Gmax;
  for (int gc = 0; gc < G; gc += kGc) {
    const int gn = min(G - gc, kGc);
    if (gc > 0) {   // later chunks: their boxes into LDS (the previous chunk's end barrier is behind)
      const Box4 bx = ld4(gt + 4 * static_cast<int64_t>(g0 + gc + min(tid & (kGc - 1), gn - 1)));
      s_gt[tid] = make_float4(bx.a, bx.b, bx.c, bx.d);
    }
    __syncthreads();
    uint32_t ev = 0u;   // objects of this chunk evaluated by this wave (wave-uniform)
    for (int j0 = 0; j0 < gn; j0 += 4) {
      Box4 t[4];   // LDS broadcast reads made scalar: the wave-box test runs on the scalar unit
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float4 v = s_gt[min(j0 + u, gn - 1)];
        t[u] = Box4{__int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v.x))),
                    __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v.y))),
                    __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v.z))),
                    __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v.w)))};
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int j = j0 + u;
        if (j >= gn) break;
        const int g = gc + j;
        const bool hitw = wlive && f2ord(t[u].c) > wx1 && f2ord(t[u].a) < wx2 && f2ord(t[u].d) > wy1 &&
                          f2ord(t[u].b) < wy2;
        // object 0 is always evaluated (it sets every prior's first best, ties included)
        if (g == 0 || hitw) {   // metrics.py:224-250, in the reference's order
          const float gx = t[u].c - t[u].a, gy = t[u].d - t[u].b;
          const float garea = gx * gy;
          const bool gzero = (fabsf(gx) < kIouEps) && (fabsf(gy) < kIouEps);
          float iw = fminf(t[u].c, a.x2) - fmaxf(t[u].a, a.x1);
          if (iw < 0.f) iw = 0.f;
          float ih = fminf(t[u].d, a.y2) - fmaxf(t[u].b, a.y1);
          if (ih < 0.f) ih = 0.f;
          const float inner = iw * ih;
          float ov = inner / (((garea + a.area) - inner) + kIouEps);
          if (gzero) ov = 0.f;
          if (a.zero) ov = -1.f;
          if (g == 0 || ov > best) {
            best = ov;
            bi = g;
          }
          s_ord[j][tid] = (valid && ov > 0.f) ? f2ord(ov) : 0u;
          ev |= 1u << j;
        }
      }
    }
    if (lane == 0) s_ev[wv] = ev;
    if (one_chunk) {
      s_fo[tid] = bi;
      s_fv[tid] = best;
    }
    __syncthreads();
    // thread -> (object j = tid / 16, segment sg = tid % 16 of 16 priors): the segment's best
    // (ord, lowest prior), then the max over the row of 16 lanes = the tile's key of object j
    {
      const int j = tid / kNSeg, sg = tid - j * kNSeg;
      unsigned long long kb = 0ull;
      if (j < gn && ((s_ev[sg / (64 / kSegCols)] >> j) & 1u)) {
        const uint4 *row = reinterpret_cast<const uint4 *>(&s_ord[j][sg * kSegCols]);
        uint32_t v[kSegCols];
#pragma unroll
        for (int q = 0; q < kSegCols / 4; ++q) {
          const uint4 x = row[q];
          v[4 * q] = x.x;
          v[4 * q + 1] = x.y;
          v[4 * q + 2] = x.z;
          v[4 * q + 3] = x.w;
        }
        uint32_t m8[8], m4[4];
#pragma unroll
        for (int c = 0; c < 8; ++c) m8[c] = max(v[c], v[c + 8]);
#pragma unroll
        for (int c = 0; c < 4; ++c) m4[c] = max(m8[c], m8[c + 4]);
        const uint32_t mx = max(max(m4[0], m4[2]), max(m4[1], m4[3]));
        uint32_t mask = 0u;
#pragma unroll
        for (int c = 0; c < kSegCols; ++c) mask |= (v[c] == mx ? 1u : 0u) << c;
        const int c0 = __builtin_ctz(mask);   // mask != 0: mx is one of v
        kb = mx ? ((static_cast<unsigned long long>(mx) << 32) |
                   (0xffffffffull - static_cast<uint32_t>(tbase + sg * kSegCols + c0)))
                : 0ull;
      }
      kb = row16_max_u64(kb);
      if (sg == 0 && j < gn) {
        // the prior's final (obj, ovl) when every object is in this chunk
        int32_t o = -1;
        float v = 0.f;
        if (one_chunk && kb) {
          const int lp = static_cast<int>(0xffffffffu - static_cast<uint32_t>(kb)) - tbase;
          o = s_fo[lp];
          v = s_fv[lp];
        }
        rrow[gc + j] = MRec{kb, o, v};
      }
    }
    if (gc + kGc < G) __syncthreads();   // s_ord / s_ev are rewritten by the next chunk
  }
  SEG_PHASE(2);
  int pos = 0;
  if (valid) {
    const int64_t i = static_cast<int64_t>(b) * P + p;
    obj[i] = bi;
    ovl[i] = best;
    int c = best < thr ? 0 : s_lab[bi];
    if ((kFlags & SBOD_MATCH_BINARY) != 0) c = c > 0;
    pos = c > 0;
    if constexpr (kOdm) {
      const float z0 = arm_scores[2 * i], z1 = arm_scores[2 * i + 1];
      const float m = fmaxf(z0, z1);
      const float e0 = expf(z0 - m), e1 = expf(z1 - m);
      if (e1 / (e0 + e1) < theta) pos = 0;
    }
  }
  pos = block_sum(pos, s_red);
  if (tid == 0) tcount[b * ntile + blockIdx.x] = pos;
  span_end(span);
  SEG_PHASE(3);
#ifdef SBOD_PHASE_CLOCKS
  if (PHASE_PRINT_SEL)
    printf("match_tile x%d b%d G=%d: start %lld objects+keys %lld store+sum %lld total %lld\n", blockIdx.x, b, G,
           ph[1] - ph[0], ph[2] - ph[1], ph[3] - ph[2], ph[3] - ph[0]);
#endif
  STAMP_END(5, 1);
}

// k_match_final: one workgroup of kFThreads per image.
constexpr int kFThreads = 256;
constexpr int kFRegs = 4;   // records per thread kept in registers (G * ntile <= 1024)

template <int kFlags>
__global__ __launch_bounds__(kFThreads) void k_match_final(
    const int64_t *__restrict__ labels, const int32_t *__restrict__ off, const MRec *__restrict__ rec,
    const int32_t *__restrict__ tcount, int ntile, int Gmax, int P, float thr,
    const float *__restrict__ arm_scores, float theta, int32_t *__restrict__ obj,
    float *__restrict__ ovl, int32_t *__restrict__ npos, int B) {
  // LDS per object g: best key, its prior's phase-1 (obj, ovl), label; the LDS forced-match
  // form also uses prior / easy | previous writer / final object
  extern __shared__ __attribute__((aligned(16))) unsigned char s_dyn[];
  unsigned long long *s_best = reinterpret_cast<unsigned long long *>(s_dyn);
  int32_t *s_o0 = reinterpret_cast<int32_t *>(s_best + Gmax);
  float *s_v0 = reinterpret_cast<float *>(s_o0 + Gmax);
  int32_t *s_lab = reinterpret_cast<int32_t *>(s_v0 + Gmax);
  int32_t *s_pr = s_lab + Gmax;
  int32_t *s_easy = s_pr + Gmax;
  int32_t *s_new = s_easy + Gmax;
  __shared__ int s_red[16];
  __shared__ int s_cnt;
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int g0 = off[b], G = off[b + 1] - g0;
  const MRec *rb = rec + static_cast<int64_t>(b) * ntile * Gmax;
  const int n = G * ntile;
  const bool inreg = n <= kFRegs * kFThreads;
  // every record of the image (and the tile counts) in flight at once
  MRec r[kFRegs];
#pragma unroll
  for (int q = 0; q < kFRegs; ++q) {
    const int it = min(tid + q * kFThreads, max(n - 1, 0));
    const int g = it / ntile, t = it - g * ntile;
    r[q] = (inreg && n > 0) ? rb[static_cast<int64_t>(t) * Gmax + g] : MRec{0ull, 0, 0.f};
  }
  int cnt = 0;
  for (int t = tid; t < ntile; t += kFThreads) cnt += tcount[b * ntile + t];
  for (int g = tid; g < G; g += kFThreads) {
    s_best[g] = 0ull;
    s_lab[g] = static_cast<int32_t>(labels[g0 + g]);
  }
  if (tid == 0) s_cnt = 0;
  __syncthreads();
  cnt = wave_sum_i32(cnt);
  if (lane == 0 && cnt) atomicAdd(&s_cnt, cnt);
  if (inreg) {
#pragma unroll
    for (int q = 0; q < kFRegs; ++q) {
      const int it = tid + q * kFThreads;
      if (it < n && r[q].key) atomicMax(&s_best[it / ntile], r[q].key);
    }
  } else {
    for (int it = tid; it < n; it += kFThreads) {
      const int g = it / ntile, t = it - g * ntile;
      const unsigned long long k = rb[static_cast<int64_t>(t) * Gmax + g].key;
      if (k) atomicMax(&s_best[g], k);
    }
  }
  __syncthreads();
  // the winning record of each object supplies its prior's phase-1 (obj, ovl)
  auto take = [&](int g, const MRec &x) {
    if (x.key && x.key == s_best[g]) {
      int32_t o = x.obj;
      float v = x.ovl;
      if (o < 0) {   // not carried (more objects than one tile chunk): phase 1's outputs
        const int64_t i = static_cast<int64_t>(b) * P + static_cast<int>(0xffffffffu - static_cast<uint32_t>(x.key));
        o = obj[i];
        v = ovl[i];
      }
      s_o0[g] = o;
      s_v0[g] = v;
    }
  };
  if (inreg) {
#pragma unroll
    for (int q = 0; q < kFRegs; ++q) {
      const int it = tid + q * kFThreads;
      if (it < n) take(it / ntile, r[q]);
    }
  } else {
    for (int it = tid; it < n; it += kFThreads) {
      const int g = it / ntile, t = it - g * ntile;
      take(g, rb[static_cast<int64_t>(t) * Gmax + g]);
    }
  }
  __syncthreads();
  const int cnt1 = s_cnt;
  auto is_pos = [&](int o, float v, int easy) {
    int c = v < thr ? 0 : s_lab[o];
    if ((kFlags & SBOD_MATCH_BINARY) != 0) c = c > 0;
    return c > 0 && !easy;
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
  auto publish = [&](int delta) {   // one lane
    const int nb = cnt1 + delta;
    npos[b] = nb;
    atomicAdd(npos + B, nb);
  };
  if (G <= 64) {
    if (wv == 0) {   // lane = object, everything in registers
      const unsigned long long k = lane < G ? s_best[lane] : 0ull;
      const int p = k ? static_cast<int>(0xffffffffu - static_cast<uint32_t>(k)) : -1;
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
      int d = 0;
      if (p >= 0) {
        const int easy = easy_of(p);
        const int o_old = prev >= 0 ? jprev : s_o0[lane];
        const float v_old = prev >= 0 ? 1.0f : s_v0[lane];
        d = (is_pos(j, 1.0f, easy) ? 1 : 0) - (is_pos(o_old, v_old, easy) ? 1 : 0);
        if (lastw) {
          const int64_t i = static_cast<int64_t>(b) * P + p;
          obj[i] = j;
          ovl[i] = 1.0f;
        }
      }
      const int delta = wave_sum_i32(d);
      if (lane == 0) publish(delta);
    }
    return;
  }
  // more objects: the LDS form of the same rules
  for (int g = tid; g < G; g += kFThreads) {
    const unsigned long long k = s_best[g];
    const int p = k ? static_cast<int>(0xffffffffu - static_cast<uint32_t>(k)) : -1;
    s_pr[g] = p;
    s_easy[g] = p >= 0 ? easy_of(p) : 0;
  }
  __syncthreads();
  for (int g = tid; g < G; g += kFThreads) {
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
  for (int g = tid; g < G; g += kFThreads) {
    if (s_pr[g] < 0) continue;
    const int easy = s_easy[g] & 1, prev = (s_easy[g] >> 1) - 1;
    const int o_old = prev >= 0 ? s_new[prev] : s_o0[g];
    const float v_old = prev >= 0 ? 1.0f : s_v0[g];
    delta += (is_pos(s_new[g], 1.0f, easy) ? 1 : 0) - (is_pos(o_old, v_old, easy) ? 1 : 0);
  }
  delta = block_sum(delta, s_red);
  for (int g = tid; g < G; g += kFThreads) {
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
// Matcher workspace: the per-(tile, object) 16-byte records [B][ntile][Gmax], then the per-tile
// positive counts [B][ntile].
struct MatchWs {
  MRec *rec;
  int32_t *tcount;
  size_t bytes;
};
MatchWs carve_match(void *w, int B, int Gmax, int P) {
  const size_t ntile = (P + kMThreads - 1) / kMThreads;
  MatchWs r;
  size_t o = 0;
  r.rec = ws_at<MRec>(w, o);
  o += align_up(static_cast<size_t>(B) * ntile * Gmax * sizeof(MRec));
  r.tcount = ws_at<int32_t>(w, o);
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
  const int ntile = (P + kMThreads - 1) / kMThreads;
  MatchWs w = carve_match(workspace, B, Gmax, P);
  dim3 grid(ntile, B);
#define SBOD_MATCH(ODM, FL)                                                                     \
  do {                                                                                          \
    {                                                                                           \
      KernelTimer kt("k_match_tile", s, true);                                                  \
      tlaunch(kt, (k_match_tile<ODM, FL>), grid, dim3(kMThreads),                                \
              static_cast<size_t>(Gmax > kMThreads ? Gmax : kMThreads) * 4, s,                      \
              gt_boxes, gt_labels, gt_offsets, anchors, priors_cxcy, arm_scores, P, Gmax, threshold, \
              theta, obj, ovl, w.rec, w.tcount, n_pos, B, kt.span());                           \
    }                                                                                           \
    SBOD_LAUNCHED("k_match_tile");                                                              \
    KernelTimer kt("k_match_final", s, true);                                                   \
    tlaunch(kt, (k_match_final<FL>), dim3(B), dim3(kFThreads), static_cast<size_t>(Gmax) * 32, s, \
            gt_labels, gt_offsets, w.rec, w.tcount, ntile, Gmax, P, threshold, arm_scores, theta, \
            obj, ovl, n_pos, B);                                                                \
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

// Box decode + batched per-class NMS + top-k (models/utils.py:181-297, detect_scripts/
// detect_tools.py:100-341) and single-segment greedy NMS (iou_utils.nms / diounms,
// torchvision.ops.nms semantics).
//
// detect() pipeline (three launches + one memset, no host sync):
//   K1 k_det_prepare  (B x P/256 workgroups): decode + clamp, softmax / sigmoid over the LDS
//      score tile, and per-(image, class) candidate compaction with wave-aggregated atomics
//      (64-bit keys: ord(score) << 32 | ~prior, unique, so every later order is deterministic).
//   K2 k_det_segment  ((C-1) x B workgroups): the top-Q window of each class (full LDS sort, or
//      an 8-pass radix select when the segment is larger than the LDS) and greedy NMS over it.
//      A box's kept status depends only on higher-scored boxes of its own class, so the window
//      decides exactly the kept status of its Q best candidates.
//   K3 k_det_merge    (B workgroups): merge the classes' kept windows, apply top_k (and the
//      detect_tools class-agnostic final NMS), and check that no candidate outside a truncated
//      window could rank among the outputs; if one could, det_count = -1 and the host re-runs
//      with the full window (exactness never depends on the window size).
// The reference processes every candidate of every class (~1,300 x 20 per image at SSD512
// with ~80 % kept); only the first top_k outputs are observable, which is what makes the
// window exact and cheap.
#include "sbod_common.h"

namespace sbod {

SBOD_STAMP_DECL

#ifndef SBOD_DTILE
#define SBOD_DTILE 256
#endif
constexpr int kDTile = SBOD_DTILE;   // k_det_prepare's rows per workgroup (A/B builds: -DSBOD_DTILE=128)
#ifndef SBOD_PREP_GLDS
#define SBOD_PREP_GLDS 1
#endif
__device__ const uint8_t kOneByte = 1;
constexpr int kSegThreads = 256;
constexpr int kMaxWindow = 4096;   // LDS-resident window (keys + boxes + areas + flags)
constexpr int kMergeThreads = 1024;
constexpr int kMergeStage = 2048;  // merged entries ordered for the final class-agnostic NMS (general path)

__device__ __forceinline__ unsigned long long make_key(float score, uint32_t low) {
  return (static_cast<unsigned long long>(f2ord(score)) << 32) | (0xffffffffu - low);
}
__device__ __forceinline__ float key_score(unsigned long long k) { return ord2f(static_cast<uint32_t>(k >> 32)); }
__device__ __forceinline__ uint32_t key_low(unsigned long long k) { return 0xffffffffu - static_cast<uint32_t>(k); }

// Suppression test of candidate j by the higher-ranked kept box i.
//   TV   (torchvision.ops.nms): iou = inter / ((a_i + a_j) - inter), suppress iff iou > thr.
//   REF  (iou_utils.py:440-448): iou = inter / ((a_j - inter) + a_i), suppress iff !(iou <= thr).
//   DIOU (iou_utils.py:495-528): REF minus (d / c)^beta with center_y2 = (yy2 + yy2) / 2.
template <int V>
__device__ __forceinline__ bool suppresses(const Box4 &bi, float ai, const Box4 &bj, float aj,
                                           float thr, float beta) {
  const float xx1 = fmaxf(bj.a, bi.a), yy1 = fmaxf(bj.b, bi.b);
  const float xx2 = fminf(bj.c, bi.c), yy2 = fminf(bj.d, bi.d);
  const float w = fmaxf(xx2 - xx1, 0.f), h = fmaxf(yy2 - yy1, 0.f);
  const float inter = w * h;
  if constexpr (V == SBOD_NMS_TV) {
    const float u = (ai + aj) - inter;
    if (u > 0.f && u < 3.0e38f) {       // decide without dividing unless within 2^-18 of thr
      const float t = thr * u;
      if (inter > t * (1.f + 3.8147e-6f)) return true;
      if (inter < t * (1.f - 3.8147e-6f)) return false;
    }
    return inter / u > thr;
  } else {
    float iou = inter / ((aj - inter) + ai);
    if constexpr (V == SBOD_NMS_DIOU) {
      const float cx1 = (bi.a + bi.c) / 2.f, cy1 = (bi.b + bi.d) / 2.f;
      const float cx2 = (bj.a + bj.c) / 2.f, cy2 = (bj.d + bj.d) / 2.f;
      const float dx = cx1 - cx2, dy = cy1 - cy2;
      const float d = dx * dx + dy * dy;
      const float ex1 = fminf(bj.a, bi.a), ey1 = fminf(bj.b, bi.b);
      const float ex2 = fmaxf(bj.c, bi.c), ey2 = fmaxf(bj.d, bi.d);
      const float c = (ex2 - ex1) * (ex2 - ex1) + (ey2 - ey1) * (ey2 - ey1);
      const float u = d / c;
      iou = iou - (beta == 1.f ? u : powf(u, beta));
    }
    return !(iou <= thr);
  }
}

// Branch-free torchvision test for wave code: sup is decided by the +-2^-18 margin; `amb`
// marks the rare lanes that need the exact division (then done under a wave-uniform branch).
__device__ __forceinline__ bool tv_fast(const Box4 &bi, float ai, const Box4 &bj, float aj, float thr,
                                        bool &amb, float &inter, float &u) {
  const float xx1 = fmaxf(bj.a, bi.a), yy1 = fmaxf(bj.b, bi.b);
  const float xx2 = fminf(bj.c, bi.c), yy2 = fminf(bj.d, bi.d);
  const float w = fmaxf(xx2 - xx1, 0.f), h = fmaxf(yy2 - yy1, 0.f);
  inter = w * h;
  u = (ai + aj) - inter;
  const float t = thr * u;
  const bool hi = inter > t * (1.f + 3.8147e-6f);
  const bool lo = inter < t * (1.f - 3.8147e-6f);
  const bool ok = u > 0.f && u < 3.0e38f;
  amb = !(ok && (hi || lo));
  return ok && hi;
}

__device__ __forceinline__ int next_pow2(int x) {
  int p = 1;
  while (p < x) p <<= 1;
  return p;
}

// Descending bitonic sort of N (power of two) 64-bit keys in LDS; every thread owns whole
// compare-exchange pairs (no idle lanes).
__device__ void bitonic_desc(unsigned long long *s, int N) {
  const int half = N >> 1;
  for (int k = 2; k <= N; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int q = threadIdx.x; q < half; q += blockDim.x) {
        const int i = ((q & ~(j - 1)) << 1) | (q & (j - 1));   // lower index of pair q
        const int ixj = i | j;
        const unsigned long long a = s[i], b = s[ixj];
        const bool up = (i & k) == 0;
        if (up ? (a < b) : (a > b)) {
          s[i] = b;
          s[ixj] = a;
        }
      }
      __syncthreads();
    }
  }
}

// Global -> LDS copy of n u64 keys, zero-padded to N (>= n): 8 loads in flight per thread before
// the LDS stores (a plain copy loop waits one HBM round trip per element).
__device__ __forceinline__ void block_copy_keys(unsigned long long *__restrict__ dst,
                                                const unsigned long long *__restrict__ src, int n, int N) {
  constexpr int kBatch = 8;
  const int nt = blockDim.x;
  for (int base = 0; base < N; base += kBatch * nt) {
    unsigned long long r[kBatch];
#pragma unroll
    for (int k = 0; k < kBatch; ++k) {
      const int i = base + k * nt + threadIdx.x;
      const unsigned long long v = src[min(i, max(n - 1, 0))];   // unconditional: keeps r in VGPRs
      r[k] = i < n ? v : 0ull;
    }
#pragma unroll
    for (int k = 0; k < kBatch; ++k) {
      const int i = base + k * nt + threadIdx.x;
      if (i < N) dst[i] = r[k];
    }
  }
}

// Top-R of n unique 64-bit keys held in LDS `in` (n > R): an 11-bit, 3-pass radix select on the
// score half (bits 63..32) finds the R-th largest score T; every key with score >= T (R plus
// ties at T) is gathered into `out` and bitonic-sorted.  Returns how many were gathered
// (>= R; the first R of `out` are the exact top-R).  hist: 2048 u32 of LDS.
__device__ __forceinline__ int block_topk_lds(const unsigned long long *in, int n, int R, unsigned long long *out,
                              int out_cap, uint32_t *hist, int *s_misc /* 4 */) {
  uint32_t prefix = 0, mask = 0;
  int kk = R;
  for (int level = 0; level < 3; ++level) {
    // digits: bits 31..21, 20..10, 9..0 (no runtime-indexed local arrays: they live in scratch)
    const int sh = level == 0 ? 21 : (level == 1 ? 10 : 0), nb = level < 2 ? 2048 : 1024;
    for (int i = threadIdx.x; i < nb; i += blockDim.x) hist[i] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      const uint32_t u = static_cast<uint32_t>(in[i] >> 32);
      if ((u & mask) == prefix) atomicAdd(&hist[(u >> sh) & (nb - 1)], 1u);
    }
    __syncthreads();
    // suffix scan from the top bin: wave 0, 32 bins per lane
    if (threadIdx.x < 64) {
      // each lane owns `per` (<= 32) consecutive bins from the top, held in registers
      const int lane = threadIdx.x, per = nb / 64;
      uint32_t hv[32];
      uint32_t mine = 0;
#pragma unroll
      for (int t = 0; t < 32; ++t) {
        hv[t] = t < per ? hist[nb - 1 - (lane * per + t)] : 0u;
        mine += hv[t];
      }
      uint32_t incl = mine;  // inclusive prefix over lanes (lane 0 = top bins)
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t v = __shfl_up(incl, o, 64);
        if (lane >= o) incl += v;
      }
      const uint32_t excl = incl - mine;
      const bool hit = excl < static_cast<uint32_t>(kk) && incl >= static_cast<uint32_t>(kk);
      if (hit) {
        uint32_t acc = excl;
        int tb = per - 1;
        bool done = false;
#pragma unroll
        for (int t = 0; t < 32; ++t) {
          if (!done && t < per) {
            if (acc + hv[t] >= static_cast<uint32_t>(kk)) {
              tb = t;
              done = true;
            } else {
              acc += hv[t];
            }
          }
        }
        s_misc[0] = nb - 1 - (lane * per + tb);
        s_misc[1] = kk - static_cast<int>(acc);
      }
    }
    __syncthreads();
    const int bin = s_misc[0];
    const int left = s_misc[1];
    prefix |= static_cast<uint32_t>(bin) << sh;
    mask |= static_cast<uint32_t>(nb - 1) << sh;
    // everything at or above this bin fits the output: stop refining, gather and sort it
    const bool enough = (R - left) + static_cast<int>(hist[bin]) <= out_cap;
    kk = left;
    __syncthreads();
    if (enough) break;
  }
  if (threadIdx.x == 0) s_misc[2] = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const unsigned long long k = in[i];
    if ((static_cast<uint32_t>(k >> 32) & mask) >= prefix) {
      const int slot = atomicAdd(&s_misc[2], 1);
      if (slot < out_cap) out[slot] = k;
    }
  }
  __syncthreads();
  const int m = s_misc[2];
  const int N = next_pow2(max(min(m, out_cap), 2));
  for (int i = min(m, out_cap) + threadIdx.x; i < N; i += blockDim.x) out[i] = 0ull;
  __syncthreads();
  bitonic_desc(out, N);
  return m;
}

// Radix select over unique 64-bit keys in global memory: the largest T with
// count(key >= T) >= q (== q exactly since keys are unique).  8 passes of 8 bits.
__device__ unsigned long long radix_select_desc(const unsigned long long *g, int n, int q,
                                                uint32_t *hist /* 256 */, unsigned long long *st) {
  unsigned long long prefix = 0, mask = 0;
  int kk = q;
  for (int level = 0; level < 8; ++level) {
    const int shift = 56 - 8 * level;
    for (int i = threadIdx.x; i < 256; i += blockDim.x) hist[i] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      const unsigned long long k = g[i];
      if ((k & mask) == prefix) atomicAdd(&hist[(k >> shift) & 255ull], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int acc = 0, d = 255;
      for (; d > 0; --d) {
        if (acc + static_cast<int>(hist[d]) >= kk) break;
        acc += hist[d];
      }
      st[0] = prefix | (static_cast<unsigned long long>(d) << shift);
      st[1] = static_cast<unsigned long long>(kk - acc);
    }
    __syncthreads();
    prefix = st[0];
    kk = static_cast<int>(st[1]);
    mask |= 0xffull << shift;
    __syncthreads();
  }
  return prefix;
}

// Block-level greedy NMS over n boxes sorted by descending score (LDS arrays).  Chunks of 64
// candidates: (A) every wave tests the chunk against a slice of the already-kept boxes, (B) the
// 64 x 64 intra-chunk suppression matrix is split by rows over the waves, then (C) wave 0
// resolves the chunk's greedy order with 64 wave-uniform column masks (ballots) — exactly the
// sequential greedy result.  keep[i] = 1 for kept.  Returns the kept count; klist = kept
// positions in order.  Stops at the first chunk boundary with >= stop_after kept.
template <int V>
__device__ int block_greedy(const Box4 *sb, const float *sa, int n, float thr, float beta,
                            uint8_t *keep, int *klist, unsigned long long *s_flag /* 16 */,
                            unsigned long long *s_m /* 16 x 64 */, int *s_nk,
                            int stop_after = 0x7fffffff) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int rpw = 64 / nw;  // chunk rows tested per wave
  if (threadIdx.x == 0) *s_nk = 0;
  __syncthreads();
  for (int s0 = 0; s0 < n; s0 += 64) {
    const int nk = *s_nk;
    if (nk >= stop_after) break;
    const int j = s0 + lane;
    const bool valid = j < n;
    bool sup = false;
    unsigned long long m = 0;
    if (valid) {
      const Box4 bj = sb[j];
      const float aj = sa[j];
      for (int k = wv; k < nk; k += nw) {          // (A)
        const int i = klist[k];
        if (suppresses<V>(sb[i], sa[i], bj, aj, thr, beta)) {
          sup = true;
          break;
        }
      }
      const int i0 = wv * rpw, i1 = min(i0 + rpw, lane);
      for (int i = i0; i < i1; ++i)                  // (B)
        if (suppresses<V>(sb[s0 + i], sa[s0 + i], bj, aj, thr, beta)) m |= 1ull << i;
    }
    const unsigned long long bal = __ballot(sup);
    if (lane == 0) s_flag[wv] = bal;
    s_m[wv * 64 + lane] = m;
    __syncthreads();
    if (wv == 0) {                                   // (C)
      unsigned long long dead = 0, mm = 0;
      for (int w = 0; w < nw; ++w) {
        dead |= s_flag[w];
        mm |= s_m[w * 64 + lane];
      }
      unsigned long long alive = __ballot(valid) & ~dead;
      unsigned long long kept = 0;
      for (int i = 0; i < 64; ++i) {
        const unsigned long long col = __ballot((mm >> i) & 1ull);  // members suppressed by i
        if ((alive >> i) & 1ull) {
          kept |= 1ull << i;
          alive &= ~col;
        }
      }
      const bool kj = (kept >> lane) & 1ull;
      if (valid) keep[j] = kj ? 1 : 0;
      const int before = __popcll(kept & ((1ull << lane) - 1ull));
      if (kj) klist[nk + before] = j;
      if (lane == 0) *s_nk = nk + __popcll(kept);
    }
    __syncthreads();
  }
  return *s_nk;
}

// Greedy NMS for n <= kMatrixMax sorted boxes.  The upper-triangular suppression bit matrix is
// built one 64-bit word per wave step: the row box is an LDS broadcast, the 64 lanes test the
// 64 columns of the word and a ballot assembles it (all waves busy, no per-thread serial loops).
// Then wave 0 sweeps the rows in order — for n <= 64 from registers (row i's word in lane i,
// read with readlane), otherwise with one alive word per lane — exactly the sequential greedy
// result.  keep/klist as block_greedy; stops after stop_after kept.
constexpr int kMatrixMax = 512;

template <int V>
__device__ int block_greedy_matrix(const Box4 *sb, const float *sa, int n, float thr, float beta,
                                   uint8_t *keep, int *klist,
                                   unsigned long long *mat /* n x (kMatrixMax/64) */, int *s_nk,
                                   int stop_after = 0x7fffffff) {
  const int nb = (n + 63) >> 6;
  const int W = nb;   // row stride in words
  const int items = n * nb;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int it = wv; it < items; it += nw) {
    const int i = it / nb, cb = it - i * nb;
    const int j = (cb << 6) + lane;
    bool sup = false;
    if (j > i && j < n) sup = suppresses<V>(sb[i], sa[i], sb[j], sa[j], thr, beta);
    const unsigned long long bits = __ballot(sup);
    if (lane == 0) mat[i * W + cb] = bits;
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    int nk = 0;
    if (nb == 1) {
      const unsigned long long row = lane < n ? mat[lane] : 0ull;
      const uint32_t rlo = static_cast<uint32_t>(row), rhi = static_cast<uint32_t>(row >> 32);
      unsigned long long alive = n == 64 ? ~0ull : ((1ull << n) - 1ull);
      unsigned long long kept = 0;
      for (int i = 0; i < n; ++i) {
        if (!((alive >> i) & 1ull)) continue;
        kept |= 1ull << i;
        if (++nk >= stop_after) break;
        const uint32_t lo = __builtin_amdgcn_readlane(rlo, i);
        const uint32_t hi = __builtin_amdgcn_readlane(rhi, i);
        alive &= ~((static_cast<unsigned long long>(hi) << 32) | lo);
      }
      if (lane < n) {
        const bool k = (kept >> lane) & 1ull;
        keep[lane] = k ? 1 : 0;
        if (k) klist[__popcll(kept & ((1ull << lane) - 1ull))] = lane;
      }
    } else {
      const bool own = lane < nb;
      unsigned long long alive = own ? (lane == nb - 1 && (n & 63) ? ((1ull << (n & 63)) - 1ull) : ~0ull) : 0ull;
      unsigned long long row = own ? mat[lane] : 0ull;  // row 0, prefetched
      for (int i = 0; i < n; ++i) {
        const unsigned long long next = (own && i + 1 < n) ? mat[(i + 1) * W + lane] : 0ull;
        const int wl = i >> 6;
        const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(alive), wl);
        const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(alive >> 32), wl);
        const unsigned long long aw = (static_cast<unsigned long long>(hi) << 32) | lo;
        const bool alive_i = (aw >> (i & 63)) & 1ull;
        if (lane == 0) keep[i] = alive_i ? 1 : 0;
        if (alive_i) {
          if (lane == 0) klist[nk] = i;
          ++nk;
          if (nk >= stop_after) {
            for (int r = i + 1 + lane; r < n; r += 64) keep[r] = 0;
            break;
          }
          alive &= ~row;
        }
        row = next;
      }
    }
    if (lane == 0) *s_nk = nk;
  }
  __syncthreads();
  return *s_nk;
}


// ----------------------------------------------------------------------------- boxes
// The decoded + clamped box of (image b, prior p) (models/utils.py:218-224), recomputed by each
// consumer from the raw locs (and the prior) instead of k_det_prepare writing all B x P of them:
// only the candidates a segment's window holds and the merged outputs are ever read (~40K of
// 328K boxes at SSD512 B=32), so the 5.2 MB box plane and its write are gone, and so is the
// decode's VALU from the grid-wide pass.  Same inputs, same device functions (-ffp-contract=off):
// the same bits as the former materialised plane.  CORNER boxes were clamped in place by
// k_det_prepare (the reference's clamp_), clamping again is the identity.
struct DetBoxes {
  const void *locs;      // [B,P,4] f32, or bf16 bit patterns (bf16 != 0)
  const float *priors;   // [P,4] cxcy (OFFSET); any valid 16-byte buffer otherwise (dummy loads)
  int P, box_type, bf16;
};
// Where a box's latency must run under other work, its loads are issued early (det_box_issue:
// unconditional, into plain registers) and decoded at the use (det_box_finish).
struct RawBox {
  Box4 l, pr;
};


__device__ __forceinline__ RawBox det_box_issue(const DetBoxes &s, int b, uint32_t p) {
  const int64_t i = static_cast<int64_t>(b) * s.P + p;
  RawBox r;
  if (s.bf16) {
    const uint2 v = *reinterpret_cast<const uint2 *>(static_cast<const uint16_t *>(s.locs) + 4 * i);
    r.l = Box4{__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xffff0000u), __uint_as_float(v.y << 16),
               __uint_as_float(v.y & 0xffff0000u)};
  } else {
    r.l = ld4(static_cast<const float *>(s.locs) + 4 * i);
  }
  r.pr = ld4(s.priors + (s.box_type == SBOD_BOX_OFFSET ? 4 * static_cast<int64_t>(p) : 0));
  return r;
}

__device__ __forceinline__ Box4 det_box_finish(const DetBoxes &s, const RawBox &r) {
  Box4 d;
  if (s.box_type == SBOD_BOX_OFFSET) {
    d = decode_tenfive_xy(r.l, r.pr);
  } else if (s.box_type == SBOD_BOX_CENTER) {
    d = Box4{r.l.a - r.l.c / 2.f, r.l.b - r.l.d / 2.f, r.l.a + r.l.c / 2.f, r.l.b + r.l.d / 2.f};
  } else {
    d = r.l;
  }
  return Box4{fminf(fmaxf(d.a, 0.f), 1.f), fminf(fmaxf(d.b, 0.f), 1.f), fminf(fmaxf(d.c, 0.f), 1.f),
              fminf(fmaxf(d.d, 0.f), 1.f)};
}

// (k_det_prepare's CORNER in-place clamp and debug boxes: the same arithmetic as det_box_finish)
__device__ __forceinline__ Box4 det_decode(Box4 l, int box_type, const float *priors, uint32_t p) {
  const RawBox r{l, box_type == SBOD_BOX_OFFSET ? ld4(priors + 4 * static_cast<int64_t>(p)) : l};
  return det_box_finish(DetBoxes{nullptr, nullptr, 0, box_type, 0}, r);
}

__device__ __forceinline__ Box4 det_box(const DetBoxes &s, int b, uint32_t p) {
  return det_box_finish(s, det_box_issue(s, b, p));
}

// ----------------------------------------------------------------------------- K1
struct DetArgs {
  int B, P, C, box_type, act;
  const float *priors;
  const uint8_t *pos;
  float min_score;
  unsigned long long *cand;        // [B,C,P]
  uint32_t *cand_count;            // [B,C]
  float *dbg_probs, *dbg_boxes;
  SpanRing *span;                  // KernelTimer span ring under graph capture, else null
  int rows = kDTile;               // rows (priors) per k_det_prepare tile
};

// exp(x) and the logistic function on the hardware exp2 / rcp units (~1-2 ulp; the detect path's
// activations are its own — parity is pinned on the activations it produces).
__device__ __forceinline__ float fast_exp(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }
__device__ __forceinline__ float fast_sigmoid(float x) { return __builtin_amdgcn_rcpf(1.f + fast_exp(-x)); }

// Candidate slots of one workgroup: the per-(wave, class) ballots in LDS become ONE returning
// atomic per (workgroup, class) on the segment's counter, all classes' atomics in flight
// together; s_wb(w, c) = the slot base of wave w's class-c candidates.  Order inside a segment
// is irrelevant (keys are unique and sorted later).  Synchronises the block.
__device__ __forceinline__ void prep_slots(const DetArgs &a, int b, int C, int tid,
                                           const unsigned long long *s_balf, uint32_t *s_wbf) {
  __syncthreads();
  for (int c = tid + 1; c < C; c += kDTile) {
    uint32_t nwv[kDTile / 64], n = 0;
#pragma unroll
    for (int w = 0; w < kDTile / 64; ++w) {
      nwv[w] = __popcll(s_balf[w * C + c]);
      n += nwv[w];
    }
    uint32_t base = n ? atomicAdd(a.cand_count + b * C + c, n) : 0u;
#pragma unroll
    for (int w = 0; w < kDTile / 64; ++w) {
      s_wbf[w * C + c] = base;
      base += nwv[w];
    }
  }
  __syncthreads();
}

// CM > 0: rows of C <= CM classes live in CM registers (padding slots hold -inf, so the max, the
// exponentials and the sum need no per-slot guards); CM == 0: any C, rows in LDS.  CE > 0: the
// class count is the compile-time CE (VOC's 21), so no slot needs a padding select or a k < C
// test, and only CE exponentials are evaluated.
// Input element types: float, or uint16_t holding bf16 bit patterns (widened exactly on load, so
// every later decision sees the fp32 value of the bf16 activation — the same values the fp32 path
// gets from a widened copy).
__device__ __forceinline__ float widen(float v) { return v; }
__device__ __forceinline__ float widen(uint16_t v) { return __uint_as_float(static_cast<uint32_t>(v) << 16); }
__device__ __forceinline__ Box4 ld_box(const float *p) { return ld4(p); }
__device__ __forceinline__ Box4 ld_box(const uint16_t *p) {
  const uint2 v = *reinterpret_cast<const uint2 *>(p);
  return Box4{__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xffff0000u), __uint_as_float(v.y << 16),
              __uint_as_float(v.y & 0xffff0000u)};
}
__device__ __forceinline__ void st_box(float *p, Box4 b) { st4(p, b); }
__device__ __forceinline__ void st_box(uint16_t *p, Box4 b) {   // values that came from bf16: exact
  *reinterpret_cast<uint2 *>(p) = make_uint2((__float_as_uint(b.a) >> 16) | (__float_as_uint(b.b) & 0xffff0000u),
                                             (__float_as_uint(b.c) >> 16) | (__float_as_uint(b.d) & 0xffff0000u));
}

template <int CM, int CE, typename T = float>
__global__ __launch_bounds__(kDTile) void k_det_prepare(DetArgs a, T *__restrict__ locs,
                                                        const T *__restrict__ scores) {
  static_assert(CM > 0 || sizeof(T) == 4, "k_det_prepare: bf16 input takes the register-row path");
  // dynamic LDS: score tile [kDTile][C] T | ballots [kDTile/64][C] u64 | slot bases [C] u32,
  // sized to C so 6+ workgroups fit per CU (one round for B x ceil(P/256) workgroups at B=32)
  extern __shared__ float s_sc[];
  STAMP_BEGIN();
  span_begin(a.span);
  const int b = blockIdx.y, p0 = blockIdx.x * a.rows, tid = threadIdx.x, lane = tid & 63;
  const int P = a.P, C = CE > 0 ? CE : a.C;
  T *const s_tile = reinterpret_cast<T *>(s_sc);
  unsigned long long *s_balf = reinterpret_cast<unsigned long long *>(s_tile + kDTile * C);
  uint32_t *s_wbf = reinterpret_cast<uint32_t *>(s_balf + (kDTile / 64) * C);   // per-wave slot bases
#define s_bal(w, c) s_balf[(w) * C + (c)]
#define s_wb(w, c) s_wbf[(w) * C + (c)]
  const int np = min(a.rows, P - p0);
  const int64_t rbase = static_cast<int64_t>(b) * P + p0;
#ifdef SBOD_PHASE_CLOCKS
  long long ph[6] = {0, 0, 0, 0, 0, 0};
#endif
  SEG_PHASE(0);
  const bool valid = tid < np;
  const int p = p0 + tid;
  const int64_t i = rbase + tid;
  // the prior's positive-mask byte goes out with the score tile (one memory round trip)
  const int64_t ic = valid ? i : rbase;
  // The prologue load is unconditional and lands in a plain register: a load under a branch
  // (or a select of two loaded values) makes the wait-count insertion at the join wait for it
  // BEFORE the score tile below is even issued — one whole memory round trip on every
  // workgroup's critical path.  Without a positive mask it reads a dummy byte of the score tile
  // this workgroup loads anyway (a dummy read of another plane fetches that plane's lines from
  // HBM: 5.2 MB per launch at SSD512 B=32 when it was the box plane).
  // The boxes are decoded by their consumers (det_box): this pass reads no locs and no priors
  // unless it clamps CORNER boxes in place (models/utils.py:224) or writes the debug boxes.
  const auto *posp = (const __attribute__((address_space(1))) uint8_t *)(
      a.pos != nullptr ? a.pos + ic : reinterpret_cast<const uint8_t *>(scores + rbase * C));
  const uint8_t posraw = *posp;
  constexpr int kPer16 = 16 / static_cast<int>(sizeof(T));   // elements per 16-byte chunk
#if SBOD_PREP_GLDS
  if (CM > 0 && (reinterpret_cast<uintptr_t>(scores + rbase * C) & 15) == 0) {
    // LDS-DMA: each wave-instruction copies 64 x 16 B of the tile straight into LDS (lane-linear,
    // no VGPR round trip, no LDS write instructions); the tail elements go the ordinary way
    const float4 *src4 = reinterpret_cast<const float4 *>(scores + rbase * C);
    const int n = np * C, n4 = n / kPer16, wv0 = tid >> 6;
#pragma unroll
    for (int k = 0; k < (CM > 0 ? (CM + kPer16 - 1) / kPer16 : 1); ++k) {
      const int q0 = k * kDTile + 64 * wv0;   // the wave's first 16-byte chunk (uniform)
      if (q0 + lane < n4)
        __builtin_amdgcn_global_load_lds(src4 + q0 + lane,
                                         (__attribute__((address_space(3))) void *)(reinterpret_cast<float4 *>(s_sc) + q0),
                                         16, 0, 0);
    }
    for (int e = n4 * kPer16 + tid; e < n; e += kDTile) s_tile[e] = scores[rbase * C + e];
  } else if constexpr (sizeof(T) == 4) {
    tile_load_f32<(CM > 0 ? (CM + 3) / 4 : 8)>(s_sc, scores + rbase * C, np * C);
  } else {
    for (int e = tid; e < np * C; e += kDTile) s_tile[e] = scores[rbase * C + e];
  }
#else
  if constexpr (sizeof(T) == 4)
    tile_load_f32<(CM > 0 ? (CM + 3) / 4 : 8)>(s_sc, scores + rbase * C, np * C);
  else
    for (int e = tid; e < np * C; e += kDTile) s_tile[e] = scores[rbase * C + e];
#endif
  drain_vm();   // this wave's LDS-DMA chunks (read by other waves' rows) have landed: s_barrier
                // does not wait for vmcnt on gfx950
  __syncthreads();
  SEG_PHASE(1);
  float *row = s_sc + tid * C;         // (CM == 0 only: fp32 rows)
  const T *rowt = s_tile + tid * C;
  if (valid && (a.box_type == SBOD_BOX_CORNER || a.dbg_boxes != nullptr)) {   // (wave-uniform test)
    const Box4 d = det_decode(ld_box(locs + 4 * i), a.box_type, a.priors, static_cast<uint32_t>(p));
    if (a.box_type == SBOD_BOX_CORNER) st_box(locs + 4 * i, d);  // models/utils.py:224 clamp_ in place
    if (a.dbg_boxes) st4(a.dbg_boxes + 4 * i, d);
  }
  if (valid) {
    if constexpr (CM == 0) {
      if (a.act == SBOD_ACT_SOFTMAX) {
        float m = row[0];
        for (int k = 1; k < C; ++k) m = fmaxf(m, row[k]);
        float s = 0.f;
        for (int k = 0; k < C; ++k) {
          const float e = fast_exp(row[k] - m);
          row[k] = e;
          s += e;
        }
        const float rs = __builtin_amdgcn_rcpf(s);
        for (int k = 0; k < C; ++k) row[k] = row[k] * rs;
      } else {
        for (int k = 0; k < C; ++k) row[k] = fast_sigmoid(row[k]);
      }
    }
  }
  const bool allowed = valid && (a.pos == nullptr || posraw != 0);
  const int wv = tid >> 6;
  const unsigned long long lt = (1ull << lane) - 1ull;
  if constexpr (CM > 0) {
    // ---- narrow rows (VOC: C = 21): the row, its activation and the candidate tests stay in
    // registers.  Activation: exp2 / rcp hardware ops (probabilities within ~1e-6 relative of
    // torch.softmax; every later decision reads these same values, so detect stays exact w.r.t.
    // them).  Each lane then walks only ITS candidate classes (~1-2 of 20) to emit keys.
    // the raw row stays in LDS: an emitted candidate's probability is recomputed from it with
    // the same operations (bit-identical), so the 20 probabilities are never written back
    // constant-offset reads (one address, no per-slot index arithmetic): a short last row reads
    // at most CM - C <= 7 floats past the tile, into the ballot area that follows it in LDS;
    // only the top 8 slots can be padding (the dispatcher picks CM with C > CM - 8)
    // KN: the slots that can hold a class (compile-time when CE > 0)
    constexpr int KN = CE > 0 ? CE : CM;
    typedef float f2 __attribute__((ext_vector_type(2)));
    float r[KN];
#pragma unroll
    for (int k = 0; k < KN; ++k) {
      const float v = widen(rowt[k]);
      r[k] = (CE > 0 || k < CM - 8 || k < C) ? v : -__builtin_inff();
    }
    const bool softmax = a.act == SBOD_ACT_SOFTMAX;
    float m = 0.f, rs = 1.f;
    if (softmax) {
      m = r[0];
#pragma unroll
      for (int k = 1; k < KN; ++k) m = fmaxf(m, r[k]);   // NaN rows give NaN probabilities either way
      // (x - m) * log2(e) two slots per packed op, hardware exp2, pairwise packed sums
      const f2 nm2 = {-m, -m}, l2 = {1.4426950408889634f, 1.4426950408889634f};
#pragma unroll
      for (int k = 0; k + 1 < KN; k += 2) {
        f2 t = {r[k], r[k + 1]};
        t = (t + nm2) * l2;
        r[k] = __builtin_amdgcn_exp2f(t.x);   // padding: exp2(-inf) = 0
        r[k + 1] = __builtin_amdgcn_exp2f(t.y);
      }
      if constexpr (KN % 2 == 1) r[KN - 1] = __builtin_amdgcn_exp2f((r[KN - 1] - m) * 1.4426950408889634f);
      f2 acc2 = {0.f, 0.f};
#pragma unroll
      for (int k = 0; k + 1 < KN; k += 2) acc2 += f2{r[k], r[k + 1]};
      float sum = acc2.x + acc2.y;
      if constexpr (KN % 2 == 1) sum += r[KN - 1];
      rs = __builtin_amdgcn_rcpf(sum);
      const f2 rs2 = {rs, rs};
#pragma unroll
      for (int k = 0; k + 1 < KN; k += 2) {
        const f2 t = f2{r[k], r[k + 1]} * rs2;
        r[k] = t.x;
        r[k + 1] = t.y;
      }
      if constexpr (KN % 2 == 1) r[KN - 1] *= rs;
    } else {
#pragma unroll
      for (int k = 0; k < KN; ++k) r[k] = fast_sigmoid(r[k]);
    }
    if (a.dbg_probs && valid) {
#pragma unroll
      for (int k = 0; k < KN; ++k)
        if (k < C) a.dbg_probs[i * C + k] = r[k];
    }
    // per class: one compare straight into a wave mask (lanes that may not emit compare against
    // +inf), kept in scalar registers; this lane's bit shifted into cmask (class k at bit KN-1-k)
    const float thr = allowed ? a.min_score : __builtin_inff();
    uint32_t cmask = 0;
    unsigned long long bals[KN];
#pragma unroll
    for (int k = 1; k < KN; ++k) {
      if (k < C) {
        const bool take = r[k] > thr;
        bals[k] = __builtin_amdgcn_ballot_w64(take);
        cmask = cmask + cmask + (take ? 1u : 0u);
      } else {
        bals[k] = 0ull;
        cmask = cmask + cmask;
      }
    }
    if (lane == 0) {   // one exec switch for all the wave's masks
#pragma unroll
      for (int k = 1; k < KN; ++k)
        if (k < C) s_bal(wv, k) = bals[k];
    }
    SEG_PHASE(2);
    prep_slots(a, b, C, tid, s_balf, s_wbf);
    SEG_PHASE(3);
    // Emission, one class at a time in a uniform loop: the wave's mask for the class is in
    // scalar registers (bals), its slot base one LDS word made scalar, and the emitting lanes'
    // probability is r[k] itself (computed once above, still in registers) — no divergent
    // per-lane loop over candidate classes and no LDS row re-read per candidate (phase clocks:
    // this phase was ~6K of ~16K cycles per workgroup in the per-lane form).
    // (plain stores: these 8-byte scattered writes must merge into full lines in L2 first —
    // streamed through they cost 1.7x the kernel time)
    // every class's slot base read from LDS up front (one wait, not one LDS round trip per
    // class); a lane's rank among the wave's takers is v_mbcnt of the scalar mask; whether the
    // lane takes class k is bit KN-1-k of cmask (no 64-bit mask test per class)
    unsigned long long *cb = a.cand + static_cast<int64_t>(b) * C * P;
    uint32_t wb[KN];
#pragma unroll
    for (int k = 1; k < KN; ++k) wb[k] = k < C ? s_wb(wv, k) : 0u;
    const uint32_t klow = 0xffffffffu - static_cast<uint32_t>(p);
#pragma unroll
    for (int k = 1; k < KN; ++k) {
      if (k < C && bals[k] != 0ull) {
        const uint32_t base = __builtin_amdgcn_readfirstlane(wb[k]);
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(bals[k] >> 32),
                                                        __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(bals[k]), 0u));
        const uint32_t slot = base + rank;
        // slot < P always with counters zero on entry (memory-safe otherwise)
        if (((cmask >> (KN - 1 - k)) & 1u) && slot < static_cast<uint32_t>(P))
          cb[static_cast<int64_t>(k) * P + slot] = (static_cast<unsigned long long>(f2ord(r[k])) << 32) | klow;
      }
    }
    (void)lt;
  } else {
    SEG_PHASE(2);
    for (int c = 1; c < C; ++c) {
      const bool take = allowed && row[c] > a.min_score;
      const unsigned long long bal = __ballot(take);
      if (lane == 0) s_bal(wv, c) = bal;
    }
    prep_slots(a, b, C, tid, s_balf, s_wbf);
    SEG_PHASE(3);
    for (int c = 1; c < C; ++c) {
      const unsigned long long bal = s_bal(wv, c);
      if (!((bal >> lane) & 1ull)) continue;
      const uint32_t slot = s_wb(wv, c) + __popcll(bal & lt);
      if (slot < static_cast<uint32_t>(P))
        a.cand[(static_cast<int64_t>(b) * C + c) * P + slot] = make_key(row[c], static_cast<uint32_t>(p));
    }
  }
  SEG_PHASE(4);
#ifdef SBOD_PHASE_CLOCKS
  if (threadIdx.x == 0 && (blockIdx.x == 0 || blockIdx.x == 20) && (blockIdx.y == 0 || blockIdx.y == 5))
    printf("prep x%d b%d: tile %lld compute %lld ballot+atomic %lld keys %lld total %lld\n", blockIdx.x, b,
           ph[1] - ph[0], ph[2] - ph[1], ph[3] - ph[2], ph[4] - ph[3], ph[4] - ph[0]);
#endif
  if constexpr (CM == 0) {
    if (a.dbg_probs) {
      __syncthreads();
      for (int k = tid; k < np * C; k += kDTile) a.dbg_probs[rbase * C + k] = s_sc[k];
    }
  }
  span_end(a.span);
  STAMP_END(1, 1);
}
#undef s_bal
#undef s_wb

// ----------------------------------------------------------------------------- K2
struct SegOut {
  unsigned long long *kept;   // [B,C,W] kept candidate keys in rank order
  uint32_t *kc;               // [B,C] kept count within the window
  unsigned long long *lastkey;// [B,C] the window's last candidate key when truncated, else 0
};

constexpr int kSegSortCap = 2048;  // segments up to this size are selected in LDS
// A candidate key's prior index is dereferenced (its decoded box) only when < P: a corrupted or
// stale candidate region (a caller's workspace contract broken) must never read out of bounds.
// The segment then reports kKcCorrupt as its kept count, and the image's merge reports
// det_count SBOD_DETECT_CORRUPT (-2) instead of detections.
constexpr uint32_t kKcCorrupt = 0xffffffffu;
constexpr int32_t kDetCorrupt = SBOD_DETECT_CORRUPT;
__device__ __forceinline__ uint32_t key_prior(unsigned long long k, int P, bool &bad) {
  const uint32_t p = key_low(k);
  bad = p >= static_cast<uint32_t>(P);
  return bad ? 0u : p;
}


// Block-level segment work for (image b, class c): top-`window` candidates by key, greedy NMS,
// kept keys in rank order.  Called by every thread of the block (it synchronises); used by
// k_det_segment (one block per segment) and by k_det_merge's inline second pass.
__device__ void segment_body(const unsigned long long *cand, const uint32_t *cand_count,
                             const DetBoxes boxes_ws, int P, int C, int b, int c, int window,
                             int stride, float thr, SegOut o, unsigned char *s_raw, uint32_t *s_hist,
                             unsigned long long *s_st, unsigned long long *s_flag, unsigned long long *s_m,
                             int *s_nk_p, int *s_cnt_p, int *s_misc) {
  int &s_nk = *s_nk_p;
  int &s_cnt = *s_cnt_p;
  const int64_t seg = static_cast<int64_t>(b) * C + c;
  const int n = min(static_cast<int>(cand_count[seg]), P);   // counters never exceed P
  const unsigned long long *g = cand + seg * P;
  const int q = min(n, window);
  // LDS: raw keys [kSegSortCap] | window keys [pow2(window)] | boxes, areas, klist, keep, matrix
  unsigned long long *raw = reinterpret_cast<unsigned long long *>(s_raw);
  const int WN = next_pow2(max(window, 2));
  unsigned long long *sk = raw + kSegSortCap;
  Box4 *sb = reinterpret_cast<Box4 *>(sk + WN);
  float *sa = reinterpret_cast<float *>(sb + window);
  int *kl = reinterpret_cast<int *>(sa + window);
  uint8_t *kf = reinterpret_cast<uint8_t *>(kl + window);
  unsigned long long *mat = reinterpret_cast<unsigned long long *>(
      reinterpret_cast<uintptr_t>(kf + window + 15) & ~static_cast<uintptr_t>(15));
  if (n == 0) {
    if (threadIdx.x == 0) {
      o.kc[seg] = 0;
      o.lastkey[seg] = 0;
    }
    __syncthreads();
    return;
  }
  if (n <= q) {  // whole segment fits the window
    const int N = next_pow2(max(n, 2));
    block_copy_keys(sk, g, n, N);
    __syncthreads();
    bitonic_desc(sk, N);
  } else if (n <= kSegSortCap) {
    block_copy_keys(raw, g, n, n);
    __syncthreads();
    const int m = block_topk_lds(raw, n, q, sk, WN, s_hist, s_misc);
    if (m > WN) {  // pathological ties at the threshold: sort the whole segment instead
      const int N = next_pow2(n);
      block_copy_keys(raw, g, n, N);
      __syncthreads();
      bitonic_desc(raw, N);
      for (int i = threadIdx.x; i < q; i += blockDim.x) sk[i] = raw[i];
      __syncthreads();
    }
  } else {
    const unsigned long long T = radix_select_desc(g, n, q, s_hist, s_st);
    const int N = next_pow2(max(q, 2));
    if (threadIdx.x == 0) s_cnt = 0;
    for (int i = threadIdx.x; i < N; i += blockDim.x) sk[i] = 0ull;
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      const unsigned long long k = g[i];
      if (k >= T) sk[atomicAdd(&s_cnt, 1)] = k;
    }
    __syncthreads();
    bitonic_desc(sk, N);
  }
  int bad_any = 0;
  for (int i = threadIdx.x; i < q; i += blockDim.x) {
    bool bad;
    const uint32_t p = key_prior(sk[i], P, bad);
    bad_any |= bad;
    const Box4 bx = det_box(boxes_ws, b, p);
    sb[i] = bx;
    sa[i] = (bx.c - bx.a) * (bx.d - bx.b);
  }
  if (__syncthreads_or(bad_any)) {
    if (threadIdx.x == 0) {
      o.kc[seg] = kKcCorrupt;
      o.lastkey[seg] = 0;
    }
    __syncthreads();
    return;
  }
  const int nk = q <= kMatrixMax
                     ? block_greedy_matrix<SBOD_NMS_TV>(sb, sa, q, thr, 1.f, kf, kl, mat, &s_nk)
                     : block_greedy<SBOD_NMS_TV>(sb, sa, q, thr, 1.f, kf, kl, s_flag, s_m, &s_nk);
  unsigned long long *ko = o.kept + seg * stride;
  for (int k = threadIdx.x; k < nk; k += blockDim.x) ko[k] = sk[kl[k]];
  if (threadIdx.x == 0) {
    o.kc[seg] = nk;
    o.lastkey[seg] = n > q ? sk[q - 1] : 0ull;
  }
  __syncthreads();   // LDS is reused by the caller right after
}

__global__ __launch_bounds__(kSegThreads) void k_det_segment(
    const unsigned long long *__restrict__ cand, const uint32_t *__restrict__ cand_count,
    const DetBoxes boxes_ws, int P, int C, int window, int stride, float thr, SegOut o,
    const int32_t *__restrict__ need) {
  extern __shared__ __attribute__((aligned(16))) unsigned char s_raw[];
  __shared__ uint32_t s_hist[2048];
  __shared__ unsigned long long s_st[2];
  __shared__ unsigned long long s_flag[16];
  __shared__ unsigned long long s_m[kSegThreads];
  __shared__ int s_nk, s_cnt, s_misc[4];
  const int c = blockIdx.x + 1, b = blockIdx.y;
  // second pass: only the truncated classes of images whose merge could not decide
  if (need != nullptr && (need[b] == 0 || o.lastkey[static_cast<int64_t>(b) * C + c] == 0ull)) return;
  segment_body(cand, cand_count, boxes_ws, P, C, b, c, window, stride, thr, o, s_raw, s_hist, s_st, s_flag,
               s_m, &s_nk, &s_cnt, s_misc);
}

// ----------------------------------------------------------------------------- K2 (exhaustive)
// Segments no bounded window can decide (a class with more candidates than the largest window
// whose survivors might still reach the image's top_k, e.g. thousands of near-duplicates): the
// class's candidates are consumed in descending key order, kAllChunk at a time — each chunk is
// the radix-selected top of the keys below the previous chunk's last key, straight from global
// memory — every chunk candidate is first tested against all boxes kept so far, then the
// chunk's survivors are resolved by block_greedy.  This is exactly the sequential greedy NMS of
// the reference (models/utils.py:265, torchvision semantics) for any candidate count; it stops
// once top_k boxes are kept, because a class's boxes beyond its own top_k can never rank in the
// image's top_k.  kept[seg] holds the kept keys in rank order, lastkey[seg] = 0 (decided).
constexpr int kAllChunk = 1024;
constexpr int kAllThreads = 1024;

// q-th largest of the unique keys below `upper` in global memory (8-bit digits from the top).
__device__ unsigned long long radix_select_below(const unsigned long long *g, int n, int q,
                                                 unsigned long long upper, uint32_t *hist,
                                                 unsigned long long *st) {
  unsigned long long prefix = 0, mask = 0;
  int kk = q;
  for (int level = 0; level < 8; ++level) {
    const int shift = 56 - 8 * level;
    for (int i = threadIdx.x; i < 256; i += blockDim.x) hist[i] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      const unsigned long long k = g[i];
      if (k < upper && (k & mask) == prefix) atomicAdd(&hist[(k >> shift) & 255ull], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int acc = 0, d = 255;
      for (; d > 0; --d) {
        if (acc + static_cast<int>(hist[d]) >= kk) break;
        acc += hist[d];
      }
      st[0] = prefix | (static_cast<unsigned long long>(d) << shift);
      st[1] = static_cast<unsigned long long>(kk - acc);
    }
    __syncthreads();
    prefix = st[0];
    kk = static_cast<int>(st[1]);
    mask |= 0xffull << shift;
    __syncthreads();
  }
  return prefix;
}

__global__ __launch_bounds__(kAllThreads) void k_det_segment_all(
    const unsigned long long *__restrict__ cand, const uint32_t *__restrict__ cand_count,
    const DetBoxes boxes_ws, int P, int C, int stride, int top_k, float thr, SegOut o) {
  extern __shared__ __attribute__((aligned(16))) unsigned char s_raw[];   // kept so far: keys [stride] | boxes [stride] | areas [stride]
  __shared__ unsigned long long s_key[kAllChunk];
  __shared__ Box4 s_box[kAllChunk];
  __shared__ float s_area[kAllChunk];
  __shared__ unsigned long long c_key[kAllChunk];   // the chunk's survivors of the kept boxes
  __shared__ Box4 c_box[kAllChunk];
  __shared__ float c_area[kAllChunk];
  __shared__ uint8_t s_keep[kAllChunk];
  __shared__ int s_kl[kAllChunk];
  __shared__ uint32_t s_hist[256];
  __shared__ unsigned long long s_st[2];
  __shared__ unsigned long long s_flag[16];
  __shared__ unsigned long long s_m[kAllThreads];
  __shared__ int s_wsum[kAllThreads / 64];
  __shared__ int s_nk, s_cnt;
  unsigned long long *kkey = reinterpret_cast<unsigned long long *>(s_raw);
  Box4 *kbox = reinterpret_cast<Box4 *>(kkey + stride);
  float *karea = reinterpret_cast<float *>(kbox + stride);
  const int c = blockIdx.x + 1, b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t seg = static_cast<int64_t>(b) * C + c;
  const int n = min(static_cast<int>(cand_count[seg]), P);
  const unsigned long long *g = cand + seg * P;
  int kept = 0, remaining = n;
  unsigned long long upper = ~0ull;
  while (remaining > 0 && kept < top_k) {
    const int q = min(kAllChunk, remaining);
    const unsigned long long T = q == remaining ? 0ull : radix_select_below(g, n, q, upper, s_hist, s_st);
    if (tid == 0) s_cnt = 0;
    for (int i = tid; i < kAllChunk; i += blockDim.x) s_key[i] = 0ull;
    __syncthreads();
    for (int i = tid; i < n; i += blockDim.x) {
      const unsigned long long k = g[i];
      if (k >= T && k < upper) s_key[atomicAdd(&s_cnt, 1)] = k;   // exactly q (keys are unique)
    }
    __syncthreads();
    bitonic_desc(s_key, kAllChunk);
    // load the chunk's boxes; test each against every box kept so far
    bool alive = false, bad = false;
    if (tid < q) {
      const uint32_t p = key_prior(s_key[tid], P, bad);
      const Box4 bx = det_box(boxes_ws, b, p);
      const float ar = (bx.c - bx.a) * (bx.d - bx.b);
      alive = true;
      for (int i = 0; i < kept && alive; ++i)
        if (suppresses<SBOD_NMS_TV>(kbox[i], karea[i], bx, ar, thr, 1.f)) alive = false;
      s_box[tid] = bx;
      s_area[tid] = ar;
    }
    if (__syncthreads_or(bad)) {
      if (tid == 0) {
        o.kc[seg] = kKcCorrupt;
        o.lastkey[seg] = 0ull;
      }
      return;
    }
    // order-preserving compaction of the survivors
    const unsigned long long bal = __ballot(alive);
    if (lane == 0) s_wsum[wv] = __popcll(bal);
    __syncthreads();
    int base = 0, m = 0;
    for (int w = 0; w < static_cast<int>(blockDim.x >> 6); ++w) {
      base += w < wv ? s_wsum[w] : 0;
      m += s_wsum[w];
    }
    if (alive) {
      const int at = base + __popcll(bal & ((1ull << lane) - 1ull));
      c_key[at] = s_key[tid];
      c_box[at] = s_box[tid];
      c_area[at] = s_area[tid];
    }
    __syncthreads();
    const int nk = m > 0 ? block_greedy<SBOD_NMS_TV>(c_box, c_area, m, thr, 1.f, s_keep, s_kl, s_flag, s_m,
                                                     &s_nk, top_k - kept)
                         : 0;
    const int take = min(nk, top_k - kept);
    for (int k = tid; k < take; k += blockDim.x) {
      const int j = s_kl[k];
      kkey[kept + k] = c_key[j];
      kbox[kept + k] = c_box[j];
      karea[kept + k] = c_area[j];
    }
    kept += take;
    remaining -= q;
    upper = s_key[q - 1];
    __syncthreads();
  }
  unsigned long long *ko = o.kept + seg * stride;
  for (int k = tid; k < kept; k += blockDim.x) ko[k] = kkey[k];
  if (tid == 0) {
    o.kc[seg] = kept;
    o.lastkey[seg] = 0ull;
  }
}

// ----------------------------------------------------------------------------- K2 (wave form)
// Pass-1 segments (window <= 64): one wave per (image, class) segment, nothing block-wide.
//   select: radix select of the q-th largest 64-bit key, 8-bit digits from the top, with a
//           per-wave LDS histogram; stops at the first digit whose bin holds exactly the keys
//           still needed.  Keys live in registers for n <= kWaveRegKeys, else are streamed.
//   sort:   the q selected keys, one per lane, bitonic over lanes (shuffles).
//   NMS:    greedy in rank order; a kept box broadcasts itself (readlane) and one ballot gives
//           its suppression row, so rows are built only for boxes that survive.
// Results are identical to k_det_segment (same keys, same rank order, same suppression test).
constexpr int kWaveRegKeys = 2048;

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float readlane_f(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

__global__ __launch_bounds__(64) void k_det_segment_wave(
    const unsigned long long *__restrict__ cand, const uint32_t *__restrict__ cand_count,
    const DetBoxes boxes_ws, int P, int C, int window, int stride, float thr, SegOut o,
    const int32_t *__restrict__ need) {
  __shared__ uint32_t s_hist[256];
  __shared__ unsigned long long s_sel[64];
  __shared__ Box4 s_box[64];
  const int lane = threadIdx.x;
  const int c = blockIdx.x + 1, b = blockIdx.y;
  const int64_t seg = static_cast<int64_t>(b) * C + c;
  if (need != nullptr && (need[b] == 0 || o.lastkey[seg] == 0ull)) return;
  const int n = min(static_cast<int>(cand_count[seg]), P);   // counters never exceed P
  if (n == 0) {
    if (lane == 0) {
      o.kc[seg] = 0;
      o.lastkey[seg] = 0;
    }
    return;
  }
  const unsigned long long *g = cand + seg * P;
  const int q = min(n, window);
  const bool regs = n <= kWaveRegKeys;
#ifdef SBOD_PHASE_CLOCKS
  long long ph[6] = {0, 0, 0, 0, 0, 0};
#endif
  SEG_PHASE(0);
  unsigned long long kr[kWaveRegKeys / 64];
  if (regs) {
#pragma unroll
    for (int t = 0; t < kWaveRegKeys / 64; ++t) {
      const int i = lane + 64 * t;
      const unsigned long long v = g[min(i, n - 1)];
      kr[t] = i < n ? v : 0ull;   // real keys are never 0 (score > 0)
    }
  }
  SEG_PHASE(1);
  // ---- select: keys with (key >> sh) >= (prefix >> sh) are exactly the top q
  unsigned long long prefix = 0;
  int sh = 64;
  if (n > q) {
    int kk = q;
    for (int level = 0; level < 8; ++level) {
      const int dsh = 56 - 8 * level;
#pragma unroll
      for (int j = 0; j < 4; ++j) s_hist[lane + 64 * j] = 0u;
      wave_lds_sync();
      auto count = [&](unsigned long long k) {
        if (k != 0ull && (level == 0 || ((k ^ prefix) >> (dsh + 8)) == 0ull))
          atomicAdd(&s_hist[(k >> dsh) & 255ull], 1u);
      };
      if (regs) {
#pragma unroll
        for (int t = 0; t < kWaveRegKeys / 64; ++t)
          if (64 * t < n) count(kr[t]);      // uniform guard: the remaining slots are padding
      } else {
        for (int i = lane; i < n; i += 64) count(g[i]);
      }
      wave_lds_sync();
      // lane owns bins 255 - 4 lane - (0..3), top first
      uint32_t hv[4], mine = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        hv[j] = s_hist[255 - 4 * lane - j];
        mine += hv[j];
      }
      uint32_t incl = mine;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t v = __shfl_up(incl, off, 64);
        if (lane >= off) incl += v;
      }
      const uint32_t excl = incl - mine;
      const bool hit = excl < static_cast<uint32_t>(kk) && incl >= static_cast<uint32_t>(kk);
      int bin = 0, left = 0, hb = 0;
      if (hit) {
        uint32_t acc = excl;
        bool done = false;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (!done) {
            if (acc + hv[j] >= static_cast<uint32_t>(kk)) {
              bin = 255 - 4 * lane - j;
              left = kk - static_cast<int>(acc);
              hb = static_cast<int>(hv[j]);
              done = true;
            } else {
              acc += hv[j];
            }
          }
        }
      }
      const unsigned long long hm = __ballot(hit);
      const int hl = __ffsll(static_cast<long long>(hm)) - 1;
      bin = __builtin_amdgcn_readlane(bin, hl);
      left = __builtin_amdgcn_readlane(left, hl);
      hb = __builtin_amdgcn_readlane(hb, hl);
      prefix |= static_cast<unsigned long long>(bin) << dsh;
      sh = dsh;
      kk = left;
      if (hb == left) break;   // the whole bin is selected: no finer digit needed
      wave_lds_sync();
    }
  }
  // ---- compact the selected keys (exactly q) into s_sel
  {
    int base = 0;
    auto take = [&](unsigned long long k) {
      const bool sel = k != 0ull && (sh >= 64 || (k >> sh) >= (prefix >> sh));
      const unsigned long long bal = __ballot(sel);
      if (sel) s_sel[base + __popcll(bal & ((1ull << lane) - 1ull))] = k;
      base += __popcll(bal);
    };
    if (regs) {
#pragma unroll
      for (int t = 0; t < kWaveRegKeys / 64; ++t)
        if (64 * t < n) take(kr[t]);
    } else {
      for (int i0 = 0; i0 < n; i0 += 64) take(lane + i0 < n ? g[lane + i0] : 0ull);
    }
  }
  wave_lds_sync();
  SEG_PHASE(2);
  // ---- sort descending over lanes; the selected boxes are fetched BEFORE the sort (their
  // latency overlaps it) and each key carries its original lane to find its box afterwards
  unsigned long long v = lane < q ? s_sel[lane] : 0ull;
  bool bad = false;
  uint32_t pr0 = 0;
  if (lane < q) pr0 = key_prior(v, P, bad);
  const RawBox rb = det_box_issue(boxes_ws, b, pr0);   // unconditional (idle lanes: prior 0)
  const bool corrupt = __ballot(bad) != 0ull;
  int pos = lane;
#pragma unroll
  for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      const unsigned long long w = shfl_xor_u64(v, j);
      const int wp = __shfl_xor(pos, j, 64);
      const bool keep_max = ((lane & j) == 0) == ((lane & k) == 0);
      const bool take = keep_max ? (w > v) : (w < v);   // keys are unique (padding 0 never moves past a key)
      v = take ? w : v;
      pos = take ? wp : pos;
    }
  }
  s_box[lane] = det_box_finish(boxes_ws, rb);
  wave_lds_sync();
  SEG_PHASE(3);
  // ---- greedy NMS over the q ranked boxes (torchvision suppression rule)
  Box4 bx{0.f, 0.f, 0.f, 0.f};
  float ar = 0.f;
  if (lane < q) {
    bx = s_box[pos];
    ar = (bx.c - bx.a) * (bx.d - bx.b);
  }
  unsigned long long alive = q == 64 ? ~0ull : ((1ull << q) - 1ull);
  unsigned long long kept = 0;
  // suppression rows do not depend on the greedy state: 8 rows are built as independent
  // chains (instruction-level parallelism for a lone wave), then applied in rank order
  constexpr int kRowBatch = 8;
  for (int i0 = 0; i0 < q; i0 += kRowBatch) {
    if (!(alive >> i0)) break;                 // nothing left alive at or after i0
    unsigned long long rows[kRowBatch];
#pragma unroll
    for (int u = 0; u < kRowBatch; ++u) {
      const int i = min(i0 + u, 63);
      const Box4 bi{readlane_f(bx.a, i), readlane_f(bx.b, i), readlane_f(bx.c, i), readlane_f(bx.d, i)};
      const float ai = readlane_f(ar, i);
      const bool act = lane > i && lane < q;
      bool amb;
      float inter, un;
      const bool sup = tv_fast(bi, ai, bx, ar, thr, amb, inter, un);
      rows[u] = __ballot(act && sup);
      const unsigned long long am = __ballot(act && amb);
      if (am != 0ull) {   // rare: exact division for the lanes within the margin
        const bool ex = act && amb && (inter / un > thr);
        rows[u] = (rows[u] & ~am) | __ballot(ex);
      }
    }
#pragma unroll
    for (int u = 0; u < kRowBatch; ++u) {
      const int i = i0 + u;
      if (i < q && ((alive >> i) & 1ull)) {
        kept |= 1ull << i;
        alive &= ~rows[u];
      }
    }
  }
  unsigned long long *ko = o.kept + seg * stride;
  if ((kept >> lane) & 1ull) ko[__popcll(kept & ((1ull << lane) - 1ull))] = v;
  const uint32_t llo = __builtin_amdgcn_readlane(static_cast<uint32_t>(v), q - 1);
  const uint32_t lhi = __builtin_amdgcn_readlane(static_cast<uint32_t>(v >> 32), q - 1);
  if (lane == 0) {
    o.kc[seg] = corrupt ? kKcCorrupt : static_cast<uint32_t>(__popcll(kept));
    o.lastkey[seg] = n > q && !corrupt ? ((static_cast<unsigned long long>(lhi) << 32) | llo) : 0ull;
  }
  SEG_PHASE(4);
#ifdef SBOD_PHASE_CLOCKS
  if (lane == 0 && (c == 1 || c == 8) && (b == 0 || b == 5))
    printf("segw b%d c%d n=%d: load %lld select+compact %lld sort+boxes %lld nms+store %lld total %lld\n", b, c, n,
           ph[1] - ph[0], ph[2] - ph[1], ph[3] - ph[2], ph[4] - ph[3], ph[4] - ph[0]);
#endif
}

// ----------------------------------------------------------------------------- K2 (4-wave form)
// Pass-1 segments (window <= 64) on one 256-thread workgroup each: the same select / sort /
// greedy as k_det_segment_wave, with the per-lane work split over four waves —
//   select: ~n/256 keys per lane (registers), one shared 256-bin LDS histogram per 8-bit digit,
//           the digit scan by wave 0;
//   sort:   wave 0 bitonic-sorts the q <= 64 selected keys over its lanes (shuffles);
//   NMS:    the q x q suppression bit matrix is built with every wave taking q/4 rows (the row
//           box is an LDS broadcast, a ballot assembles each row), then wave 0 sweeps the rows
//           in rank order from registers (row i in lane i, readlane).
// Same keys, same rank order, same suppression test: results identical to k_det_segment_wave.
constexpr int kSegWRegKeys = 2048;             // keys held in registers (2048 / (64 W) per lane)

// The segment work of one (image, class) on W waves (the kernel's whole workgroup), shared by
// k_det_segment_w4 (W = 4) and the fused k_det_nms (W = 8).  kWT: the outputs (kept keys, kc,
// lastkey) are written through (sc1) for an in-launch reader.  Waves 1..W-1 return before the
// sweep (no barrier follows it).
template <int W, bool kWT>
__device__ __forceinline__ void segment_w(
    const unsigned long long *__restrict__ cand, const uint32_t *__restrict__ cand_count,
    const DetBoxes boxes_ws, int P, int C, int window, int stride, float thr, SegOut o) {
  constexpr int kSegW = W;
  constexpr int NT = 64 * kSegW, KR = kSegWRegKeys / NT;
  STAMP_BEGIN();
  __shared__ uint32_t s_hist[256];
  __shared__ unsigned long long s_sel[64];
  __shared__ Box4 s_bxu[64], s_bx[64];
  __shared__ float s_ar[64];
  __shared__ unsigned long long s_rows[64];
  __shared__ int s_misc[4];
  __shared__ unsigned long long s_red[2 * kSegW];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int c = blockIdx.x + 1, b = blockIdx.y;
  const int64_t seg = static_cast<int64_t>(b) * C + c;
  const int n = min(static_cast<int>(cand_count[seg]), P);   // counters never exceed P
  if (n == 0) {
    if (tid == 0) {
      if constexpr (kWT) {
        st_wt_u32(reinterpret_cast<int32_t *>(o.kc) + seg, 0u);
        st_wt_u64(o.lastkey + seg, 0ull);
      } else {
        o.kc[seg] = 0;
        o.lastkey[seg] = 0;
      }
    }
    return;
  }
  const unsigned long long *g = cand + seg * P;
  const int q = min(n, window);
#ifdef SBOD_PHASE_CLOCKS
  long long ph[6] = {0, 0, 0, 0, 0, 0};
#endif
  SEG_PHASE(0);
  const bool regs = n <= kSegWRegKeys;
  unsigned long long kr[KR];
  if (regs) {
#pragma unroll
    for (int t = 0; t < KR; ++t) {
      const int i = tid + NT * t;
      const unsigned long long v = g[min(i, n - 1)];
      kr[t] = i < n ? v : 0ull;   // real keys are never 0 (score > 0)
    }
  }
  // ---- common high bits of all keys (OR vs AND): the radix digits start at the highest bit
  // where keys differ (scores in (0.01, 1] share their top ~6 bits, so a fixed top digit wastes
  // a level and piles every key onto a few contended histogram bins)
  unsigned long long vor = 0ull, vand = ~0ull;
  if (regs) {
#pragma unroll
    for (int t = 0; t < KR; ++t)
      if (kr[t] != 0ull) {
        vor |= kr[t];
        vand &= kr[t];
      }
  } else {
    for (int i = tid; i < n; i += NT) {
      const unsigned long long k = g[i];
      vor |= k;
      vand &= k;
    }
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    vor |= shfl_xor_u64(vor, m);
    vand &= shfl_xor_u64(vand, m);
  }
  if (lane == 0) {
    s_red[wv] = vor;
    s_red[kSegW + wv] = vand;
  }
  if (tid == 0) s_misc[3] = 0;
  __syncthreads();
  SEG_PHASE(1);
  // ---- select: keys with (key >> sh) >= (prefix >> sh) are exactly the top q
  unsigned long long prefix = 0;
  int sh = 64;
  if (n > q) {
    unsigned long long all_or = 0ull, all_and = ~0ull;
#pragma unroll
    for (int w = 0; w < kSegW; ++w) {
      all_or |= s_red[w];
      all_and &= s_red[kSegW + w];
    }
    const int top = 63 - __clzll(static_cast<long long>(all_or ^ all_and));   // keys unique, n > 1
    prefix = top >= 63 ? 0ull : (all_and & ~((2ull << top) - 1ull));          // the shared bits
    int kk = q;
    for (int hb = top; hb >= 0;) {
      const int lo = hb >= 7 ? hb - 7 : 0, width = hb - lo + 1;
      const unsigned long long dmask = (1ull << width) - 1ull;
      if (tid < 256) s_hist[tid] = 0u;
      __syncthreads();
      auto count = [&](unsigned long long k) {
        if (k != 0ull && (hb >= 63 || ((k ^ prefix) >> (hb + 1)) == 0ull))
          atomicAdd(&s_hist[(k >> lo) & dmask], 1u);
      };
      if (regs) {
#pragma unroll
        for (int t = 0; t < KR; ++t)
          if (NT * t < n) count(kr[t]);
      } else {
        for (int i = tid; i < n; i += NT) count(g[i]);
      }
      __syncthreads();
      if (wv == 0) {
        // lane owns bins 255 - 4 lane - (0..3), top first (bins >= 2^width stay 0)
        uint32_t hv[4], mine = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          hv[j] = s_hist[255 - 4 * lane - j];
          mine += hv[j];
        }
        uint32_t incl = mine;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
          const uint32_t v = __shfl_up(incl, off, 64);
          if (lane >= off) incl += v;
        }
        const uint32_t excl = incl - mine;
        if (excl < static_cast<uint32_t>(kk) && incl >= static_cast<uint32_t>(kk)) {
          uint32_t acc = excl;
          bool done = false;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (!done) {
              if (acc + hv[j] >= static_cast<uint32_t>(kk)) {
                s_misc[0] = 255 - 4 * lane - j;
                s_misc[1] = kk - static_cast<int>(acc);
                s_misc[2] = static_cast<int>(hv[j]);
                done = true;
              } else {
                acc += hv[j];
              }
            }
          }
        }
      }
      __syncthreads();
      const int bin = s_misc[0], left = s_misc[1], hbin = s_misc[2];
      prefix |= static_cast<unsigned long long>(bin) << lo;
      sh = lo;
      kk = left;
      if (hbin == left) break;   // the whole bin is selected: no finer digit needed
      hb = lo - 1;
    }
  }
  // ---- compact the selected keys (exactly q) into s_sel (any order: sorted next)
  {
    auto take = [&](unsigned long long k) {
      const bool sel = k != 0ull && (sh >= 64 || (k >> sh) >= (prefix >> sh));
      const unsigned long long bal = __ballot(sel);
      if (bal == 0ull) return;
      int base = 0;
      if (lane == 0) base = atomicAdd(&s_misc[3], __popcll(bal));
      base = __shfl(base, 0, 64);
      if (sel) s_sel[base + __popcll(bal & ((1ull << lane) - 1ull))] = k;
    };
    if (regs) {
#pragma unroll
      for (int t = 0; t < KR; ++t)
        if (NT * t < n) take(kr[t]);
    } else {
      for (int i0 = 0; i0 < n; i0 += NT) take(tid + i0 < n ? g[tid + i0] : 0ull);
    }
  }
  __syncthreads();
  SEG_PHASE(2);
  // ---- wave 0: sort descending over lanes; boxes fetched before the sort (latency overlap),
  // each key carries its original lane to find its box afterwards
  unsigned long long v = 0ull;
  bool corrupt = false;
  if (wv == 0) {
    v = lane < q ? s_sel[lane] : 0ull;
    bool bad = false;
    uint32_t p = 0;
    if (lane < q) p = key_prior(v, P, bad);
    // the box's loads issued now (unconditional: an idle lane reads prior 0), decoded after the
    // sort, so their latency runs under it
    const RawBox rb = det_box_issue(boxes_ws, b, p);
    corrupt = __ballot(bad) != 0ull;
    int pos = lane;
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
      for (int j = k >> 1; j > 0; j >>= 1) {
        const unsigned long long w = shfl_xor_u64(v, j);
        const int wp = __shfl_xor(pos, j, 64);
        const bool keep_max = ((lane & j) == 0) == ((lane & k) == 0);
        const bool tk = keep_max ? (w > v) : (w < v);
        v = tk ? w : v;
        pos = tk ? wp : pos;
      }
    }
    s_bxu[lane] = det_box_finish(boxes_ws, rb);
    wave_lds_sync();
    const Box4 bs = s_bxu[pos];
    s_bx[lane] = bs;
    s_ar[lane] = (bs.c - bs.a) * (bs.d - bs.b);
  }
  __syncthreads();
  SEG_PHASE(3);
  // ---- suppression columns: col_i = the higher-ranked boxes j < i that would suppress box i
  // (the torchvision test is symmetric in the pair).  Wave w builds columns w, w + 4, ...,
  // four at a time (independent LDS broadcasts and ballots in flight).
  {
    const Box4 bj = lane < q ? s_bx[lane] : Box4{0.f, 0.f, 0.f, 0.f};
    const float aj = lane < q ? s_ar[lane] : 0.f;
    constexpr int kU = 4;
    for (int i0 = wv; i0 < q; i0 += kSegW * kU) {
      Box4 bi[kU];
      float ai[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int i = min(i0 + kSegW * u, 63);
        bi[u] = s_bx[i];
        ai[u] = s_ar[i];
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int i = i0 + kSegW * u;
        const bool act = lane < i && i < q;
        bool amb;
        float inter, un;
        const bool sup = tv_fast(bi[u], ai[u], bj, aj, thr, amb, inter, un);
        unsigned long long col = __ballot(act && sup);
        const unsigned long long am = __ballot(act && amb);
        if (am != 0ull) {   // rare: exact division for the lanes within the margin
          const bool ex = act && amb && (inter / un > thr);
          col = (col & ~am) | __ballot(ex);
        }
        if (lane == 0 && i < q) s_rows[i] = col;
      }
    }
  }
#ifdef SBOD_PHASE_CLOCKS
  long long ph_rows = clock64();
#endif
  __syncthreads();
  if (wv != 0) return;
#ifdef SBOD_PHASE_CLOCKS
  long long ph_sync = clock64();
#endif
  // ---- wave 0: the greedy result as a parallel fixpoint (column i in lane i).  Box i is kept
  // once every possible suppressor above it is known suppressed, and suppressed once a kept box
  // above it suppresses it; each round decides at least the first undecided box, so this is
  // exactly the sequential greedy order, in as many rounds as the longest suppression chain.
  const unsigned long long mycol = lane < q ? s_rows[lane] : 0ull;
  const unsigned long long valid = q == 64 ? ~0ull : ((1ull << q) - 1ull);
  unsigned long long kept = 0, supp = 0;
  for (int round = 0; round < 64; ++round) {
    const unsigned long long und = valid & ~(kept | supp);
    if (und == 0ull) break;
    const bool mine = (und >> lane) & 1ull;
    kept |= __ballot(mine && (mycol & ~supp) == 0ull);
    supp |= __ballot(mine && (mycol & kept) != 0ull);
  }
#ifdef SBOD_PHASE_CLOCKS
  long long ph_sweep = clock64();
#endif
  unsigned long long *ko = o.kept + seg * stride;
  const uint32_t llo = __builtin_amdgcn_readlane(static_cast<uint32_t>(v), q - 1);
  const uint32_t lhi = __builtin_amdgcn_readlane(static_cast<uint32_t>(v >> 32), q - 1);
  const unsigned long long lk = n > q && !corrupt ? ((static_cast<unsigned long long>(lhi) << 32) | llo) : 0ull;
  const uint32_t kcv = corrupt ? kKcCorrupt : static_cast<uint32_t>(__popcll(kept));
  if constexpr (kWT) {
    if ((kept >> lane) & 1ull) st_wt_u64(ko + __popcll(kept & ((1ull << lane) - 1ull)), v);
    if (lane == 0) {
      st_wt_u32(reinterpret_cast<int32_t *>(o.kc) + seg, kcv);
      st_wt_u64(o.lastkey + seg, lk);
    }
  } else {
    if ((kept >> lane) & 1ull) ko[__popcll(kept & ((1ull << lane) - 1ull))] = v;
    if (lane == 0) {
      o.kc[seg] = kcv;
      o.lastkey[seg] = lk;
    }
  }
  STAMP_END(2, 0);
#ifdef SBOD_PHASE_CLOCKS
  if (lane == 0) ph[4] = clock64();
  if (lane == 0 && (c == 1 || c == 8) && (b == 0 || b == 5))
    printf("seg4 b%d c%d n=%d: load %lld select+compact %lld sort+boxes %lld rows %lld sync %lld sweep %lld store %lld total %lld\n",
           b, c, n, ph[1] - ph[0], ph[2] - ph[1], ph[3] - ph[2], ph_rows - ph[3], ph_sync - ph_rows, ph_sweep - ph_sync,
           ph[4] - ph_sweep, ph[4] - ph[0]);
#endif
}

#ifndef SBOD_SEG_W
#define SBOD_SEG_W 4
#endif
// waves per pass-1 segment workgroup.  A/B builds: -DSBOD_SEG_W=8 made the kernel 0.6 us faster
// alone but the pipelined step's GPU interval 34.0-34.9 vs 30.5-31.7 us (r6_det_ab_a.jsonl)
constexpr int kSegPassW = SBOD_SEG_W;
__global__ __launch_bounds__(64 * kSegPassW) void k_det_segment_w4(
    const unsigned long long *__restrict__ cand, const uint32_t *__restrict__ cand_count,
    const DetBoxes boxes_ws, int P, int C, int window, int stride, float thr, SegOut o) {
  segment_w<kSegPassW, false>(cand, cand_count, boxes_ws, P, C, window, stride, thr, o);
}

// ----------------------------------------------------------------------------- K3
constexpr int kMergeLdsKeys = 8192;   // general path: merged keys sorted in LDS (radix-select first)
constexpr int kRankScores = 8192;     // fast path: staged class-prefix merged keys
constexpr int kFastOut = 1024;        // fast path: selected top-R (+ ties) keys
constexpr int kFastStage = 512;       // fast path: merged prefix ordered for the final NMS
constexpr int kRankC = 64;            // rank path: classes (incl. background) handled by wave-0 lanes
constexpr int kRankLds = (kRankScores + kFastOut) * 8;   // rank path: dynamic LDS it may use

// Count of entries of a non-increasing score list that precede score s in the merged order:
// scores > s, plus scores == s when the list's class is lower (the concatenation is in class order).
__device__ __forceinline__ int count_before(const float *a, int n, float s, bool ties_before) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    const float v = a[mid];
    if (v > s || (ties_before && v == s)) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// Rank path of the per-image merge (detect without a final NMS, C <= 64): the first top_k of the
// merged order (score desc, then class, then in-class rank — models/utils.py:274-290: the
// class-order concatenation, then a descending sort when more than top_k were kept).
//   1. the kept windows of all classes -> LDS (one coalesced pass; kc / lastkey meanwhile);
//   2. wave 0 (one lane per class): class offsets, truncation bound, and a lower bound L on the
//      top_k-th merged key — with k* the smallest k such that the first min(kc_c, k) entries of
//      all classes number >= top_k, every one of those is >= L = min_c (entry min(kc_c,k*)-1 of
//      class c), so no entry below L can rank < top_k;
//   3. the entries >= L (typically ~2 top_k of the ~20 x 64 kept) are compacted, and each one's
//      merged rank is counted against all of them (broadcast LDS reads, the count split over
//      the block's threads) — no sort, no radix select, three barriers;
//   4. entries with rank < top_k are written at their rank.
// Returns -1 when not applicable (the caller's general merge runs), else the merge status.
template <bool kWT = false>   // kWT: kept / kc / lastkey were written in this launch (sc1 loads)
__device__ __forceinline__ int merge_rank(
    const unsigned long long *kept, const uint32_t *kc, const unsigned long long *lastkey,
    const DetBoxes boxes_ws, int P, int C, int stride, int wmax, int top_k, int pass,
    int32_t *__restrict__ need, float *__restrict__ out_boxes, int64_t *__restrict__ out_labels,
    float *__restrict__ out_scores, int32_t *__restrict__ out_count, int b) {
  extern __shared__ __attribute__((aligned(16))) unsigned char s_raw[];
  __shared__ uint32_t r_off[kRankC + 1], r_kc[kRankC];
  __shared__ unsigned long long r_L;
  __shared__ uint32_t r_trunc, r_kth;
  __shared__ int r_m, r_total, r_any, r_corrupt;
  const int nslot = (C - 1) * wmax;   // kc <= wmax entries per class (stored at `stride`)
  if (C > kRankC || static_cast<size_t>(nslot) * 20 > static_cast<size_t>(kRankLds) || (nslot & 1)) return -1;
  const int tid = threadIdx.x, NT = blockDim.x;
  const int64_t sb0 = static_cast<int64_t>(b) * C;
#ifdef SBOD_PHASE_CLOCKS
  long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
  SEG_PHASE(0);
  unsigned long long *sl = reinterpret_cast<unsigned long long *>(s_raw);   // [nslot] kept windows
  unsigned long long *sk = sl + nslot;                                      // [<= nslot] entries >= L
  uint32_t *rk = reinterpret_cast<uint32_t *>(sk + nslot);                 // [<= nslot] ranks
  {
    const unsigned long long *kb = kept + (sb0 + 1) * stride;   // classes 1..C-1
    constexpr int kB = 4;
    for (int s0 = 0; s0 < nslot; s0 += kB * NT) {
      unsigned long long r[kB];
#pragma unroll
      for (int k = 0; k < kB; ++k) {
        const int sidx = min(s0 + k * NT + tid, nslot - 1), cc = sidx / wmax;
        const unsigned long long *kp = kb + static_cast<int64_t>(cc) * stride + (sidx - cc * wmax);
        r[k] = kWT ? ld_wt_u64(kp) : *kp;
      }
#pragma unroll
      for (int k = 0; k < kB; ++k) {
        const int s = s0 + k * NT + tid;
        if (s < nslot) {
          sl[s] = r[k];
          rk[s] = 0u;
        }
      }
    }
  }
  uint32_t kcv = 0;
  if (tid < 64) {
    const int c = tid;
    const bool cv = c >= 1 && c < C;
    const int64_t sc = sb0 + (cv ? c : 1);
    const uint32_t kc0 = kWT ? ld_wt_u32(reinterpret_cast<const int32_t *>(kc) + sc) : kc[sc];
    const unsigned long long lk0 = kWT ? ld_wt_u64(lastkey + sc) : lastkey[sc];
    kcv = cv ? kc0 : 0u;
    const unsigned long long lk = cv ? lk0 : 0ull;
    uint32_t incl = kcv;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t v = __shfl_up(incl, off, 64);
      if (c >= off) incl += v;
    }
    if (c <= C) r_off[c] = incl - kcv;
    r_kc[c] = kcv;
    uint32_t tr = lk != 0ull ? static_cast<uint32_t>(lk >> 32) : 0u;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) tr = max(tr, static_cast<uint32_t>(__shfl_xor(tr, m, 64)));
    const int total = static_cast<int>(__shfl(incl, 63, 64));
    const bool any = __ballot(lk != 0ull) != 0ull;   // whole wave (not inside the lane-0 branch)
    const bool corrupt = __ballot(kcv == kKcCorrupt) != 0ull;
    if (c == 0) {
      r_corrupt = corrupt;
      r_trunc = tr;
      r_any = any;
      r_total = total;
      r_m = 0;
      r_kth = 0u;
    }
  }
  __syncthreads();
  SEG_PHASE(1);
  if (r_corrupt) {   // a segment met a prior index >= P: no detections, the caller is told
    if (tid == 0) {
      if (pass == 1) need[b] = 0;
      out_count[b] = kDetCorrupt;
    }
    return 0;
  }
  const int total = r_total;
  const bool any_trunc = r_any != 0;
  float *ob = out_boxes + static_cast<int64_t>(b) * top_k * 4;
  int64_t *ol = out_labels + static_cast<int64_t>(b) * top_k;
  float *os = out_scores + static_cast<int64_t>(b) * top_k;
  auto emit = [&](int r, int c, unsigned long long key) {
    st4(ob + 4 * r, det_box(boxes_ws, b, key_low(key)));
    ol[r] = c;
    os[r] = key_score(key);
  };
  auto undecided = [&]() {
    if (tid == 0) {
      if (pass == 1) need[b] = 1;
      out_count[b] = -1;
    }
    return 1;
  };
  if (total <= top_k) {
    if (any_trunc) return undecided();   // a truncated window hides how many more exist
    if (total == 0) {                    // models/utils.py:274-277 placeholder
      if (tid == 0) {
        st4(ob, Box4{0.f, 0.f, 1.f, 1.f});
        ol[0] = 0;
        os[0] = 0.f;
        out_count[b] = 1;
      }
      return 0;
    }
    for (int r = tid; r < total; r += NT) {   // all kept, in class order
      int lo = 1, hi = C - 1;
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (r_off[mid] <= static_cast<uint32_t>(r)) lo = mid;
        else hi = mid - 1;
      }
      emit(r, lo, sl[(lo - 1) * wmax + (r - static_cast<int>(r_off[lo]))]);
    }
    if (tid == 0) out_count[b] = total;
    return 0;
  }
  auto mkey = [&](int c, int pos) {
    return (sl[(c - 1) * wmax + pos] & 0xffffffff00000000ull) |
           (0xffffffffu - ((static_cast<uint32_t>(c) << 24) | static_cast<uint32_t>(pos)));
  };
  if (tid < 64) {
    const int c = tid;
    const bool cv = c >= 1 && c < C && kcv > 0u;
    // k*: the smallest k with sum_c min(kc_c, k) >= top_k (exists: total > top_k); lane l tests
    // k = base + l + 1, the class counts read from the lanes that hold them
    int kstar = 1;
    for (int base = 0;; base += 64) {
      const uint32_t k = static_cast<uint32_t>(base + c + 1);
      uint32_t f = 0;
      for (int c2 = 1; c2 < C; ++c2) f += min(static_cast<uint32_t>(__builtin_amdgcn_readlane(kcv, c2)), k);
      const unsigned long long hit = __ballot(f >= static_cast<uint32_t>(top_k));
      if (hit) {
        kstar = base + __builtin_ctzll(hit) + 1;
        break;
      }
    }
    unsigned long long lc = cv ? mkey(c, static_cast<int>(min(kcv, static_cast<uint32_t>(kstar))) - 1) : ~0ull;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
      const unsigned long long o = shfl_xor_u64(lc, m);
      lc = o < lc ? o : lc;
    }
    if (c == 0) r_L = lc;
  }
  __syncthreads();
  SEG_PHASE(2);
  const unsigned long long L = r_L;
  for (int s = tid; s < nslot; s += NT) {
    const int c = s / wmax + 1, pos = s - (c - 1) * wmax;
    if (pos < static_cast<int>(min(r_kc[c], static_cast<uint32_t>(top_k)))) {
      const unsigned long long k = mkey(c, pos);
      if (k >= L) sk[atomicAdd(&r_m, 1)] = k;
    }
  }
  __syncthreads();
  SEG_PHASE(3);
  const int m = r_m;
  // the box of this thread's first entry, loaded now (unconditional, clamped: m >= top_k >= 1)
  // so its latency runs under the rank counting; emitted below if the entry's rank < top_k
  const int e0 = min(tid, m - 1);
  const uint32_t low0 = 0xffffffffu - static_cast<uint32_t>(sk[e0]);
  const RawBox box0 = det_box_issue(
      boxes_ws, b, key_low(sl[(static_cast<int>(low0 >> 24) - 1) * wmax + static_cast<int>(low0 & 0xffffffu)]));
  const int nsplit = max(1, min(16, NT / m)), per = (m + nsplit - 1) / nsplit;
  for (int t = tid; t < m * nsplit; t += NT) {
    const int e = t % m, part = t / m;
    const int j0 = part * per, j1 = min(m, j0 + per);
    const unsigned long long ke = sk[e];
    uint32_t cnt = 0;
    int j = j0;
    if ((j & 1) && j < j1) cnt += sk[j++] > ke ? 1u : 0u;
    // 16-byte broadcast reads (ds_read_b128: 4 LDS cycles per 2 keys, half of ds_read2_b64's),
    // four in flight; sk is 16-byte aligned (nslot even, see the carve above)
    const ulonglong2 *sk2 = reinterpret_cast<const ulonglong2 *>(sk);
    for (; j + 8 <= j1; j += 8) {
      ulonglong2 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = sk2[(j >> 1) + u];
#pragma unroll
      for (int u = 0; u < 4; ++u) cnt += (v[u].x > ke ? 1u : 0u) + (v[u].y > ke ? 1u : 0u);
    }
    for (; j < j1; ++j) cnt += sk[j] > ke ? 1u : 0u;
    if (cnt) atomicAdd(&rk[e], cnt);
  }
  __syncthreads();
  SEG_PHASE(4);
  for (int e = tid; e < m; e += NT) {
    const uint32_t rank = rk[e];
    if (rank < static_cast<uint32_t>(top_k)) {
      const unsigned long long k = sk[e];
      const uint32_t low = 0xffffffffu - static_cast<uint32_t>(k);
      const int c = static_cast<int>(low >> 24), pos = static_cast<int>(low & 0xffffffu);
      const unsigned long long key = sl[(c - 1) * wmax + pos];
      if (e == tid) {   // the prefetched box
        st4(ob + 4 * rank, det_box_finish(boxes_ws, box0));
        ol[rank] = c;
        os[rank] = key_score(key);
      } else {
        emit(static_cast<int>(rank), c, key);
      }
      if (rank == static_cast<uint32_t>(top_k - 1)) r_kth = static_cast<uint32_t>(k >> 32);
    }
  }
  __syncthreads();
  SEG_PHASE(5);
#ifdef SBOD_PHASE_CLOCKS
  if (tid == 0 && (b == 0 || b == 5))
    printf("mrank p%d b%d total=%d m=%d: load+scan %lld L %lld compact %lld rank %lld emit %lld total %lld\n", pass, b,
           total, m, ph[1] - ph[0], ph[2] - ph[1], ph[3] - ph[2], ph[4] - ph[3], ph[5] - ph[4], ph[5] - ph[0]);
#endif
  // a truncated class may hide candidates scoring up to its window's last key: the top_k-th
  // output must beat them all (else the wider second-pass window decides)
  if (any_trunc && !(r_kth > r_trunc)) return undecided();
  if (tid == 0) out_count[b] = top_k;
  return 0;
}

// pass: 0 = single pass (invalid -> count -1), 1 = first of two (invalid -> need[b] = 1),
// 2 = second (only images with need[b]; invalid -> count -1).
__device__ __forceinline__ int merge_body(
    const unsigned long long *kept, const uint32_t *kc,
    const unsigned long long *lastkey, const DetBoxes boxes_ws, int P,
    int C, int window, int wmax, int top_k, float final_nms, int general, int pass,
    int32_t *__restrict__ need, unsigned long long *__restrict__ scratch,
    float *__restrict__ out_boxes, int64_t *__restrict__ out_labels,
    float *__restrict__ out_scores, int32_t *__restrict__ out_count) {
  extern __shared__ __attribute__((aligned(16))) unsigned char s_raw[];
  __shared__ uint32_t s_off[257], s_zoff[257];
  __shared__ uint32_t s_hist[2048];
  __shared__ int s_misc[4];
  __shared__ unsigned long long s_st[2];
  __shared__ float s_trunc;
  __shared__ int s_any_trunc, s_cnt, s_corrupt;
  __shared__ unsigned long long s_flag[16];
  __shared__ unsigned long long s_m[kMergeThreads];
  __shared__ int s_nk;
  __shared__ uint32_t s_kc[256];
  __shared__ float s_lk[256];
  const int b = blockIdx.x, tid = threadIdx.x;
  const int64_t sb0 = static_cast<int64_t>(b) * C;
  if (pass == 2 && need[b] == 0) return 0;
  if (final_nms < 0.f && !general) {
    const int st = merge_rank(kept, kc, lastkey, boxes_ws, P, C, window, wmax, top_k, pass, need, out_boxes,
                              out_labels, out_scores, out_count, b);
    if (st >= 0) return st;
  }
#ifdef SBOD_PHASE_CLOCKS
  long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
  SEG_PHASE(0);
  const int window_stride = window;
  for (int c = tid; c < C; c += blockDim.x) {   // all per-class loads in flight together
    s_kc[c] = c == 0 ? 0u : kc[sb0 + c];
    const unsigned long long lk = c == 0 ? 0ull : lastkey[sb0 + c];
    s_lk[c] = lk != 0ull ? key_score(lk) : __builtin_nanf("");
  }
  __syncthreads();
  if (tid == 0) {
    uint32_t acc = 0;
    float tr = -__builtin_inff();
    int any = 0, corrupt = 0;
    s_off[0] = 0;
    for (int c = 0; c < C; ++c) {
      corrupt |= s_kc[c] == kKcCorrupt;
      acc += s_kc[c];
      s_off[c + 1] = acc;
      if (s_lk[c] == s_lk[c]) {
        any = 1;
        tr = fmaxf(tr, s_lk[c]);
      }
    }
    s_trunc = tr;
    s_any_trunc = any;
    s_corrupt = corrupt;
  }
  __syncthreads();
  if (s_corrupt) {   // a segment met a prior index >= P: no detections, the caller is told
    if (tid == 0) {
      if (pass == 1) need[b] = 0;
      out_count[b] = kDetCorrupt;
    }
    return 0;
  }
  // an undecidable image: ask for the second pass (pass 1) or report -1
  auto undecided = [&]() {
    if (tid == 0) {
      if (pass == 1) need[b] = 1;
      out_count[b] = -1;
    }
  };
  SEG_PHASE(1);
  if (pass == 1 && tid == 0) need[b] = 0;
  const int total = static_cast<int>(s_off[C]);
  const bool any_trunc = s_any_trunc != 0;
  const float trunc_score = s_trunc;
  float *ob = out_boxes + static_cast<int64_t>(b) * top_k * 4;
  int64_t *ol = out_labels + static_cast<int64_t>(b) * top_k;
  float *os = out_scores + static_cast<int64_t>(b) * top_k;
  auto emit = [&](int r, int c, unsigned long long key) {
    const uint32_t p = key_low(key);
    st4(ob + 4 * r, det_box(boxes_ws, b, p));
    ol[r] = c;
    os[r] = key_score(key);
  };
  auto class_of = [&](const uint32_t *off, int i) {   // largest c in [1, C-1] with off[c] <= i
    int lo = 1, hi = C - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (off[mid] <= static_cast<uint32_t>(i)) lo = mid;
      else hi = mid - 1;
    }
    return lo;
  };
  auto ck_of = [&](int c, int pos) { return kept[(sb0 + c) * window_stride + pos]; };
  if (total == 0) {  // models/utils.py:274-277 placeholder
    if (any_trunc) {
      undecided();
      return 1;
    } else if (tid == 0) {
      st4(ob, Box4{0.f, 0.f, 1.f, 1.f});
      ol[0] = 0;
      os[0] = 0.f;
      out_count[b] = 1;
    }
    return 0;
  }
  if (final_nms < 0.f && !any_trunc && total <= top_k) {  // all kept, in class order
    for (int r = tid; r < total; r += blockDim.x) {
      const int c = class_of(s_off, r);
      emit(r, c, ck_of(c, r - s_off[c]));
    }
    if (tid == 0) out_count[b] = total;
    return 0;
  }
  if (final_nms < 0.f && total <= top_k) {  // a truncated window hides how many more exist
    undecided();
    return 1;
  }
  // R = how many leading entries of the merged order are needed
  const int R = final_nms < 0.f ? top_k : min(total, general ? kMergeStage : kFastStage);
  int *ord = nullptr;          // ord[r] = class << 24 | position, r < R
  unsigned long long *sk = nullptr;
  bool fast = !general && R <= kFastOut;
  if (fast) {
    if (tid == 0) {
      uint32_t acc = 0;
      s_zoff[0] = 0;
      for (int c = 0; c < C; ++c) {
        const uint32_t k = min(s_kc[c], static_cast<uint32_t>(R));   // s_kc[0] == 0 (LDS, not HBM)
        acc += k;
        s_zoff[c + 1] = acc;
      }
    }
    __syncthreads();
    fast = s_zoff[C] <= static_cast<uint32_t>(kRankScores);
  }
  if (fast) {
    // class prefixes (<= R each) -> LDS, then the exact top-R of their merged keys
    unsigned long long *mk = reinterpret_cast<unsigned long long *>(s_raw);     // [kRankScores]
    unsigned long long *top = mk + kRankScores;                                // [kFastOut]
    ord = reinterpret_cast<int *>(top + kFastOut);                             // [R]
    const int nz = static_cast<int>(s_zoff[C]);
    for (int e = tid; e < nz; e += blockDim.x) {
      const int c = class_of(s_zoff, e);
      const uint32_t pos = e - s_zoff[c];
      mk[e] = (ck_of(c, pos) & 0xffffffff00000000ull) |
              (0xffffffffu - ((static_cast<uint32_t>(c) << 24) | pos));
    }
    __syncthreads();
    SEG_PHASE(2);
    int m;
    if (nz <= R) {
      const int N = next_pow2(max(nz, 2));
      for (int i = tid; i < N; i += blockDim.x) top[i] = i < nz ? mk[i] : 0ull;
      __syncthreads();
      bitonic_desc(top, N);
      m = nz;
    } else {
      m = block_topk_lds(mk, nz, R, top, kFastOut, s_hist, s_misc);
    }
    if (m > kFastOut) {  // pathological ties: re-run on the general path
      if (tid == 0) out_count[b] = -1;
      return 0;
    }
    SEG_PHASE(3);
    for (int r = tid; r < R; r += blockDim.x) ord[r] = static_cast<int>(0xffffffffu - static_cast<uint32_t>(top[r]));
    __syncthreads();
  } else {
    // general path: sort merged keys (radix-select the leading R first when they do not fit)
    sk = reinterpret_cast<unsigned long long *>(s_raw);
    auto merged_key = [&](int i) {
      const int c = class_of(s_off, i);
      const uint32_t pos = i - s_off[c];
      return (ck_of(c, pos) & 0xffffffff00000000ull) |
             (0xffffffffu - ((static_cast<uint32_t>(c) << 24) | pos));
    };
    int N;
    if (total <= kMergeLdsKeys) {
      N = next_pow2(max(total, 2));
      for (int i = tid; i < N; i += blockDim.x) sk[i] = i < total ? merged_key(i) : 0ull;
    } else {
      unsigned long long *g = scratch + static_cast<int64_t>(b) * C * window_stride;
      for (int i = tid; i < total; i += blockDim.x) g[i] = merged_key(i);
      __threadfence_block();
      __syncthreads();
      const unsigned long long T = radix_select_desc(g, total, R, s_hist, s_st);
      N = next_pow2(max(R, 2));
      if (tid == 0) s_cnt = 0;
      for (int i = tid; i < N; i += blockDim.x) sk[i] = 0ull;
      __syncthreads();
      for (int i = tid; i < total; i += blockDim.x) {
        const unsigned long long k = g[i];
        if (k >= T) sk[atomicAdd(&s_cnt, 1)] = k;
      }
    }
    __syncthreads();
    bitonic_desc(sk, N);
    ord = reinterpret_cast<int *>(sk + kMergeLdsKeys);
    for (int r = tid; r < R; r += blockDim.x) ord[r] = static_cast<int>(0xffffffffu - static_cast<uint32_t>(sk[r]));
    __syncthreads();
  }
  auto entry = [&](int r, int &c) {
    const int v = ord[r];
    c = v >> 24;
    return ck_of(c, v & 0xffffff);
  };
  if (final_nms < 0.f) {  // n_objects > top_k: the top_k by score (models/utils.py:286-290)
    int c;
    if (any_trunc && !(key_score(entry(top_k - 1, c)) > trunc_score)) {
      undecided();
      return 1;
    }
    SEG_PHASE(4);
    for (int r = tid; r < top_k; r += blockDim.x) {
      const unsigned long long ck = entry(r, c);
      emit(r, c, ck);
    }
    if (tid == 0) out_count[b] = top_k;
    SEG_PHASE(5);
#ifdef SBOD_PHASE_CLOCKS
    if (tid == 0 && (b == 0 || b == 5))
      printf("merge p%d b%d nz=%d: prologue %lld gather %lld select+sort %lld ord+check %lld emit %lld total %lld\n",
             pass, b, total, ph[1] - ph[0], ph[2] - ph[1], ph[3] - ph[2], ph[4] - ph[3], ph[5] - ph[4], ph[5] - ph[0]);
#endif
    return 0;
  }
  // detect_tools: class-agnostic greedy NMS at final_nms over the merged order, first top_k
  Box4 *bx = reinterpret_cast<Box4 *>(ord + kMergeStage);
  float *ar = reinterpret_cast<float *>(bx + R);
  int *kl = reinterpret_cast<int *>(ar + R);
  uint8_t *kf = reinterpret_cast<uint8_t *>(kl + R);
  unsigned long long *mat = reinterpret_cast<unsigned long long *>(
      reinterpret_cast<uintptr_t>(kf + R + 15) & ~static_cast<uintptr_t>(15));
  for (int i = tid; i < R; i += blockDim.x) {
    int c;
    const unsigned long long ck = entry(i, c);
    const Box4 q = det_box(boxes_ws, b, key_low(ck));
    bx[i] = q;
    ar[i] = (q.c - q.a) * (q.d - q.b);
  }
  __syncthreads();
  const int nk = R <= kMatrixMax
                     ? block_greedy_matrix<SBOD_NMS_TV>(bx, ar, R, final_nms, 1.f, kf, kl, mat, &s_nk, top_k)
                     : block_greedy<SBOD_NMS_TV>(bx, ar, R, final_nms, 1.f, kf, kl, s_flag, s_m, &s_nk, top_k);
  const int nout = min(nk, top_k);
  // complete if every candidate that could precede the top_k-th survivor was ordered
  const bool enough = nk >= top_k || (R == total && !any_trunc);
  int c0;
  const bool ok = enough && (!any_trunc || key_score(entry(kl[top_k - 1], c0)) > trunc_score);
  if (!ok) {
    undecided();
    return 1;
  }
  for (int r = tid; r < nout; r += blockDim.x) {
    int c;
    const unsigned long long ck = entry(kl[r], c);
    emit(r, c, ck);
  }
  if (tid == 0) out_count[b] = nout;
  return 0;
}

__host__ __device__ inline size_t seg_lds(int window) {
  size_t wn = 2;
  while (wn < static_cast<size_t>(window)) wn <<= 1;
  const size_t mat = window <= kMatrixMax ? static_cast<size_t>(window) * ((window + 63) / 64) * 8 : 0;
  return static_cast<size_t>(kSegSortCap) * 8 + wn * 8 + static_cast<size_t>(window) * (16 + 4 + 4 + 1) + 16 + mat;
}

// Inline second pass scratch, after the segment layout in the merge's dynamic LDS:
// hist [2048] u32 | m [kMergeThreads] u64 | st [2] u64 | flag [16] u64 | nk, cnt, misc[4], tr[256] int
__host__ __device__ inline size_t inline2_lds(int window) {
  return ((seg_lds(window) + 15) & ~static_cast<size_t>(15)) + 2048 * 4 + (kMergeThreads + 2 + 16) * 8 + (6 + 256) * 4;
}

// Per-image merge.  pass 0: single pass; pass 1 (two-pass mode): an undecidable image runs the
// second pass inline — its truncated classes are re-selected with window w2 by segment_body in
// this block, then the merge is repeated (pass 2) — so no extra launches when (as usual) no
// image needs it.
// One by-value argument (the host cost of a launch grows with the argument count on this runtime:
// scripts/micro/launch_cost.hip).
struct MergeArgs {
  const unsigned long long *kept;
  const uint32_t *kc;
  const unsigned long long *lastkey;
  DetBoxes boxes_ws;
  int P, C, window, wfirst, top_k;
  float final_nms;
  int general, pass;
  int32_t *need;
  unsigned long long *scratch;
  float *out_boxes;
  int64_t *out_labels;
  float *out_scores;
  int32_t *out_count, *out_count_host;
  const unsigned long long *cand;
  uint32_t *cand_count;
  float thr;
  SegOut so;
};
__global__ __launch_bounds__(kMergeThreads) void k_det_merge(const MergeArgs ma) {
  const unsigned long long *kept = ma.kept;
  const uint32_t *kc = ma.kc;
  const unsigned long long *lastkey = ma.lastkey;
  const DetBoxes boxes_ws = ma.boxes_ws;
  const int P = ma.P, C = ma.C, window = ma.window, wfirst = ma.wfirst, top_k = ma.top_k;
  const float final_nms = ma.final_nms;
  const int general = ma.general, pass = ma.pass;
  int32_t *__restrict__ need = ma.need;
  unsigned long long *__restrict__ scratch = ma.scratch;
  float *__restrict__ out_boxes = ma.out_boxes;
  int64_t *__restrict__ out_labels = ma.out_labels;
  float *__restrict__ out_scores = ma.out_scores;
  int32_t *__restrict__ out_count = ma.out_count;
  int32_t *out_count_host = ma.out_count_host;
  const unsigned long long *cand = ma.cand;
  uint32_t *cand_count = ma.cand_count;
  const float thr = ma.thr;
  const SegOut so = ma.so;
  extern __shared__ __attribute__((aligned(16))) unsigned char s_raw[];
  STAMP_BEGIN();
  const int b = blockIdx.x;
  // the last reader of this image's candidate counters leaves them at zero for the next call
  // (no memset node in front of a captured detect); the image's count also goes straight to the
  // caller's pinned host buffer (thread 0 wrote out_count[b] itself: no copy launch)
  auto clear_counters = [&]() {
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += blockDim.x) cand_count[static_cast<int64_t>(b) * C + c] = 0u;
    if (out_count_host != nullptr && threadIdx.x == 0) out_count_host[b] = out_count[b];
  };
  const int st = merge_body(kept, kc, lastkey, boxes_ws, P, C, window, wfirst, top_k, final_nms, general, pass, need,
                            scratch, out_boxes, out_labels, out_scores, out_count);
  STAMP_END(3, 1);
  if (st == 0 || pass != 1) {
    clear_counters();
    return;
  }
  uint32_t *h2 = reinterpret_cast<uint32_t *>(s_raw + ((seg_lds(window) + 15) & ~static_cast<size_t>(15)));
  unsigned long long *m2 = reinterpret_cast<unsigned long long *>(h2 + 2048);
  unsigned long long *st2 = m2 + kMergeThreads, *fl2 = st2 + 2;
  int *iv = reinterpret_cast<int *>(fl2 + 16);   // nk, cnt, misc[4], tr[256]
  int *s_tr = iv + 6;
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x)   // classes truncated by the first window
    s_tr[c] = c > 0 && __builtin_nontemporal_load(lastkey + static_cast<int64_t>(b) * C + c) != 0ull;
  __syncthreads();
  for (int c = 1; c < C; ++c)
    if (s_tr[c])
      segment_body(cand, cand_count, boxes_ws, P, C, b, c, window, window, thr, so, s_raw, h2, st2, fl2, m2,
                   iv, iv + 1, iv + 2);
  __syncthreads();
  merge_body(kept, kc, lastkey, boxes_ws, P, C, window, window, top_k, final_nms, general, 2, need, scratch, out_boxes,
             out_labels, out_scores, out_count);
  clear_counters();
}

// ----------------------------------------------------------------------------- K2 + K3 fused
// The segment pass and the per-image merge in ONE launch (detect without a final NMS, the rank
// path of the merge): (C - 1) x B workgroups of W waves run segment_w for their (image, class),
// write the class's kept window through (sc1), drain, and count themselves in at their image; the
// image's last class runs the merge (merge_rank over sc1 loads of the image's windows), writes the
// outputs and the host count, and leaves the image's candidate counters and arrival word zero.
// No workgroup waits for another (the last arriver is told by its own atomic), so the grid needs
// no co-residency.  An image the first window cannot decide reports -1, exactly as the
// single-pass merge does (the host re-runs it with a wider window).
template <int W>
__global__ __launch_bounds__(64 * W) void k_det_nms(
    const unsigned long long *__restrict__ cand, uint32_t *cand_count, const DetBoxes boxes_ws, int P,
    int C, int window, int stride, float thr, SegOut o, uint32_t *arrive, int top_k, float *__restrict__ out_boxes,
    int64_t *__restrict__ out_labels, float *__restrict__ out_scores, int32_t *__restrict__ out_count,
    int32_t *out_count_host) {
  __shared__ int s_last;
  segment_w<W, true>(cand, cand_count, boxes_ws, P, C, window, stride, thr, o);
  drain_vm();   // this wave's kept keys / kc / lastkey written through
  __syncthreads();
  const int b = blockIdx.y;
  if (threadIdx.x == 0) {
    const uint32_t old = __hip_atomic_fetch_add(arrive + b, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool last = old == static_cast<uint32_t>(C - 2);
    if (last) __hip_atomic_store(arrive + b, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = last ? 1 : 0;
  }
  __syncthreads();
  if (!s_last) return;
  merge_rank<true>(o.kept, o.kc, o.lastkey, boxes_ws, P, C, stride, window, top_k, 0, nullptr, out_boxes, out_labels,
                   out_scores, out_count, b);
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) cand_count[static_cast<int64_t>(b) * C + c] = 0u;
  if (out_count_host != nullptr && threadIdx.x == 0) out_count_host[b] = out_count[b];
}
constexpr int kNmsW = 8;   // waves per (image, class) in k_det_nms

// ----------------------------------------------------------------------------- single segment
template <int V>
__global__ __launch_bounds__(1024) void k_nms_single(const float *__restrict__ boxes,
                                                     const float *__restrict__ scores, int n,
                                                     int q, float thr, float beta,
                                                     unsigned long long *__restrict__ gkeys,
                                                     int64_t *__restrict__ keep,
                                                     int32_t *__restrict__ count) {
  extern __shared__ __attribute__((aligned(16))) unsigned char s_raw[];
  __shared__ uint32_t s_hist[256];
  __shared__ unsigned long long s_st[2];
  __shared__ unsigned long long s_flag[16];
  __shared__ unsigned long long s_m[1024];
  __shared__ int s_nk, s_cnt;
  const int N = next_pow2(max(q, 2));
  unsigned long long *sk = reinterpret_cast<unsigned long long *>(s_raw);
  Box4 *sb = reinterpret_cast<Box4 *>(sk + N);
  float *sa = reinterpret_cast<float *>(sb + q);
  int *kl = reinterpret_cast<int *>(sa + q);
  uint8_t *kf = reinterpret_cast<uint8_t *>(kl + q);
  if (q == n) {
    for (int i = threadIdx.x; i < N; i += blockDim.x)
      sk[i] = i < n ? make_key(scores[i], static_cast<uint32_t>(i)) : 0ull;
  } else {
    for (int i = threadIdx.x; i < n; i += blockDim.x) gkeys[i] = make_key(scores[i], static_cast<uint32_t>(i));
    __syncthreads();
    const unsigned long long T = radix_select_desc(gkeys, n, q, s_hist, s_st);
    if (threadIdx.x == 0) s_cnt = 0;
    for (int i = threadIdx.x; i < N; i += blockDim.x) sk[i] = 0ull;
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      const unsigned long long k = gkeys[i];
      if (k >= T) sk[atomicAdd(&s_cnt, 1)] = k;
    }
  }
  __syncthreads();
  bitonic_desc(sk, N);
  for (int i = threadIdx.x; i < q; i += blockDim.x) {
    const Box4 bx = ld4(boxes + 4 * static_cast<int64_t>(key_low(sk[i])));
    sb[i] = bx;
    sa[i] = (bx.c - bx.a) * (bx.d - bx.b);
  }
  __syncthreads();
  const int nk = block_greedy<V>(sb, sa, q, thr, beta, kf, kl, s_flag, s_m, &s_nk);
  for (int k = threadIdx.x; k < n; k += blockDim.x) keep[k] = k < nk ? static_cast<int64_t>(key_low(sk[kl[k]])) : 0;
  if (threadIdx.x == 0) *count = nk;
}


size_t single_lds(int q) {
  return static_cast<size_t>(next_pow2_host(q < 2 ? 2 : q)) * 8 + static_cast<size_t>(q) * (16 + 4 + 4 + 1) + 64;
}

}  // namespace sbod

using namespace sbod;

namespace {
struct DetWs {
  unsigned long long *cand, *kept, *lastkey, *scratch;
  uint32_t *count, *kc, *arrive;
  int32_t *need;
  size_t bytes;
};
DetWs carve_det(void *w, int B, int P, int C, int window) {
  DetWs r;
  size_t o = 0;
  // the candidate counters first: their place depends on B * C only (sbod_detect_f32's
  // SBOD_DETECT_COUNTERS_ZEROED contract)
  r.count = ws_at<uint32_t>(w, o);
  r.arrive = ws_at<uint32_t>(w, static_cast<size_t>(B) * C * 4);   // [B] after the counters
  o += align_up(static_cast<size_t>(B) * C * 4 + static_cast<size_t>(B) * 4);
  r.cand = ws_at<unsigned long long>(w, o);
  o += align_up(static_cast<size_t>(B) * C * P * 8);
  r.kept = ws_at<unsigned long long>(w, o);
  o += align_up(static_cast<size_t>(B) * C * window * 8);
  r.kc = ws_at<uint32_t>(w, o);
  o += align_up(static_cast<size_t>(B) * C * 4);
  r.lastkey = ws_at<unsigned long long>(w, o);
  o += align_up(static_cast<size_t>(B) * C * 8);
  r.scratch = ws_at<unsigned long long>(w, o);
  o += align_up(static_cast<size_t>(B) * C * window * 8);
  r.need = ws_at<int32_t>(w, o);
  o += align_up(static_cast<size_t>(B) * 4);
  r.bytes = o;
  return r;
}
constexpr int kFirstWindow = 64;
int clampw(int w, int P) {
  if (w > kMaxWindow) w = kMaxWindow;
  if (w > P) w = P < 1 ? 1 : P;
  return w < 1 ? 1 : w;
}
}  // namespace

extern "C" {

size_t sbod_detect_counter_bytes(int B, int C) {
  return align_up(static_cast<size_t>(B) * C * 4 + static_cast<size_t>(B) * 4);   // counters + arrival words
}

size_t sbod_detect_workspace_bytes(int B, int P, int C) {
  return carve_det(nullptr, B, P, C, clampw(kMaxWindow, P)).bytes;
}

int sbod_detect_f32(void *locs, const void *scores, int B, int P, int C,
                    const float *priors_cxcy, const uint8_t *pos_mask, int box_type, int act,
                    float min_score, float max_overlap, int top_k, float final_nms, int window,
                    int flags, float *det_boxes, int64_t *det_labels, float *det_scores,
                    int32_t *det_count, int32_t *det_count_host, float *debug_probs,
                    float *debug_boxes, void *workspace, size_t workspace_bytes, void *stream) {
  SBOD_REQUIRE((flags & ~(SBOD_DETECT_COUNTERS_ZEROED | SBOD_DETECT_INPUT_BF16 | SBOD_DETECT_FUSED)) == 0,
               "sbod_detect_f32: unknown flags 0x%x", flags);
  const bool bf16 = (flags & SBOD_DETECT_INPUT_BF16) != 0;
  SBOD_REQUIRE(!bf16 || C <= 32, "sbod_detect_f32: bf16 input supports C <= 32 (C=%d)", C);
  SBOD_REQUIRE(B > 0 && P > 0 && C >= 2 && C <= 256 && locs && scores && det_boxes && det_labels &&
                   det_scores && det_count && top_k > 0,
               "sbod_detect_f32: bad arguments (B=%d P=%d C=%d top_k=%d)", B, P, C, top_k);
  SBOD_REQUIRE(box_type != SBOD_BOX_OFFSET || priors_cxcy, "sbod_detect_f32: offset boxes need priors");
  SBOD_REQUIRE(C * (kDTile * 4 + (kDTile / 64) * 12) <= 160 * 1024, "sbod_detect_f32: C=%d too large", C);
  SBOD_REQUIRE(P < (1 << 24), "sbod_detect_f32: P=%d >= 2^24 unsupported", P);
  // window 0 (auto): a first window of 64 candidates per class, then next_pow2(top_k + 1) for
  // the truncated classes of images the first merge could not decide; window > 0: one pass;
  // window < 0: exhaustive (every class's candidates in chunks, k_det_segment_all).
  const bool exhaustive = window < 0;
  if (exhaustive) window = 0;
  const bool two = window <= 0 && !exhaustive;
  const int w2 = clampw(two || exhaustive ? next_pow2_host(top_k + 1 > 64 ? top_k + 1 : 64) : window, P);
  const int w1 = two ? clampw(kFirstWindow < w2 ? kFirstWindow : w2, P) : w2;
  DetWs ws = carve_det(workspace, B, P, C, w2);
  if (workspace_bytes < ws.bytes) {
    set_error("sbod_detect_f32: workspace %zu < %zu", workspace_bytes, ws.bytes);
    return SBOD_E_WORKSPACE;
  }
  SBOD_REQUIRE(top_k <= kMergeStage, "sbod_detect_f32: top_k %d > %d unsupported", top_k, kMergeStage);
  const int general = w2 >= kMaxWindow ? 1 : 0;   // the retry window takes the general merge
  // fast path: keys [kRankScores] + top [kFastOut] | general: keys [kMergeLdsKeys]; then ord
  // [kMergeStage] and, for the final NMS, boxes/areas/klist/keep [R] + the bit matrix
  const size_t head = static_cast<size_t>(kRankScores + kFastOut) * 8 > static_cast<size_t>(kMergeLdsKeys) * 8
                          ? static_cast<size_t>(kRankScores + kFastOut) * 8 : static_cast<size_t>(kMergeLdsKeys) * 8;
  const size_t tools_general = static_cast<size_t>(kMergeStage) * 25;
  const size_t tools_fast = static_cast<size_t>(kMatrixMax) * 25 + 16 + static_cast<size_t>(kMatrixMax) * (kMatrixMax / 64) * 8;
  const size_t merge_lds = head + static_cast<size_t>(kMergeStage) * 4 +
                           (final_nms >= 0.f ? (tools_general > tools_fast ? tools_general : tools_fast) : 0);
  // every argument / LDS check comes before the first launch: k_det_prepare adds to the
  // candidate counters that only k_det_merge clears again, so a call must not stop in between
  const size_t all_lds = static_cast<size_t>(w2) * (8 + 16 + 4);
  SBOD_REQUIRE(!exhaustive || ((w2 >= top_k || w2 >= P) && all_lds <= 64 * 1024),
               "sbod_detect_f32: exhaustive mode supports top_k <= 2047");
  hipStream_t s = as_stream(stream);
  // the WHOLE aligned prefix (sbod_detect_counter_bytes): a caller that trusts it clean later (a
  // larger B * C whose counters reach into this call's alignment padding) must find zeros there,
  // not the candidate keys of an earlier, smaller call whose key region began inside it
  if ((flags & SBOD_DETECT_COUNTERS_ZEROED) == 0 &&
      hipMemsetAsync(ws.count, 0, sbod_detect_counter_bytes(B, C), s) != hipSuccess)
    return launch_status("hipMemsetAsync(detect)");
  DetArgs a{B, P, C, box_type, act, priors_cxcy, pos_mask, min_score, ws.cand, ws.count,
            debug_probs, debug_boxes, nullptr};
  // a.rows stays kDTile: balanced tiles (216 rows, six workgroups per CU at SSD512 B = 32) made
  // this kernel slower, 12.92 / 12.96 vs 12.58 / 12.54 us (the loss pass gains from them)
  // decoded on demand (det_box); without priors (CENTER / CORNER boxes) the dummy prior loads
  // read the output buffer's first 16 bytes (values unused)
  const DetBoxes bxs{locs, priors_cxcy ? priors_cxcy : det_boxes, P, box_type, bf16 ? 1 : 0};
  {
    KernelTimer kt("k_det_prepare", s, true);
    a.span = kt.span();
    const dim3 pg((P + a.rows - 1) / a.rows, B);
    const size_t pl = static_cast<size_t>(kDTile) * C * (bf16 ? 2 : 4) + (kDTile / 64) * C * 12;
    uint16_t *lh = reinterpret_cast<uint16_t *>(locs);
    const uint16_t *sh = reinterpret_cast<const uint16_t *>(scores);
    float *lf = reinterpret_cast<float *>(locs);
    const float *sf = reinterpret_cast<const float *>(scores);
    if (bf16) {
      if (C <= 8) tlaunch(kt, k_det_prepare<8, 0, uint16_t>, pg, dim3(kDTile), pl, s, a, lh, sh);
      else if (C <= 16) tlaunch(kt, k_det_prepare<16, 0, uint16_t>, pg, dim3(kDTile), pl, s, a, lh, sh);
      else if (C == 21) tlaunch(kt, k_det_prepare<24, 21, uint16_t>, pg, dim3(kDTile), pl, s, a, lh, sh);
      else if (C <= 24) tlaunch(kt, k_det_prepare<24, 0, uint16_t>, pg, dim3(kDTile), pl, s, a, lh, sh);
      else tlaunch(kt, k_det_prepare<32, 0, uint16_t>, pg, dim3(kDTile), pl, s, a, lh, sh);
    } else if (C <= 8) tlaunch(kt, k_det_prepare<8, 0>, pg, dim3(kDTile), pl, s, a, lf, sf);
    else if (C <= 16) tlaunch(kt, k_det_prepare<16, 0>, pg, dim3(kDTile), pl, s, a, lf, sf);
    else if (C == 21) tlaunch(kt, k_det_prepare<24, 21>, pg, dim3(kDTile), pl, s, a, lf, sf);
    else if (C <= 24) tlaunch(kt, k_det_prepare<24, 0>, pg, dim3(kDTile), pl, s, a, lf, sf);
    else if (C <= 32) tlaunch(kt, k_det_prepare<32, 0>, pg, dim3(kDTile), pl, s, a, lf, sf);
    else tlaunch(kt, k_det_prepare<0, 0>, pg, dim3(kDTile),
                 static_cast<size_t>(kDTile) * C * 4 + (kDTile / 64) * C * 12, s, a, lf, sf);
  }
  SBOD_LAUNCHED("k_det_prepare");
  SegOut so{ws.kept, ws.kc, ws.lastkey};
  // K2 + K3 in one launch (k_det_nms): the rank path of the merge (no final NMS, C <= kRankC, the
  // first window's kept lists fit its LDS), a first window of <= 64, and the single-pass contract
  // (an undecidable image reports -1 and the host widens its window)
  const int rank_slots = (C - 1) * w1;
  const bool fuse = !exhaustive && final_nms < 0.f && two && w1 <= 64 && C <= kRankC &&
                    static_cast<size_t>(rank_slots) * 20 <= static_cast<size_t>(kRankLds) && (rank_slots & 1) == 0 &&
                    (flags & SBOD_DETECT_FUSED) != 0;
  if (fuse) {
    KernelTimer kt("k_det_nms", s, true);
    tlaunch(kt, k_det_nms<kNmsW>, dim3(C - 1, B), dim3(64 * kNmsW), static_cast<size_t>(rank_slots) * 20, s,
            ws.cand, ws.count, bxs, P, C, w1, w2, max_overlap, so, ws.arrive, top_k, det_boxes, det_labels,
            det_scores, det_count, det_count_host);
    SBOD_LAUNCHED("k_det_nms");
    return SBOD_OK;
  }
  if (exhaustive) {
    KernelTimer kt("k_det_segment", s, true);
    tlaunch(kt, k_det_segment_all, dim3(C - 1, B), dim3(kAllThreads), all_lds, s, ws.cand, ws.count, bxs, P, C,
            w2, top_k, max_overlap, so);
  } else {
    KernelTimer kt("k_det_segment", s, true);
    if (w1 <= 64)
#ifdef SBOD_SEG_WAVE
      tlaunch(kt, k_det_segment_wave, dim3(C - 1, B), dim3(64), 0, s, ws.cand, ws.count, bxs,
                         P, C, w1, w2, max_overlap, so, nullptr);
#else
      tlaunch(kt, k_det_segment_w4, dim3(C - 1, B), dim3(64 * kSegPassW), 0, s, ws.cand, ws.count, bxs,
                         P, C, w1, w2, max_overlap, so);
#endif
    else
      tlaunch(kt, k_det_segment, dim3(C - 1, B), dim3(kSegThreads), seg_lds(w1), s, ws.cand,
                         ws.count, bxs, P, C, w1, w2, max_overlap, so, nullptr);
  }
  SBOD_LAUNCHED("k_det_segment");
  {
    // two-pass mode: the second pass runs inline in the merge blocks of undecidable images,
    // so the merge's dynamic LDS also covers one segment with window w2
    const size_t seg2 = two ? inline2_lds(w2) : 0;
    KernelTimer kt("k_det_merge", s, true);
    tlaunch(kt, k_det_merge, dim3(B), dim3(kMergeThreads), merge_lds > seg2 ? merge_lds : seg2, s,
            MergeArgs{ws.kept, ws.kc, ws.lastkey, bxs, P, C, w2, w1, top_k, final_nms, two ? 0 : general,
                      two ? 1 : 0, ws.need, ws.scratch, det_boxes, det_labels, det_scores, det_count,
                      det_count_host, ws.cand, ws.count, max_overlap, so});
  }
  SBOD_LAUNCHED("k_det_merge");
  return SBOD_OK;
}

size_t sbod_nms_workspace_bytes(int64_t n) { return align_up(static_cast<size_t>(n > 0 ? n : 1) * 8); }

int sbod_nms_f32(const float *boxes, const float *scores, int64_t n, float overlap, int top_k,
                 int variant, float beta1, int64_t *keep, int32_t *count, void *workspace,
                 size_t workspace_bytes, void *stream) {
  SBOD_REQUIRE(n >= 0 && keep && count && variant >= 0 && variant <= 2 && (n == 0 || (boxes && scores)),
               "sbod_nms_f32: bad arguments");
  hipStream_t s = as_stream(stream);
  if (n == 0) {
    if (hipMemsetAsync(count, 0, 4, s) != hipSuccess) return launch_status("hipMemsetAsync(nms)");
    return SBOD_OK;
  }
  SBOD_REQUIRE(n < (1ll << 31), "sbod_nms_f32: n too large");
  // TV: every candidate; REF / DIOU: the top_k highest BEFORE suppression (iou_utils.py:407)
  int q = static_cast<int>(n);
  if (variant != SBOD_NMS_TV && top_k > 0 && top_k < q) q = top_k;
  if (q > kMaxWindow) {
    set_error("sbod_nms_f32: %d candidates exceed the LDS window (%d)", q, kMaxWindow);
    return SBOD_E_UNSUPPORTED;
  }
  if (q < n && workspace_bytes < sbod_nms_workspace_bytes(n)) {
    set_error("sbod_nms_f32: workspace %zu < %zu", workspace_bytes, sbod_nms_workspace_bytes(n));
    return SBOD_E_WORKSPACE;
  }
  const size_t lds = single_lds(q);
  auto *gk = static_cast<unsigned long long *>(workspace);
  if (variant == SBOD_NMS_TV)
    hipLaunchKernelGGL(k_nms_single<SBOD_NMS_TV>, dim3(1), dim3(1024), lds, s, boxes, scores,
                       static_cast<int>(n), q, overlap, beta1, gk, keep, count);
  else if (variant == SBOD_NMS_REF)
    hipLaunchKernelGGL(k_nms_single<SBOD_NMS_REF>, dim3(1), dim3(1024), lds, s, boxes, scores,
                       static_cast<int>(n), q, overlap, beta1, gk, keep, count);
  else
    hipLaunchKernelGGL(k_nms_single<SBOD_NMS_DIOU>, dim3(1), dim3(1024), lds, s, boxes, scores,
                       static_cast<int>(n), q, overlap, beta1, gk, keep, count);
  SBOD_LAUNCHED("k_nms_single");
  return SBOD_OK;
}

}  // extern "C"

SBOD_STAMP_EXPORT(nms)

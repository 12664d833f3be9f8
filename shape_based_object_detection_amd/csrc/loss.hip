// Detection losses: the fused per-prior criterion pass (every criterion of models/*.py), the
// hard-negative mining top-k (radix select), the finaliser, and the standalone operators.Loss
// kernels.
//
// Fused pass, one workgroup = 256 priors of one image:
//   * the [256 x C] score tile is staged through LDS with coalesced loads (rows of C floats,
//     C odd -> conflict-free per-lane row reads), softmax / focal / CE and their gradients are
//     computed per lane in registers + LDS, and the gradient tile is stored back coalesced;
//   * locs are one 16-byte load per lane; the label / positive / negative state is derived
//     from the matcher's (obj, ovl) planes and the image's GT labels;
//   * gradients are produced in the same pass (forward-with-grad), scaled by the global
//     normaliser read from device memory (matcher total or an all-reduced copy for DP), so a
//     training step reads the predictions once and writes their gradients once.
// Roofline: HBM-bound; algorithmic bytes per launch = B*P*(4+C)*s read + B*P*(4+C)*s written.
#include <hip/hip_bf16.h>

#include <atomic>
#include <cstdlib>
#include <mutex>
#include <vector>

#include "match_dev.h"

namespace sbod {

SBOD_STAMP_DECL

// Diagnostic build only (-DSBOD_BLOCK_STAMPS, scripts/build_stamps_lib.sh): k_multibox's
// workgroups record eight wall-clock marks each while its stamps are armed — 0 wave 0's score
// tile committed, 1 the positive list's barrier passed, 2 wave 0's box regression done, 3..6
// each wave's rows done, 7 the gradient tile stored and the block sums taken — read by
// sbod_debug_mb_marks (scripts/mb_imbalance.py).  Compiles to nothing otherwise.
#ifdef SBOD_BLOCK_STAMPS
static __device__ unsigned long long g_mb_marks[SBOD_STAMP_REGION * 8];
#define MB_MARK(slot, cond)                                                                   \
  do {                                                                                        \
    if ((g_stamp_armed & (1 << 4)) && (cond)) {                                               \
      const unsigned _b = blockIdx.x + gridDim.x * blockIdx.y;                                \
      if (_b < SBOD_STAMP_REGION) g_mb_marks[_b * 8 + (slot)] = __builtin_amdgcn_s_memrealtime(); \
    }                                                                                         \
  } while (0)
// the fused finish's gatherer: when it first saw each record, and its own marks (0 entered,
// 1 thread 0's first sweep done, 2 every record folded, 3 loss written; 4 thread 0's sweeps)
static __device__ unsigned long long g_fin_seen[SBOD_STAMP_REGION];
static __device__ unsigned long long g_fin_marks[8];
#define FIN_SEEN(i)                                                                                 \
  do {                                                                                              \
    if ((g_stamp_armed & (1 << 4)) && (i) < SBOD_STAMP_REGION) g_fin_seen[i] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define FIN_MARK(slot, v)                                      \
  do {                                                         \
    if ((g_stamp_armed & (1 << 4))) g_fin_marks[slot] = (v);   \
  } while (0)
#else
#define MB_MARK(slot, cond) do { } while (0)
#define FIN_SEEN(i) do { } while (0)
#define FIN_MARK(slot, v) do { } while (0)
#endif

constexpr int kLTile = 256;
constexpr float kHalfBetaDefault = 0.5f / 9.f;

__device__ __forceinline__ float ldf(const float *p) { return *p; }
__device__ __forceinline__ float ldf(const uint16_t *p) {
  return __uint_as_float(static_cast<uint32_t>(*p) << 16);
}
__device__ __forceinline__ void stf(float *p, float v) { *p = v; }
__device__ __forceinline__ void stf(uint16_t *p, float v) {
  __hip_bfloat16 h = __float2bfloat16(v);
  *p = *reinterpret_cast<uint16_t *>(&h);
}

// torch.maximum / torch.minimum backward: on ties the gradient is split in half.
__device__ __forceinline__ float dmax_a(float a, float b) { return a > b ? 1.f : (a == b ? 0.5f : 0.f); }
__device__ __forceinline__ float dmin_a(float a, float b) { return a < b ? 1.f : (a == b ? 0.5f : 0.f); }

// [n] floats global <-> LDS, 16 bytes per lane when the global side is 16-byte aligned.
__device__ __forceinline__ void tile_load(float *dst, const float *src, int n) { tile_load_f32<>(dst, src, n); }
// bf16 -> f32 staging, 8 requests in flight per thread before the LDS stores (see tile_load_f32)
__device__ __forceinline__ void tile_load(float *__restrict__ dst, const uint16_t *__restrict__ src, int n) {
  constexpr int kBatch = 8;
  const int nt = blockDim.x;
  if ((reinterpret_cast<uintptr_t>(src) & 7) == 0) {
    const int n4 = n >> 2;
    const uint2 *s4 = reinterpret_cast<const uint2 *>(src);
    for (int base = 0; base < n4; base += kBatch * nt) {
      uint2 r[kBatch];
#pragma unroll
      for (int k = 0; k < kBatch; ++k) r[k] = s4[min(base + k * nt + static_cast<int>(threadIdx.x), n4 - 1)];
#pragma unroll
      for (int k = 0; k < kBatch; ++k) {   // unguarded clamped stores: see tile_load_f32
        const int i = min(base + k * nt + static_cast<int>(threadIdx.x), n4 - 1);
        *reinterpret_cast<float4 *>(dst + 4 * i) =
            make_float4(__uint_as_float(r[k].x << 16), __uint_as_float(r[k].x & 0xffff0000u),
                        __uint_as_float(r[k].y << 16), __uint_as_float(r[k].y & 0xffff0000u));
      }
    }
    for (int i = (n4 << 2) + threadIdx.x; i < n; i += nt) dst[i] = ldf(src + i);
  } else {
    for (int i = threadIdx.x; i < n; i += nt) dst[i] = ldf(src + i);
  }
}
// LDS -> global, threads [t0, t0 + nt) of the workgroup (the others return at once).
__device__ __forceinline__ void tile_store(float *dst, const float *src, int n, int t0, int nt) {
  const int t = static_cast<int>(threadIdx.x) - t0;
  if (t < 0) return;
  if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
    const int n4 = n >> 2;
    float4 *d4 = reinterpret_cast<float4 *>(dst);
    const float4 *s4 = reinterpret_cast<const float4 *>(src);
    for (int i = t; i < n4; i += nt) st4_nt(reinterpret_cast<float *>(d4 + i), s4[i]);
    for (int i = (n4 << 2) + t; i < n; i += nt) dst[i] = src[i];
  } else {
    for (int i = t; i < n; i += nt) dst[i] = src[i];
  }
}
__device__ __forceinline__ uint32_t bf16_bits(float v) {
  __hip_bfloat16 h = __float2bfloat16(v);
  return *reinterpret_cast<uint16_t *>(&h);
}
// f32 -> bf16 (round to nearest even, as stf), four per 8-byte store from the first 8-byte
// boundary on (the head and tail one by one)
__device__ __forceinline__ void tile_store(uint16_t *dst, const float *src, int n, int t0, int nt) {
  const int t = static_cast<int>(threadIdx.x) - t0;
  if (t < 0) return;
  int h = static_cast<int>((8 - (reinterpret_cast<uintptr_t>(dst) & 7)) & 7) >> 1;   // elements to the boundary
  if (h > n) h = n;
  if (t < h) stf(dst + t, src[t]);
  const int n4 = (n - h) >> 2;
  uint2 *d4 = reinterpret_cast<uint2 *>(dst + h);
  for (int i = t; i < n4; i += nt) {
    const float *q = src + h + 4 * i;
    d4[i] = make_uint2(bf16_bits(q[0]) | (bf16_bits(q[1]) << 16), bf16_bits(q[2]) | (bf16_bits(q[3]) << 16));
  }
  for (int i = h + (n4 << 2) + t; i < n; i += nt) stf(dst + i, src[i]);
}

// Score tile split into issue (loads into registers) and commit (LDS stores), so a kernel can
// issue its per-row loads, then the tile's, then the loads that depend on the per-row values,
// with every request in flight together.  NB vector loads per thread cover the tile when
// n <= 4 * NB * blockDim; `fast_tile` says whether this tile qualifies (else tile_load).
template <typename T> struct TileVec;
template <> struct TileVec<float> { using V = float4; static constexpr int kAlign = 16; };
template <> struct TileVec<uint16_t> { using V = uint2; static constexpr int kAlign = 8; };

template <typename T, int NB>
__device__ __forceinline__ bool fast_tile(const T *src, int n) {
  return NB > 0 && (reinterpret_cast<uintptr_t>(src) & (TileVec<T>::kAlign - 1)) == 0 && (n & 3) == 0 &&
         n <= 4 * NB * static_cast<int>(blockDim.x);
}
template <typename T, int NB>
__device__ __forceinline__ void tile_issue(typename TileVec<T>::V (&r)[NB], const T *src, int n) {
  const auto *s4 = reinterpret_cast<const typename TileVec<T>::V *>(src);
  const int n4 = n >> 2;
#pragma unroll
  for (int k = 0; k < NB; ++k) r[k] = s4[min(k * static_cast<int>(blockDim.x) + static_cast<int>(threadIdx.x), n4 - 1)];
}
__device__ __forceinline__ float4 widen4(float4 v) { return v; }
__device__ __forceinline__ float4 widen4(uint2 v) {
  return make_float4(__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xffff0000u),
                     __uint_as_float(v.y << 16), __uint_as_float(v.y & 0xffff0000u));
}
template <typename V, int NB>
__device__ __forceinline__ void tile_commit(float *dst, const V (&r)[NB], int n) {
  const int n4 = n >> 2;
#pragma unroll
  for (int k = 0; k < NB; ++k)   // unguarded clamped stores (see tile_load_f32)
    reinterpret_cast<float4 *>(dst)[min(k * static_cast<int>(blockDim.x) + static_cast<int>(threadIdx.x), n4 - 1)] =
        widen4(r[k]);
}

struct OvOut {
  float v;
  float g[4];   // d v / d b1 (x1, y1, x2, y2)
  float g2[4];  // d v / d b2 (only with kG2)
};

// Row-wise IoU / GIoU / DIoU / CIoU of iou_utils.py:6-164 (forward in the reference's
// evaluation order) and the hand-derived reverse mode of the same graph (clamp masks inclusive,
// CIoU's alpha / arctan / w_temp treated as constants as under its torch.no_grad()).
template <bool kG2 = false>
__device__ OvOut aligned_overlap(int kind, Box4 p, Box4 t, bool want_grad) {
  const float x1 = p.a, y1 = p.b, x2 = p.c, y2 = p.d;
  const float X1 = t.a, Y1 = t.b, X2 = t.c, Y2 = t.d;
  const float w1 = x2 - x1, h1 = y2 - y1, w2 = X2 - X1, h2 = Y2 - Y1;
  const float a1 = w1 * h1, a2 = w2 * h2;
  const float ix2 = fminf(x2, X2), iy2 = fminf(y2, Y2), ix1 = fmaxf(x1, X1), iy1 = fmaxf(y1, Y1);
  const float iwr = ix2 - ix1, ihr = iy2 - iy1;
  const float iw = iwr < 0.f ? 0.f : iwr, ih = ihr < 0.f ? 0.f : ihr;
  const float ia = iw * ih;
  const float U = a1 + a2 - ia;
  const float iou = ia / U;
  float ow = 0.f, oh = 0.f, owr = 0.f, ohr = 0.f, ox2 = 0.f, oy2 = 0.f, ox1 = 0.f, oy1 = 0.f;
  if (kind != SBOD_OV_IOU) {
    ox2 = fmaxf(x2, X2);
    oy2 = fmaxf(y2, Y2);
    ox1 = fminf(x1, X1);
    oy1 = fminf(y1, Y1);
    owr = ox2 - ox1;
    ohr = oy2 - oy1;
    ow = owr < 0.f ? 0.f : owr;
    oh = ohr < 0.f ? 0.f : ohr;
  }
  float raw, lo = -1.f;
  // gradient seeds (for d raw)
  float g_ia = 0.f, g_U = 0.f, g_ow = 0.f, g_oh = 0.f, g_cx1 = 0.f, g_cy1 = 0.f, g_w1 = 0.f, g_h1 = 0.f;
  const float cx1 = (x2 + x1) / 2.f, cy1 = (y2 + y1) / 2.f;
  const float cx2 = (X2 + X1) / 2.f, cy2 = (Y2 + Y1) / 2.f;
  if (kind == SBOD_OV_IOU) {
    raw = iou;
    lo = 0.f;
    g_ia = 1.f / U;
    g_U = -iou / U;
  } else if (kind == SBOD_OV_GIOU) {
    const float C = ow * oh;
    raw = iou - (C - U) / C;
    g_ia = 1.f / U;
    g_U = -iou / U + 1.f / C;
    const float g_C = -U / (C * C);
    g_ow = g_C * oh;
    g_oh = g_C * ow;
  } else {
    const float dx = cx2 - cx1, dy = cy2 - cy1;
    const float idiag = dx * dx + dy * dy;
    const float odiag = ow * ow + oh * oh;
    const float u = idiag / odiag;
    float g_u = -1.f;
    if (kind == SBOD_OV_DIOU) {
      raw = iou - u;
    } else {  // CIoU (iou_utils.py:84-93)
      const float K4 = static_cast<float>(4.0 / (M_PI * M_PI));
      const float K8 = static_cast<float>(8.0 / (M_PI * M_PI));
      const float arct = atanf(w2 / h2) - atanf(w1 / h1);
      const float v = K4 * (arct * arct);
      const float S = 1.f - iou;
      const float alpha = v / (S + v);
      const float wt = 2.f * w1;
      const float m = w1 - wt;
      const float ar = (K8 * arct) * (m * h1);
      raw = iou - (u + alpha * ar);
      const float g_ar = -alpha;
      g_w1 += g_ar * (K8 * arct) * h1;  // through m = w1 - w_temp (w_temp constant)
      g_h1 += g_ar * (K8 * arct) * m;
    }
    g_ia = 1.f / U;
    g_U = -iou / U;
    const float g_idiag = g_u / odiag;
    const float g_odiag = -g_u * idiag / (odiag * odiag);
    g_cx1 = g_idiag * (-2.f * dx);
    g_cy1 = g_idiag * (-2.f * dy);
    g_ow = g_odiag * 2.f * ow;
    g_oh = g_odiag * 2.f * oh;
  }
  OvOut r;
  r.v = fminf(fmaxf(raw, lo), 1.f);
  r.g[0] = r.g[1] = r.g[2] = r.g[3] = 0.f;
  if constexpr (kG2) r.g2[0] = r.g2[1] = r.g2[2] = r.g2[3] = 0.f;
  if (!want_grad || !(raw >= lo && raw <= 1.f)) return r;
  // U = a1 + a2 - ia
  const float g_a1 = g_U;
  g_ia -= g_U;
  if constexpr (kG2) {
    // the second box set: the same graph through X1..Y2 (min / max ties split in half; CIoU's
    // alpha * ar term depends on b1 only, its arctan / alpha being constants)
    const float g_iwr2 = iwr >= 0.f ? g_ia * ih : 0.f;
    const float g_ihr2 = ihr >= 0.f ? g_ia * iw : 0.f;
    float gX1 = -g_iwr2 * dmax_a(X1, x1), gX2 = g_iwr2 * dmin_a(X2, x2);
    float gY1 = -g_ihr2 * dmax_a(Y1, y1), gY2 = g_ihr2 * dmin_a(Y2, y2);
    if (kind != SBOD_OV_IOU) {
      const float g_owr = owr >= 0.f ? g_ow : 0.f;
      const float g_ohr = ohr >= 0.f ? g_oh : 0.f;
      gX2 += g_owr * dmax_a(X2, x2);
      gX1 -= g_owr * dmin_a(X1, x1);
      gY2 += g_ohr * dmax_a(Y2, y2);
      gY1 -= g_ohr * dmin_a(Y1, y1);
    }
    // centre distance: dx = cx2 - cx1, so d/dcx2 = -d/dcx1
    const float g_w2 = g_U * h2, g_h2 = g_U * w2;   // a2 = w2 * h2 (U = a1 + a2 - ia)
    gX1 += -0.5f * g_cx1 - g_w2;
    gX2 += -0.5f * g_cx1 + g_w2;
    gY1 += -0.5f * g_cy1 - g_h2;
    gY2 += -0.5f * g_cy1 + g_h2;
    r.g2[0] = gX1;
    r.g2[1] = gY1;
    r.g2[2] = gX2;
    r.g2[3] = gY2;
  }
  g_w1 += g_a1 * h1;
  g_h1 += g_a1 * w1;
  const float g_iwr = iwr >= 0.f ? g_ia * ih : 0.f;
  const float g_ihr = ihr >= 0.f ? g_ia * iw : 0.f;
  float gx1 = -g_iwr * dmax_a(x1, X1), gx2 = g_iwr * dmin_a(x2, X2);
  float gy1 = -g_ihr * dmax_a(y1, Y1), gy2 = g_ihr * dmin_a(y2, Y2);
  if (kind != SBOD_OV_IOU) {
    const float g_owr = owr >= 0.f ? g_ow : 0.f;
    const float g_ohr = ohr >= 0.f ? g_oh : 0.f;
    gx2 += g_owr * dmax_a(x2, X2);
    gx1 -= g_owr * dmin_a(x1, X1);
    gy2 += g_ohr * dmax_a(y2, Y2);
    gy1 -= g_ohr * dmin_a(y1, Y1);
  }
  gx1 += 0.5f * g_cx1 - g_w1;
  gx2 += 0.5f * g_cx1 + g_w1;
  gy1 += 0.5f * g_cy1 - g_h1;
  gy2 += 0.5f * g_cy1 + g_h1;
  r.g[0] = gx1;
  r.g[1] = gy1;
  r.g[2] = gx2;
  r.g[3] = gy2;
  return r;
}

// d/d(gcxgcy) of cxcy_to_xy(gcxgcy_to_cxcy(g, prior)) given d/d(x1,y1,x2,y2).
__device__ __forceinline__ void decode_backward(const float gb[4], Box4 g, Box4 pr, float out[4]) {
  const float w = expf(g.c / 5.f) * pr.c, h = expf(g.d / 5.f) * pr.d;
  const float gcx = gb[0] + gb[2], gcy = gb[1] + gb[3];
  const float gw = 0.5f * (gb[2] - gb[0]), gh = 0.5f * (gb[3] - gb[1]);
  out[0] = gcx * pr.c / 10.f;
  out[1] = gcy * pr.d / 10.f;
  out[2] = gw * w / 5.f;
  out[3] = gh * h / 5.f;
}

__device__ __forceinline__ float powg(float x, float gamma) {
  return gamma == 2.f ? x * x : powf(x, gamma);
}
__device__ __forceinline__ float powg1(float x, float gamma) {  // x^(gamma-1)
  return gamma == 2.f ? x : powf(x, gamma - 1.f);
}

// Softmax-focal of one row (Loss.py:9-38): q = p_t; background rows weighted by p_bg (sic).
// e[] holds exp(z - max) on entry; writes d loss / d z (times scale) into e[] when grad.
// Returns the row loss (NaN when any class probability is exactly 0, as 0 * log 0 in the
// reference).
__device__ __forceinline__ float focal_row(float *e, int C, int t, float s, float afg, float abg,
                                           float gamma, float scale, bool grad) {
  const float inv = 1.f / s;
  float pmin = 1.f;
  for (int c = 0; c < C; ++c) pmin = fminf(pmin, e[c] * inv);
  const float q = e[t] * inv;
  const float lq = logf(q);
  float loss, dq;
  if (t == 0) {  // alpha_bg * p0^gamma * (-log p0)
    loss = abg * powg(q, gamma) * -lq;
    dq = abg * (gamma * powg1(q, gamma) * -lq - powg1(q, gamma));
  } else {       // alpha_fg * (1 - p_t)^gamma * (-log p_t)
    const float om = 1.f - q;
    loss = afg * powg(om, gamma) * -lq;
    dq = afg * (-gamma * powg1(om, gamma) * -lq - powg(om, gamma) / q);
  }
  if (!(pmin > 0.f)) loss = __builtin_nanf("");
  if (grad) {
    const float k = dq * q * scale;
    for (int c = 0; c < C; ++c) {
      const float pc = e[c] * inv;
      e[c] = loss != loss ? loss : k * ((c == t ? 1.f : 0.f) - pc);
    }
  }
  return loss;
}

struct LossArgs {
  int B, P, C;
  const float *priors, *arm_locs, *arm_scores, *gt;
  const int64_t *labels;
  const int32_t *off, *obj, *npos_total;
  const float *ovl;
  float thr, nthr, theta;
  int reg, cls, flags;
  float reg_weight, afg, abg, gamma;
  float *partials, *pool;
  SpanRing *span;             // KernelTimer span ring under graph capture, else null
  // fused finish (no mining pass): fixed-point sums {conf, loc}, non-finite flags and the
  // arrival counter of the workgroups; null: partials for k_loss_final
  unsigned long long *fin;
  float *out;                 // the loss vector {total, conf, loc, n_pos} (fused finish)
  // one-launch criterion (k_multibox<..., true>): the matcher's in-launch state and outputs
  const float *anchors;       // priors_xy [P,4]
  int Gmax;
  int32_t *obj_out, *npos_out;   // [B,P] object per prior, [B+1] positives per image and total
  float *ovl_out;             // [B,P] overlap per prior
  unsigned long long *keys;   // [B][kKeyShards][Gmax] best-prior keys, zero on entry
  unsigned long long *arrive; // [B] (tiles arrived << 32) | their phase-1 positives, zero on entry
  unsigned long long *done;   // (images finished << 32) | their positives, zero on entry
  unsigned *status;           // nonzero: a wait gave up (see kSpinLimit)
  unsigned long long *forced; // [B][Gmax] (prior << 32 | object) rewritten by the forced match
  int32_t *nforced;           // [B]
  void *recs;                 // fused finish: [nblk] 16-byte records {conf, tag, loc, tag}
  int rows = kLTile;          // rows (priors) per k_multibox tile (mb_rows; the one-launch form: kLTile)
};

// The fused finish of k_multibox (focal / no mining).  Each workgroup folds its partial sums
// into exact 128-bit fixed-point accumulators (two's complement, 64 fraction bits: value * 2^64
// as {lo, hi} u64 words) with agent-scope atomics executed at the memory side: the lo add
// returns the word's previous value, so the adder knows its own carry out of bit 63 and adds it
// to hi with the high part.  Integer adds are exact and order-free, so the sum is bitwise
// reproducible, with a resolution of 2^-64 per partial (a loss total of 1e-12 keeps 1e-7
// relative) and a range of 2^63.  A partial of magnitude >= 2^40 (or a non-finite one) cannot be
// folded exactly: it travels as a flag bit, and the finishing workgroup then sums every
// workgroup's fp32 partial in double instead (each workgroup also writes its two partials
// through with sc1 stores before it counts itself in), as k_loss_final would — the finish is
// never silently wrong (a NaN row of the focal loss, the reference's 0 * log 0, makes a NaN loss
// that way).  The adds are drained (s_waitcnt with a compiler memory clobber) before the arrival
// add, and every hand-off moves through memory-side atomics or sc1 stores/loads, so no cache
// write-back or invalidation is needed between the XCDs.
constexpr float kFinLimit = 1099511627776.f;   // 2^40: larger partials take the double fallback
struct Fx128 {
  unsigned long long lo, hi;
};
// v * 2^64 rounded to an integer (|v| < 2^40, finite), as a 128-bit two's complement pair.
__device__ __forceinline__ Fx128 to_fx128(float v) {
  const uint32_t bits = __float_as_uint(v) & 0x7fffffffu;
  const uint32_t E = bits >> 23;
  const unsigned long long m = E ? ((bits & 0x7fffffu) | 0x800000u) : (bits & 0x7fffffu);
  const int sh = (E ? static_cast<int>(E) - 150 : -149) + 64;   // |v| * 2^64 = m * 2^sh
  unsigned long long lo = 0, hi = 0;
  if (sh >= 64) {
    hi = m << (sh - 64);
  } else if (sh >= 0) {
    lo = m << sh;
    hi = sh > 40 ? (m >> (64 - sh)) : 0ull;
  } else if (sh > -25) {
    lo = (m + (1ull << (-sh - 1))) >> (-sh);   // round half up
  }
  if (__float_as_uint(v) >> 31) {   // negate the pair
    lo = ~lo + 1ull;
    hi = ~hi + (lo == 0ull ? 1ull : 0ull);
  }
  return Fx128{lo, hi};
}
__device__ __forceinline__ double fx128_value(unsigned long long lo, unsigned long long hi) {
  return static_cast<double>(static_cast<long long>(hi)) + static_cast<double>(lo) * 5.421010862427522170e-20;
}
__device__ __forceinline__ bool fx_foldable(float v) { return fabsf(v) < kFinLimit; }   // false for NaN / inf
__device__ __forceinline__ void loss_outputs(double c, double l, float n, int reg, int cls, int flags,
                                             float reg_weight, float *out) {
  const float conf = (cls == SBOD_CLS_CE || (flags & SBOD_LOSS_FOCAL_NORM)) ? static_cast<float>(c) / n
                                                                            : static_cast<float>(c);
  const float loc = reg == SBOD_REG_L1 ? static_cast<float>(l) / (4.f * n) : static_cast<float>(l) / n;
  out[0] = conf + reg_weight * loc;
  out[1] = conf;
  out[2] = loc;
  out[3] = n;
}
constexpr int kFinGroups = 32;   // workgroup groups (linear id mod 32), then one global level
constexpr int kFinStride = 16;   // u64 words per accumulator set: one 128-byte line each
constexpr size_t kFinBytes = sizeof(unsigned long long) * kFinStride * (kFinGroups + 1);   // 4224
// Accumulator set (one 128-byte line): conf {lo, hi}, loc {lo, hi}, fallback flag, arrivals.
enum { kFinConf = 0, kFinLoc = 2, kFinFlag = 4, kFinArrive = 5 };
// w[0..1] += v (128-bit): the lo add returns the previous word, which gives this add's carry.
__device__ __forceinline__ void fx_add(unsigned long long *w, Fx128 v) {
  unsigned long long carry = 0;
  if (v.lo) {
    const unsigned long long old = __hip_atomic_fetch_add(w, v.lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    carry = old + v.lo < old ? 1ull : 0ull;
  }
  if (v.hi + carry) __hip_atomic_fetch_add(w + 1, v.hi + carry, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long xchg0(unsigned long long *w) {
  return __hip_atomic_exchange(w, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ Fx128 fx128_add(Fx128 x, Fx128 y) {
  const unsigned long long lo = x.lo + y.lo;
  return Fx128{lo, x.hi + y.hi + (lo < x.lo ? 1ull : 0ull)};
}
// exp on the hardware exp2 unit (~1-2 ulp + 2^-24 relative argument rounding): the losses'
// budget is 1e-4 relative; the all-classes underflow test (p == 0 -> NaN) stays exact (below).
__device__ __forceinline__ float fast_exp(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }

// Two block-wide sums with one pair of barriers (blockDim.x a multiple of 64, <= 1024); results
// valid in every thread.
__device__ __forceinline__ void block_sum2(float &x, float &y, float *scratch /* >= 32 */) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    x += __shfl_xor(x, m, kWave);
    y += __shfl_xor(y, m, kWave);
  }
  __syncthreads();
  if (lane == 0) {
    scratch[w] = x;
    scratch[16 + w] = y;
  }
  __syncthreads();
  float sx = 0.f, sy = 0.f;
  for (int i = 0; i < nw; ++i) {
    sx += scratch[i];
    sy += scratch[16 + i];
  }
  x = sx;
  y = sy;
}

// The fused finish of k_multibox (focal criteria, no mining pass): no counters.  Every
// workgroup publishes its fp32 partials as ONE 16-byte write-through record {conf, tag, loc, tag}
// — two 8-byte granules {value, tag}, each validating itself (MI355X_MICROARCH.md inter-workgroup
// visibility, the data-is-the-flag form) — and retires; the grid's last workgroup (linear id
// nblk - 1: dispatched last, so every other workgroup is already resident or done, and it is the
// only one that waits: no co-residency assumption, nothing can starve it) stores its own tile,
// then sweeps every record with 16-byte sc1 loads until each carries this call's tag, folding each
// the first time it is seen, EXACTLY: each fp32 partial as a 128-bit fixed-point integer (value *
// 2^64, two's complement), integer adds — the total is the same in any order, bitwise
// reproducible, with a resolution of 2^-64 per partial (a loss total of 1e-12 keeps 1e-7
// relative).  A partial of magnitude >= 2^40 or a non-finite one cannot be folded exactly: then
// the double sum of all partials in record order (a second, ordered pass) is the result, as
// k_loss_final computes it — never silently wrong (a NaN row of the focal loss, the reference's
// 0 * log 0, makes a NaN loss that way).
// Tags: a record slot is zero on entry (sbod_loss_zero_bytes: the records are the zero-on-entry
// prefix) and holds tag 1 once written; the finisher zeroes every slot after folding it, so the
// workspace is left as it was found (any later call, any shape).  The finisher's wait is bounded
// (kGatherTicks of the 100 MHz clock): a timeout — a hardware fault, never a schedule — makes
// this and every later call's loss NaN (a sticky word, cleared only by the zeroing memset), since
// a record landing after it would look like a later call's.
// Critical path after the last record is issued: its write landing + one sweep + the fold.
// (Rounds 4-5a counted arrivals on 32 group counters and a top counter: a drain, two dependent
// far-memory atomics and the partials read after the last tile, 3.6-4.5 us of an 18 us launch,
// scripts/mb_imbalance.py.)
constexpr int kFinSticky = kFinStride * kFinGroups + 9;   // u64 word index in the fin region
constexpr unsigned long long kGatherTicks = 200000000ull;   // 2 s
constexpr unsigned kRecTag = 1u;
// One lane: the workgroup's record, written through.
__device__ __forceinline__ void loss_publish(const LossArgs &a, float conf_l, float loc_l, unsigned tag, unsigned nblk,
                                             unsigned blk) {
  const u32x4_t v = {__float_as_uint(conf_l), tag, __float_as_uint(loc_l), tag};
  st_wt_b128(a.recs, nblk * 16u, blk * 16u, v);
}
// The whole workgroup (the finisher): every record of this call, folded exactly, then zeroed;
// thread 0 writes the loss.
__device__ void loss_gather(const LossArgs &a, unsigned nblk, unsigned tag, float n, float *out,
                            unsigned long long *s_fx, double *s_red) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(a.recs, static_cast<short>(0), static_cast<int>(nblk * 16u),
                                                    0x00020000);
  constexpr int kB = 8;   // records per thread per sweep: 2,048 workgroups in one batch
  const unsigned nk = (nblk + kLTile - 1u) / kLTile;
  Fx128 fc{0ull, 0ull}, fl{0ull, 0ull};
  bool ok = true, late = false;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  if (tid == 0) FIN_MARK(0, t0);
  unsigned sweeps = 0;
  for (unsigned k0 = 0; k0 < nk && !late; k0 += kB) {
    unsigned pend = 0;
#pragma unroll
    for (int k = 0; k < kB; ++k)
      if ((k0 + k) * kLTile + tid < nblk) pend |= 1u << k;
    while (pend != 0u) {
      u32x4_t w[kB];
#pragma unroll
      for (int k = 0; k < kB; ++k)   // past the last record: zero through the range check
        w[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>(((k0 + k) * kLTile + tid) * 16u), 0, kCpolSc1);
#pragma unroll
      for (int k = 0; k < kB; ++k) {
        if (((pend >> k) & 1u) && w[k][1] == tag && w[k][3] == tag) {
          const float c = __uint_as_float(w[k][0]), l = __uint_as_float(w[k][2]);
          const bool f = fx_foldable(c) && fx_foldable(l);
          ok = ok && f;
          fc = fx128_add(fc, to_fx128(f ? c : 0.f));
          fl = fx128_add(fl, to_fx128(f ? l : 0.f));
          pend &= ~(1u << k);
          FIN_SEEN((k0 + k) * kLTile + tid);
        }
      }
      ++sweeps;
      if (tid == 0 && sweeps == 1) FIN_MARK(1, __builtin_amdgcn_s_memrealtime());
      if (pend != 0u) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > kGatherTicks) {
          late = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    fc = fx128_add(fc, Fx128{shfl_xor_u64(fc.lo, m), shfl_xor_u64(fc.hi, m)});
    fl = fx128_add(fl, Fx128{shfl_xor_u64(fl.lo, m), shfl_xor_u64(fl.hi, m)});
  }
  const bool wave_ok = __ballot(!ok) == 0ull, wave_late = __ballot(late) != 0ull;
  if (lane == 0) {
    s_fx[5 * wv + 0] = fc.lo;
    s_fx[5 * wv + 1] = fc.hi;
    s_fx[5 * wv + 2] = fl.lo;
    s_fx[5 * wv + 3] = fl.hi;
    s_fx[5 * wv + 4] = (wave_ok ? 1ull : 0ull) | (wave_late ? 2ull : 0ull);
  }
  __syncthreads();
  if (tid == 0) {
    FIN_MARK(2, __builtin_amdgcn_s_memrealtime());
    FIN_MARK(4, sweeps);
  }
  bool all_ok = true, any_late = false;
  fc = Fx128{0ull, 0ull};
  fl = Fx128{0ull, 0ull};
  for (int w2 = 0; w2 < kLTile / 64; ++w2) {
    fc = fx128_add(fc, Fx128{s_fx[5 * w2 + 0], s_fx[5 * w2 + 1]});
    fl = fx128_add(fl, Fx128{s_fx[5 * w2 + 2], s_fx[5 * w2 + 3]});
    all_ok = all_ok && (s_fx[5 * w2 + 4] & 1ull) != 0ull;
    any_late = any_late || (s_fx[5 * w2 + 4] & 2ull) != 0ull;
  }
  double c = fx128_value(fc.lo, fc.hi), l = fx128_value(fl.lo, fl.hi);
  if (!all_ok && !any_late) {
    // a non-finite or huge partial: the double sum of every workgroup's fp32 partials in record
    // order (thread-strided, then the block tree: the same order every call)
    c = 0.0;
    l = 0.0;
    for (unsigned i = tid; i < nblk; i += kLTile) {
      const u32x4_t w = __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>(i * 16u), 0, kCpolSc1);
      c += static_cast<double>(__uint_as_float(w[0]));
      l += static_cast<double>(__uint_as_float(w[2]));
    }
    __syncthreads();
    c = block_sum(c, s_red);
    __syncthreads();
    l = block_sum(l, s_red);
  }
  if (!any_late)   // every slot back to zero (every one was seen: no writer is left)
    for (unsigned i = tid; i < nblk; i += kLTile) reinterpret_cast<u32x4_t *>(a.recs)[i] = u32x4_t{0u, 0u, 0u, 0u};
  if (tid == 0) {
    unsigned long long *fin = a.fin;
    if (any_late) st_wt_u64(fin + kFinSticky, 1ull);
    if (any_late || ld_wt_u64(fin + kFinSticky) != 0ull) c = l = __builtin_nan("");
    loss_outputs(c, l, n, a.reg, a.cls, a.flags, a.reg_weight, out);
    FIN_MARK(3, __builtin_amdgcn_s_memrealtime());
  }
}

#ifdef SBOD_VARIANT_ONE_LAUNCH
// Called by wave 0 of every workgroup (all 64 lanes; conf_l / loc_l uniform).  The partials
// array holds each workgroup's fp32 {conf, loc} for the double fallback.
// fxc / fxl (k_multibox_tiles): the exact sums of the workgroup's per-tile partials, already in
// fixed point (fx_ok: every partial foldable); conf_l / loc_l are then only the fallback's values.
__device__ void multibox_finish(const LossArgs &a, float conf_l, float loc_l, unsigned nblk, float n, float *out,
                                const Fx128 *fxc = nullptr, const Fx128 *fxl = nullptr, bool fx_ok = true) {
  // accumulators: kFinGroups group lines, then the top line.  Two levels because atomics on one
  // word serialise at the memory side (~10 ns each): ~41 arrivals per group word and 32 on the
  // top word instead of every workgroup on one word.
  const int lane = threadIdx.x & 63;
  const unsigned blk = blockIdx.x + gridDim.x * blockIdx.y;
  const unsigned ng = nblk < kFinGroups ? nblk : kFinGroups, g = blk % ng;
  const unsigned in_group = (nblk - g + ng - 1) / ng;
  unsigned long long *acc = a.fin + kFinStride * g, *top = a.fin + kFinStride * kFinGroups;
  int last = 0;
  if (lane == 0) {
    const bool ok = fxc ? fx_ok : (fx_foldable(conf_l) && fx_foldable(loc_l));
    st_wt_u32(reinterpret_cast<int32_t *>(a.partials) + 2 * blk, __float_as_uint(conf_l));
    st_wt_u32(reinterpret_cast<int32_t *>(a.partials) + 2 * blk + 1, __float_as_uint(loc_l));
    if (ok) {
      fx_add(acc + kFinConf, fxc ? *fxc : to_fx128(conf_l));
      fx_add(acc + kFinLoc, fxl ? *fxl : to_fx128(loc_l));
    } else {
      __hip_atomic_fetch_or(acc + kFinFlag, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    drain_vm();   // the adds (and the partials' write-through) are performed before the count
    last = __hip_atomic_fetch_add(acc + kFinArrive, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == in_group - 1;
  }
  if (!__builtin_amdgcn_readfirstlane(last)) return;
  // this group is complete (every member's adds were performed before it counted itself in):
  // its totals move to the top line (exchanges in flight together, leaving the group line zero),
  // and the workgroup that completes the top line drains it.  (Draining all 32 group lines from
  // the last workgroup instead serialised one lane's exchanges: +9 µs.)
  if (lane == 0) {
    const Fx128 c{xchg0(acc + kFinConf), xchg0(acc + kFinConf + 1)};
    const Fx128 l{xchg0(acc + kFinLoc), xchg0(acc + kFinLoc + 1)};
    const unsigned long long f = xchg0(acc + kFinFlag);
    xchg0(acc + kFinArrive);
    fx_add(top + kFinConf, c);
    fx_add(top + kFinLoc, l);
    if (f) __hip_atomic_fetch_or(top + kFinFlag, f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    drain_vm();
    last = __hip_atomic_fetch_add(top + kFinArrive, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ng - 1;
  }
  if (!__builtin_amdgcn_readfirstlane(last)) return;
  double c = 0.0, l = 0.0;
  int fallback = 0;
  if (lane == 0) {
    const unsigned long long clo = xchg0(top + kFinConf), chi = xchg0(top + kFinConf + 1);
    const unsigned long long llo = xchg0(top + kFinLoc), lhi = xchg0(top + kFinLoc + 1);
    fallback = xchg0(top + kFinFlag) != 0ull;
    xchg0(top + kFinArrive);
    c = fx128_value(clo, chi);
    l = fx128_value(llo, lhi);
  }
  if (__builtin_amdgcn_readfirstlane(fallback)) {
    // a non-finite or huge partial: the double sum of every workgroup's fp32 partials, as
    // k_loss_final computes it (the partials were written through before their arrivals)
    c = 0.0;
    l = 0.0;
    const int32_t *pp = reinterpret_cast<const int32_t *>(a.partials);
    for (unsigned i = lane; i < nblk; i += 64) {
      c += static_cast<double>(__uint_as_float(ld_wt_u32(pp + 2 * i)));
      l += static_cast<double>(__uint_as_float(ld_wt_u32(pp + 2 * i + 1)));
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
      c += __shfl_xor(c, m, 64);
      l += __shfl_xor(l, m, 64);
    }
  }
  if (lane == 0) {
    loss_outputs(c, l, n, a.reg, a.cls, a.flags, a.reg_weight, out);
    if (a.done != nullptr) {   // one-launch criterion: every workgroup has passed its wait
      a.npos_out[a.B] = static_cast<int32_t>(n);
      // the wait-timeout word is cleared here with `done` (zero on entry for the next call); its
      // value moves to the sticky diagnostics word after it (sbod_criterion_status)
      const unsigned st = __hip_atomic_exchange(a.status, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (st != 0u) {
        out[0] = out[1] = out[2] = __builtin_nanf("");
        __hip_atomic_fetch_or(a.status + 1, st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __hip_atomic_store(a.done, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// One-launch criterion: every workgroup waits until all images' forced matches are counted in
// (their positives are the gradients' normaliser).  The grid is co-resident (the host checks it
// against the occupancy query before choosing this form), so the wait ends within microseconds;
// a bound on it keeps a broken launch from hanging the device: past kSpinLimit ticks of the
// 100 MHz real-time clock the workgroup sets *status and goes on (the loss becomes NaN).
constexpr unsigned long long kSpinLimit = 2000000ull;   // 20 ms
__device__ __forceinline__ unsigned wait_all_images(unsigned long long *done, int B, unsigned *status,
                                                    int *timed_out) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  *timed_out = 0;
  for (;;) {
    const unsigned long long v = ld_wt_u64(done);
    if ((v >> 32) >= static_cast<unsigned long long>(B)) return static_cast<unsigned>(v);
    if (__builtin_amdgcn_s_memrealtime() - t0 > kSpinLimit) {
      __hip_atomic_fetch_or(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *timed_out = 1;
      return static_cast<unsigned>(v);
    }
    __builtin_amdgcn_s_sleep(1);
  }
}
#endif  // SBOD_VARIANT_ONE_LAUNCH

// The box-regression inputs of a row that can be positive (IoU >= threshold: every positive is,
// the forced matches included, since the matcher wrote 1.0 for them): its loc, prior, matched GT
// box and (RefineDet ODM) ARM loc, loaded together with the row's label — in the same memory
// round trip as the score tile, instead of a second one after the class decision.  Every load is
// unconditional (a conditional one makes the wait-count insertion at the join wait for the whole
// batch); a row that cannot be positive loads a dummy line shared by the workgroup (its prior's
// first row: L2-resident, one request per wave).
struct RegIn {
  Box4 l, pc, t, arm;
};
template <typename T, int CLS>
__device__ __forceinline__ RegIn reg_prefetch(const LossArgs &a, const T *__restrict__ locs, int p0, int row,
                                              int64_t i, int objv, int offb, bool cand) {
  const float *dummy = a.priors + 4 * static_cast<int64_t>(p0);
  RegIn r;
  if constexpr (sizeof(T) == 4) {
    r.l = ld4(cand ? reinterpret_cast<const float *>(locs) + 4 * i : dummy);
  } else {
    const uint2 u = *reinterpret_cast<const uint2 *>(cand ? reinterpret_cast<const void *>(locs + 4 * i)
                                                          : reinterpret_cast<const void *>(dummy));
    const float4 w = widen4(u);
    r.l = Box4{w.x, w.y, w.z, w.w};
  }
  r.pc = ld4(cand ? a.priors + 4 * static_cast<int64_t>(p0 + row) : dummy);
  r.t = ld4(cand ? a.gt + 4 * static_cast<int64_t>(offb + objv) : dummy);
  if constexpr (CLS == SBOD_CLS_CE)   // RefineDet's ODM (CE criteria only): the ARM box the target is encoded on
    r.arm = ld4(cand && (a.flags & SBOD_MATCH_ODM) ? a.arm_locs + 4 * i : dummy);
  else
    r.arm = Box4{0.f, 0.f, 0.f, 0.f};
  return r;
}

// The tile's rows after their matcher outputs are known: the class decision, the box regression
// of the positives and the classification (loss + gradient row into the LDS tile).  Shared by
// k_multibox (one tile per workgroup) and the A/B variants.  Every thread of the workgroup calls
// it (one barrier inside); conf_l / loc_l accumulate.  before_cls() runs after the last global
// load of the rows and before the classification (LDS and ALU only): k_multibox_tiles issues the
// next tile's loads there, so that no wait for this tile's loads (the wait counter is in order)
// also waits for them.
struct NoPrefetch {
  __device__ void operator()() const {}
};
// CE > 0: rows of exactly CE classes (CE <= CM; VOC's 21): the per-slot loops run over CE slots,
// with no padding slots to compute or guard — the same values as the CM-slot form (a padding
// slot only ever adds exp(-inf) = 0 or an ignored value).
template <typename T, int CM, int CLS, int CE = 0, typename Pf = NoPrefetch>
__device__ __forceinline__ void multibox_rows(const LossArgs &a, T *__restrict__ glocs, T *__restrict__ gsc,
                                              bool valid, int64_t ic, float v, int64_t labg, const RegIn &rg,
                                              float n, float *s_sc, float &conf_l, float &loc_l,
                                              Pf before_cls = Pf()) {
  const int tid = threadIdx.x;
  const int C = a.C;
  const bool odm = (a.flags & SBOD_MATCH_ODM) != 0;
  const bool grad = gsc != nullptr;
  int c = 0;
  bool negrow = false, easy = false, pos = false;
  if (valid) {
    c = v < a.thr ? 0 : static_cast<int>(labg);
    if (a.flags & SBOD_MATCH_BINARY) c = c > 0 ? 1 : 0;
    negrow = v < a.nthr;
    if (odm) {  // RefineDet512.py:894-899
      const float z0 = a.arm_scores[2 * ic], z1 = a.arm_scores[2 * ic + 1];
      const float m = fmaxf(z0, z1);
      const float e0 = expf(z0 - m), e1 = expf(z1 - m);
      easy = e1 / (e0 + e1) < a.theta;
    }
    pos = c > 0 && !easy;
  }
  // ---------------- box regression of the positive rows (~1-3 % of them) on the lanes that hold
  // them, from the registers reg_prefetch filled with the tile's loads; a wave without a positive
  // row skips the DIoU / encode path (a dozen IEEE divisions, exps) as a whole.  (Packing the
  // tile's positives onto one wave re-read their rows after a barrier: a second memory round trip,
  // +2 us on the ~20 % of workgroups with a positive, scripts/mb_imbalance.py.)
  float gl[4] = {0.f, 0.f, 0.f, 0.f};
  if (__ballot(pos)) {
    if (pos) {
      const Box4 l = rg.l, pc = rg.pc, t = rg.t;
      if (a.reg == SBOD_REG_DIOU) {  // SSD512.py:579-581: IouLoss(Diou) on decoded boxes
        const Box4 d = decode_tenfive_xy(l, pc);
        const OvOut r = aligned_overlap(SBOD_OV_DIOU, d, t, grad);
        loc_l += 1.f - r.v;
        if (grad) {
          const float s = -a.reg_weight / n;
          const float gb[4] = {r.g[0] * s, r.g[1] * s, r.g[2] * s, r.g[3] * s};
          decode_backward(gb, l, pc, gl);
        }
      } else {  // smooth-L1 (Loss.py:213-217) or L1 on encoded targets
        const Box4 pr = odm ? xy_to_cxcy(decode_tenfive_xy(rg.arm, pc)) : pc;
        const Box4 en = encode_tenfive(xy_to_cxcy(t), pr);
        const float lv[4] = {l.a, l.b, l.c, l.d}, ev[4] = {en.a, en.b, en.c, en.d};
        const bool l1 = a.reg == SBOD_REG_L1;
        const float beta = 1.f / 9.f;
        const float s = l1 ? a.reg_weight / (4.f * n) : a.reg_weight / n;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float d = lv[k] - ev[k];
          const float x = fabsf(d);
          const float sg = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
          if (l1) {
            loc_l += x;
            gl[k] = sg * s;
          } else if (x >= beta) {
            loc_l += x - kHalfBetaDefault;
            gl[k] = sg * s;
          } else {
            loc_l += 0.5f * (x * x) / beta;
            gl[k] = (x / beta) * sg * s;
          }
        }
      }
    }
  }
  MB_MARK(2, tid == 0);
  // LDS-DMA tile (fp32 fast path): a wave's DMA chunks are read by OTHER waves' rows, and on
  // gfx950 neither s_barrier nor the workgroup release fence waits for vmcnt — so every wave
  // waits for its own DMA explicitly before the barrier (a wave whose rows are all
  // invalid, e.g. SSD300's 28-row last tile, has no later use that would wait for it)
  drain_vm();
  __syncthreads();   // the score tile is in LDS (every thread committed its part)
  MB_MARK(1, tid == 0);
  before_cls();
  if (valid) {
    const int64_t i = ic;
    if (glocs) {   // the row's box gradient (zero unless positive)
      if constexpr (sizeof(T) == 4) {
        st4_nt(reinterpret_cast<float *>(glocs) + 4 * i, Box4{gl[0], gl[1], gl[2], gl[3]});
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) stf(glocs + 4 * i + k, gl[k]);
      }
    }
    // ---------------- classification
    float *row = s_sc + tid * C;
    if constexpr (CM > 0) {
      constexpr int KN = CE > 0 ? CE : CM;   // slots walked
      float r[CM];
      float m = -__builtin_inff(), zmin = __builtin_inff();
      // constant-offset reads (no per-slot index arithmetic; a short last row reads into the 8
      // padding floats after the tile); only the top 8 slots can be padding (C > CM - 8)
      auto in_row = [&](int k) { return CE > 0 || k < CM - 8 || k < C; };
#pragma unroll
      for (int k = 0; k < KN; ++k) {
        const float x = row[k];
        r[k] = in_row(k) ? x : -__builtin_inff();
        m = fmaxf(m, r[k]);                       // a NaN logit gives a NaN loss either way
        // (only the top 8 slots can be padding: the others take one v_min instead of a compare
        // and a select — same minimum; a NaN logit is skipped either way)
        if (CE > 0 || k < CM - 8)
          zmin = fminf(zmin, r[k]);
        else
          zmin = (in_row(k) && r[k] < zmin) ? r[k] : zmin;
      }
      const float zt = row[c];
      float s = 0.f;
      // focal: the exponentials stay in registers for the gradient (computed once), packed
      // fp32 for the elementwise steps — this pass is VALU-issue-bound (a v_exp costs 8 cycles
      // of a wave's issue, a plain or packed op 4), every wave of the round computing at once
      typedef float f2 __attribute__((ext_vector_type(2)));
      if constexpr (CLS == SBOD_CLS_FOCAL) {
        // the exponentials replace the logits in the LDS row (the gradient pass reads them back:
        // LDS operations instead of a second v_exp per class, and no register array live across
        // the loss math's powf / logf)
        const f2 nm2 = {-m, -m}, l2 = {1.4426950408889634f, 1.4426950408889634f};
        f2 acc2 = {0.f, 0.f};
#pragma unroll
        for (int k = 0; k + 1 < KN; k += 2) {   // CM is a multiple of 8
          const f2 t = (f2{r[k], r[k + 1]} + nm2) * l2;
          const f2 ex = {__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};   // padding: 0
          acc2 += ex;
          if (in_row(k)) row[k] = ex.x;
          if (in_row(k + 1)) row[k + 1] = ex.y;
        }
        if constexpr (KN % 2 == 1) {   // the last (even) slot: the x lane of its pair
          const float ex = __builtin_amdgcn_exp2f((r[KN - 1] + nm2.x) * l2.x);
          acc2.x += ex;
          row[KN - 1] = ex;
        }
        s = acc2.x + acc2.y;
      } else {
        // CE feeds the hard-negative selection (a ranking): the accurate exp keeps its values
        // within an ulp of the reference's so near-ties at the top-k boundary do not move
#pragma unroll
        for (int k = 0; k < KN; ++k) s += expf(r[k] - m);
      }
      const float inv = 1.f / s;
      if constexpr (CLS == SBOD_CLS_FOCAL) {
        if (pos || negrow) {  // SSD512.py:588-593: rows = positives ++ negatives(IoU < thr - 0.1)
          const float scale = (a.flags & SBOD_LOSS_FOCAL_NORM) ? 1.f / n : 1.f;
          // Loss.py:9-38: q = p_t; background rows weighted by p_bg (sic)
          const float q = fast_exp(zt - m) * inv;
          const float lq = logf(q);
          float loss, dq;
          if (c == 0) {  // alpha_bg * p0^gamma * (-log p0)
            loss = a.abg * powg(q, a.gamma) * -lq;
            dq = a.abg * (a.gamma * powg1(q, a.gamma) * -lq - powg1(q, a.gamma));
          } else {       // alpha_fg * (1 - p_t)^gamma * (-log p_t)
            const float om = 1.f - q;
            loss = a.afg * powg(om, a.gamma) * -lq;
            dq = a.afg * (-a.gamma * powg1(om, a.gamma) * -lq - powg(om, a.gamma) / q);
          }
          // 0 * log 0 in the reference when any class probability is exactly 0: decided on the
          // smallest logit with the accurate exp (underflow is monotone in the logit).  Above
          // -80 no probability can underflow (exp >= 1.8e-35, 1 / sum >= 1 / C), so the accurate
          // exp runs only in rows that come near it (a branch the wave skips when no lane does).
          const float zd = zmin - m;
          bool nanrow = false;
          if (zd < -80.f) nanrow = !(expf(zd) * inv > 0.f);
          if (nanrow) loss = __builtin_nanf("");
          conf_l += loss;
          if (grad) {
            if (loss != loss) {
#pragma unroll
              for (int k = 0; k < KN; ++k)
                if (in_row(k)) row[k] = loss;
            } else {
              // kq * (onehot - p), p = e * inv (the same values the loss used), two classes per op:
              // every slot gets p * (-kq) (= (0 - p) * kq exactly), then the target slot is
              // rewritten as (1 - p_t) * kq with p_t = q (e_t * inv, the same value) — the one-hot
              // selects per slot cost a compare and a select each
              const float kq = dq * q * scale;
              const f2 inv2 = {inv, inv}, nkq2 = {-kq, -kq};
#pragma unroll
              for (int k = 0; k + 1 < KN; k += 2) {
                // constant-offset reads of every slot (a padding slot reads the next row or the 8
                // floats past the tile, and its value is never stored)
                const f2 pp = f2{row[k], row[k + 1]} * inv2;
                const f2 g = pp * nkq2;
                if (in_row(k)) row[k] = g.x;
                if (in_row(k + 1)) row[k + 1] = g.y;
              }
              if constexpr (KN % 2 == 1) row[KN - 1] = (row[KN - 1] * inv2.x) * nkq2.x;
              row[c] = (1.f - q) * kq;
            }
          }
        } else if (grad) {
#pragma unroll
          for (int k = 0; k < KN; ++k)
            if (in_row(k)) row[k] = 0.f;
        }
      } else {
        const float ce = -((zt - m) - logf(s));  // cross_entropy = -log_softmax[t]
        if (pos) {
          conf_l += ce;
          a.pool[i] = -1.f;
          if (grad) {
            const float sc = 1.f / n;
#pragma unroll
            for (int k = 0; k < KN; ++k)
              if (in_row(k)) row[k] = (expf(row[k] - m) * inv - (k == c ? 1.f : 0.f)) * sc;
          }
        } else {
          bool member;
          const int pool = a.flags & (SBOD_POOL_NEG | SBOD_POOL_GLOBAL_NEG | SBOD_POOL_NONPOS_NOT_EASY);
          if (pool == SBOD_POOL_NEG || pool == SBOD_POOL_GLOBAL_NEG) member = negrow;
          else if (pool == SBOD_POOL_NONPOS_NOT_EASY) member = !easy;
          else member = true;
          a.pool[i] = member ? ce : -1.f;
          if (grad) {
#pragma unroll
            for (int k = 0; k < KN; ++k)
              if (in_row(k)) row[k] = 0.f;
          }
        }
      }
    } else {
      float m = row[0];
      for (int k = 1; k < C; ++k) m = fmaxf(m, row[k]);
      const float zt = row[c];
      float s = 0.f;
      for (int k = 0; k < C; ++k) {
        const float e = expf(row[k] - m);
        row[k] = e;
        s += e;
      }
      if (a.cls == SBOD_CLS_FOCAL) {
        if (pos || negrow) {  // SSD512.py:588-593: rows = positives ++ negatives(IoU < thr - 0.1)
          const float scale = (a.flags & SBOD_LOSS_FOCAL_NORM) ? 1.f / n : 1.f;
          conf_l += focal_row(row, C, c, s, a.afg, a.abg, a.gamma, scale, grad);
        } else if (grad) {
          for (int k = 0; k < C; ++k) row[k] = 0.f;
        }
      } else {
        const float ce = -((zt - m) - logf(s));  // cross_entropy = -log_softmax[t]
        if (pos) {
          conf_l += ce;
          a.pool[i] = -1.f;
          if (grad) {
            const float inv = 1.f / s, sc = 1.f / n;
            for (int k = 0; k < C; ++k) row[k] = (row[k] * inv - (k == c ? 1.f : 0.f)) * sc;
          }
        } else {
          bool member;
          const int pool = a.flags & (SBOD_POOL_NEG | SBOD_POOL_GLOBAL_NEG | SBOD_POOL_NONPOS_NOT_EASY);
          if (pool == SBOD_POOL_NEG || pool == SBOD_POOL_GLOBAL_NEG) member = negrow;
          else if (pool == SBOD_POOL_NONPOS_NOT_EASY) member = !easy;
          else member = true;
          a.pool[i] = member ? ce : -1.f;
          if (grad)
            for (int k = 0; k < C; ++k) row[k] = 0.f;
        }
      }
    }
  }
  MB_MARK(3 + (tid >> 6), (tid & 63) == 0);
}

// CM > 0: class rows of C <= CM in registers (padding slots -inf: no per-slot guards in the
// max / exp / sum); CM == 0: any C, rows in LDS.
// kFused (focal criteria, shared priors, one rank): the matcher runs in the same launch — the
// workgroup first matches its own 256 priors (match_wave, keys into the shards, phase-1 (obj, ovl)
// written through), counts itself in at its image, and the image's last tile runs the image's
// forced match (match_final_image) and counts the image in; every workgroup then loads its score
// tile, waits for all images (the normaliser), applies the forced rewrites of its own priors from
// the image's list, and goes on with the loss pass on registers it already holds.
template <typename T, int CM, int CLS, bool kFused, int CE = 0>
__global__ __launch_bounds__(kLTile, (CM > 24 ? 5 : 6)) void k_multibox(LossArgs a, const T *__restrict__ locs,
                                                     const T *__restrict__ scores,
                                                     T *__restrict__ glocs, T *__restrict__ gsc) {
  extern __shared__ __attribute__((aligned(16))) float s_sc[];
  __shared__ float s_red[32];
#ifdef SBOD_VARIANT_ONE_LAUNCH
  __shared__ int s_wcnt[kLTile / 64];
  __shared__ int s_misc[16];
#endif
  STAMP_BEGIN();
  span_begin(a.span);
  PHASE_DECL;
  SEG_PHASE(0);
  const int b = blockIdx.y, p0 = blockIdx.x * a.rows, tid = threadIdx.x;
  const int P = a.P, C = a.C;
  const int np = min(a.rows, P - p0);
  const int64_t rbase = static_cast<int64_t>(b) * P + p0;
  const bool valid = tid < np;
  const int64_t ic = rbase + (valid ? tid : 0);
  constexpr int NB = CM / 4;
  const T *tsrc = scores + rbase * C;
  const bool fast = fast_tile<T, NB>(tsrc, np * C);
  int objv, offb;
  float v, n;
  int64_t labg;
  RegIn rg;
  typename TileVec<T>::V tr[NB > 0 ? NB : 1];
  if constexpr (kFused) {
#ifdef SBOD_VARIANT_ONE_LAUNCH
    const int lane = tid & 63, wv = tid >> 6;
    offb = a.off[b];
    // ---- phase 1: this tile's match (the dynamic LDS holds the waves' key rows until the
    // score tile is loaded)
    uint32_t(*s_od)[kSlots][64] = reinterpret_cast<uint32_t(*)[kSlots][64]>(s_sc);
    int *s_slot = reinterpret_cast<int *>(s_sc) + (kLTile / 64) * kSlots * 64;
    unsigned long long *brow =
        a.keys + (static_cast<int64_t>(b) * kKeyShards + (blockIdx.x & (kKeyShards - 1))) * a.Gmax;
    const MatchLane m = match_wave<false, 0>(a.gt, a.labels, a.off, a.anchors, nullptr, nullptr, P, b,
                                             p0 + (tid & ~63), brow, s_od[wv], s_slot + wv * kSlots);
    if (m.valid) {   // phase-1 (obj, ovl), written through: the image's forced match reads them
      st_wt_u32(a.obj_out + ic, static_cast<uint32_t>(m.bi));
      st_wt_u32(reinterpret_cast<int32_t *>(a.ovl_out) + ic, __float_as_uint(m.best));
    }
    const int n1 = __popcll(__ballot(phase1_positive<false>(m, a.thr, 0.f)));
    drain_vm();   // this wave's key atomics performed and its (obj, ovl) stores written through
    if (lane == 0) s_wcnt[wv] = n1;
    __syncthreads();
    // ---- the tile counts itself in at its image: (1 << 32) | its phase-1 positives; the image's
    // last tile gets the count of all of them and runs the image's forced match
    if (tid == 0) {
      const unsigned nt = static_cast<unsigned>(s_wcnt[0] + s_wcnt[1] + s_wcnt[2] + s_wcnt[3]);
      const unsigned long long old =
          __hip_atomic_fetch_add(a.arrive + b, (1ull << 32) | nt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      int last = -1;
      if ((old >> 32) == static_cast<unsigned long long>(gridDim.x - 1)) {
        last = static_cast<int>(static_cast<unsigned>(old) + nt);
        __hip_atomic_store(a.arrive + b, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // zero for the next call
      }
      s_misc[15] = last;
    }
    __syncthreads();
    const int cnt1 = s_misc[15];
    if (cnt1 >= 0) {
      match_final_image<0, true>(b, a.labels, a.off, a.keys, nullptr, 0, a.Gmax, P, a.thr, nullptr, 0.f, a.obj_out,
                                 a.ovl_out, a.npos_out, a.B, cnt1, ForcedOut{a.forced, a.nforced, a.done},
                                 reinterpret_cast<unsigned char *>(s_sc), s_misc);
      __syncthreads();
    }
    // ---- the score tile -> LDS, in flight while the other images finish
    if (!fast) tile_load(s_sc, tsrc, np * C);
    if constexpr (NB > 0)
      tile_issue<T, NB>(tr, fast ? tsrc : reinterpret_cast<const T *>(a.partials), fast ? np * C : 4);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (NB > 0)
      if (fast) tile_commit(s_sc, tr, np * C);
    // ---- every image counted in: the batch's positives, then this tile's forced rewrites
    if (tid == 0) s_misc[14] = static_cast<int>(wait_all_images(a.done, a.B, a.status, &s_misc[13]));
    __syncthreads();
    n = static_cast<float>(s_misc[14]);
    objv = m.bi;
    v = m.best;
    const int nf = static_cast<int>(ld_wt_u32(a.nforced + b));
    for (int k = 0; k < nf; ++k) {
      const unsigned long long e = ld_wt_u64(a.forced + static_cast<int64_t>(b) * a.Gmax + k);
      if (static_cast<int>(e >> 32) == m.p) {
        objv = static_cast<int>(static_cast<uint32_t>(e));
        v = 1.0f;
      }
    }
    labg = a.labels[offb + objv];
    rg = reg_prefetch<T, CLS>(a, locs, p0, tid, ic, objv, offb, valid && v >= a.thr);
#else
    return;   // the one-launch criterion is built into the variant library only
#endif
  } else {
    // memory schedule: the row's matcher outputs first, then the score tile, then the loads that
    // depend on the matcher outputs (the label; the loc, prior and GT box of a row that can be
    // positive) — all in flight together; the tile is committed to LDS last (a tile that does
    // not qualify for the register path is staged first, with nothing live)
    if (!fast) tile_load(s_sc, tsrc, np * C);
    objv = a.obj[ic];
    v = a.ovl[ic];
    offb = a.off[b];
    if constexpr (NB > 0 && sizeof(T) == 4) {
      // fp32 tile by LDS-DMA: each wave-instruction copies 64 x 16 B straight into LDS (lane-
      // linear: the same layout tile_commit writes), so the tile holds no VGPRs while the row's
      // dependent loads below are in flight with it
      if (fast) {
        const float4 *src4 = reinterpret_cast<const float4 *>(tsrc);
        const int n4 = (np * C) >> 2, q = 64 * (tid >> 6), lane = tid & 63;
#pragma unroll
        for (int k = 0; k < NB; ++k) {
          const int q0 = k * kLTile + q;   // the wave's first 16-byte chunk of this round (uniform)
          if (q0 + lane < n4)
            __builtin_amdgcn_global_load_lds(src4 + q0 + lane,
                                             (__attribute__((address_space(3))) void *)(reinterpret_cast<float4 *>(s_sc) + q0),
                                             16, 0, 0);
        }
      }
    } else if constexpr (NB > 0) {   // bf16: widened in registers (the workspace's partials, 256-byte
      // aligned, are the dummy source of a tile that does not qualify: every load unconditional —
      // a conditional load makes the wait-count insertion at the join wait for the whole batch)
      tile_issue<T, NB>(tr, fast ? tsrc : reinterpret_cast<const T *>(a.partials), fast ? np * C : 4);
    }
    __builtin_amdgcn_sched_barrier(0);   // keep the tile's loads ahead of the dependent chain
    labg = a.labels[offb + objv];
    rg = reg_prefetch<T, CLS>(a, locs, p0, tid, ic, objv, offb, valid && v >= a.thr);
    if constexpr (NB > 0 && sizeof(T) != 4)
      if (fast) tile_commit(s_sc, tr, np * C);
    n = static_cast<float>(*a.npos_total);
    MB_MARK(0, tid == 0);
  }
  SEG_PHASE(1);
  const bool grad = gsc != nullptr;
  float conf_l = 0.f, loc_l = 0.f;
  multibox_rows<T, CM, CLS, CE>(a, glocs, gsc, valid, ic, v, labg, rg, n, s_sc, conf_l, loc_l);
  __syncthreads();   // every gradient row is in the LDS tile
#ifdef SBOD_VARIANT_ONE_LAUNCH
  if constexpr (kFused) {
    if (s_misc[13]) {   // this workgroup's wait gave up: its normaliser and forced rows are not
      // final, so its gradients are poisoned (NaN) rather than plausible-looking and wrong
      for (int e = tid; e < np * C; e += kLTile) s_sc[e] = __builtin_nanf("");
      if (glocs && valid)
        for (int k = 0; k < 4; ++k) stf(glocs + 4 * ic + k, __builtin_nanf(""));
      __syncthreads();
    }
  }
#endif
  SEG_PHASE(2);
  const unsigned nblk = gridDim.x * gridDim.y, blk = blockIdx.x + gridDim.x * blockIdx.y;
  if (a.fin != nullptr && !kFused) {
    // the fused finish (focal): this workgroup's record, its tile, and in the grid's last
    // workgroup the gather of every record
    block_sum2(conf_l, loc_l, s_red);
    const unsigned tag = kRecTag;
    if (tid == 0) loss_publish(a, conf_l, loc_l, tag, nblk, blk);
    if (grad) tile_store(gsc + rbase * C, s_sc, np * C, 0, kLTile);
    MB_MARK(7, tid == 0);
    if (blk == nblk - 1u) {
      __syncthreads();   // the tile's LDS reads done: the gather's scratch reuses it
      loss_gather(a, nblk, tag, n, a.out, reinterpret_cast<unsigned long long *>(s_sc),
                  reinterpret_cast<double *>(s_sc) + 32);
    }
  } else {
    if (grad) tile_store(gsc + rbase * C, s_sc, np * C, 0, kLTile);
    block_sum2(conf_l, loc_l, s_red);
    MB_MARK(7, tid == 0);
    if (a.fin != nullptr) {
#ifdef SBOD_VARIANT_ONE_LAUNCH
      if (tid < 64) multibox_finish(a, conf_l, loc_l, nblk, n, a.out);
#endif
    } else if (tid == 0) {
      a.partials[2 * blk] = conf_l;
      a.partials[2 * blk + 1] = loc_l;
    }
  }
  SEG_PHASE(3);
#ifdef SBOD_PHASE_CLOCKS
  if (tid == 0) ph[4] = __builtin_amdgcn_s_memrealtime();
  if (PHASE_PRINT_SEL)
    printf("PH multibox x%d b%d start %lld load %lld compute %lld store+sum %lld finish %lld\n", blockIdx.x, b,
           ph[0], ph[1] - ph[0], ph[2] - ph[1], ph[3] - ph[2], ph[4] - ph[3]);
#endif
  span_end(a.span);
  STAMP_END(4, 1);
}

// ----------------------------------------------------------------------------- hard negatives
// Per segment (one image, or the whole batch for SSD300's global pool) the sum of the k
// largest pool values (k = ratio * positives), found by a 4-pass 8-bit radix select on the
// float bits (pool values are >= 0; excluded rows hold -1).  Ties at the threshold take the
// lowest indices.  Selected rows get the CE gradient (softmax - onehot(0)) / n_pos.
constexpr int kHBlock = 1024;
constexpr int kHWaves = kHBlock / 64;
constexpr int kHStage = 32768;  // values staged in LDS when the segment fits

__device__ __forceinline__ bool pool_key(float v, uint32_t &u) {
  if (!(v >= 0.f)) return false;
  u = __float_as_uint(v + 0.f);  // -0 -> +0
  return true;
}

// Global pool (SSD300, SSD300.py:580-588): the selection runs over n_all values of which this
// caller owns [local_off, local_off + B*P) — the whole batch on one device (n_all = B*P,
// local_off = 0) or, data-parallel, the rank-major concatenation of every rank's pool
// (all-gathered by the caller), so the threshold, its tie order and k = ratio * (global
// positives) are those of one device holding the whole batch; gradients and the returned sum
// cover the local rows only.
template <typename T, bool kStaged>
__global__ __launch_bounds__(kHBlock) void k_hnm(const float *__restrict__ pool, int P, int B,
                                                 int global, const int32_t *__restrict__ npos,
                                                 int ratio, const T *__restrict__ scores,
                                                 T *__restrict__ gsc, int C,
                                                 const int32_t *__restrict__ npos_total,
                                                 float *__restrict__ hnm_sum, int64_t n_all,
                                                 int64_t local_off) {
  extern __shared__ float s_val[];
  __shared__ uint32_t s_hist[kHWaves][256];
  __shared__ uint32_t s_tot[256];
  __shared__ uint32_t s_state[4];  // prefix, kk, all, eq
  __shared__ float s_red[16];
  __shared__ int s_wcnt[kHWaves];
  const int seg = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t n = global ? n_all : P;
  const int64_t base = global ? 0 : static_cast<int64_t>(seg) * P;
  const int64_t n_local = static_cast<int64_t>(B) * P;
  const int64_t k = static_cast<int64_t>(ratio) * (global ? *npos_total : npos[seg]);
  const float *src = pool + base;
  if (kStaged) {
    for (int64_t i = tid; i < n; i += kHBlock) s_val[i] = src[i];
    __syncthreads();
  }
  auto val = [&](int64_t i) -> float { return kStaged ? s_val[i] : src[i]; };
  if (k <= 0) {
    if (tid == 0) hnm_sum[seg] = 0.f;
    return;
  }
  uint32_t prefix = 0, mask = 0;
  int64_t kk = k;
  bool all = false;
  uint32_t eqcount = 0;
  for (int level = 0; level < 4; ++level) {
    const int shift = 24 - 8 * level;
    for (int i = tid; i < kHWaves * 256; i += kHBlock) (&s_hist[0][0])[i] = 0;
    __syncthreads();
    for (int64_t i = tid; i < n; i += kHBlock) {
      uint32_t u;
      if (pool_key(val(i), u) && (u & mask) == prefix) atomicAdd(&s_hist[wv][(u >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (tid < 256) {
      uint32_t t = 0;
      for (int w = 0; w < kHWaves; ++w) t += s_hist[w][tid];
      s_tot[tid] = t;
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t all_flag = 0;
      if (level == 0) {
        uint64_t total = 0;
        for (int d = 0; d < 256; ++d) total += s_tot[d];
        if (total <= static_cast<uint64_t>(kk)) all_flag = 1;
      }
      uint64_t acc = 0;
      int d = 255;
      if (!all_flag) {
        for (; d > 0; --d) {
          if (acc + s_tot[d] >= static_cast<uint64_t>(kk)) break;
          acc += s_tot[d];
        }
      }
      s_state[0] = prefix | (static_cast<uint32_t>(d) << shift);
      s_state[1] = static_cast<uint32_t>(kk - static_cast<int64_t>(acc));
      s_state[2] = all_flag;
      s_state[3] = s_tot[d];
    }
    __syncthreads();
    all = s_state[2] != 0;
    if (all) break;
    prefix = s_state[0];
    kk = s_state[1];
    eqcount = s_state[3];
    mask |= 0xffu << shift;
    __syncthreads();
  }
  const float nrm = 1.f / static_cast<float>(*npos_total);
  const bool ordered = !all && eqcount > static_cast<uint32_t>(kk);
  float sum = 0.f;
  int64_t running = 0;
  for (int64_t c0 = 0; c0 < n; c0 += kHBlock) {
    const int64_t i = c0 + tid;
    uint32_t u = 0;
    const bool mem = i < n && pool_key(val(i), u);
    bool sel = mem && (all || u > prefix || (u == prefix && !ordered));
    if (ordered) {  // ties at the threshold: lowest indices first
      const bool eq = mem && u == prefix;
      const unsigned long long bal = __ballot(eq);
      const int before = __popcll(bal & ((1ull << lane) - 1ull));
      if (lane == 0) s_wcnt[wv] = __popcll(bal);
      __syncthreads();
      int64_t off = running;
      for (int w = 0; w < wv; ++w) off += s_wcnt[w];
      if (eq && off + before < kk) sel = true;
      int64_t tot = 0;
      for (int w = 0; w < kHWaves; ++w) tot += s_wcnt[w];
      running += tot;
      __syncthreads();
    }
    const int64_t r = global ? i - local_off : base + i;   // row in this caller's batch
    if (sel && r >= 0 && r < n_local) {
      sum += val(i);
      if (gsc) {
        const T *z = scores + r * C;
        float m = ldf(z);
        for (int q = 1; q < C; ++q) m = fmaxf(m, ldf(z + q));
        float s = 0.f;
        for (int q = 0; q < C; ++q) s += expf(ldf(z + q) - m);
        const float inv = 1.f / s;
        T *gz = gsc + r * C;
        for (int q = 0; q < C; ++q) stf(gz + q, (expf(ldf(z + q) - m) * inv - (q == 0 ? 1.f : 0.f)) * nrm);
      }
    }
  }
  sum = block_sum(sum, s_red);
  if (tid == 0) hnm_sum[seg] = sum;
}

// The separate finaliser (CE criteria after the mining pass, or a focal criterion with
// SBOD_LOSS_UNFUSED_FINISH): one block sums every workgroup's fp32 partials and the mining
// segments' sums EXACTLY (128-bit fixed point, as the fused finish: the same loss bit for bit
// whichever finish ran), falling back to a double sum when a value cannot be folded.
constexpr int kFinThreads = 256;   // k_loss_final's block (a constant: no hidden-argument load for blockDim)
__device__ __forceinline__ void loss_final_body(const float *__restrict__ partials, int nparts,
                                                const float *__restrict__ hnm, int nseg,
                                                const int32_t *__restrict__ npos_total, int reg, int cls,
                                                int flags, float reg_weight, float *__restrict__ out) {
  STAMP_BEGIN();
  __shared__ double s_red[16];
  __shared__ unsigned long long s_fx[5 * 4];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  Fx128 fc{0ull, 0ull}, fl{0ull, 0ull};
  bool ok = true;
  // eight partials per thread in flight per batch (a 1-block launch: its time is load latency)
  constexpr int kB = 8;
  const float2 *p2 = reinterpret_cast<const float2 *>(partials);
  for (int i0 = 0; i0 < nparts; i0 += kB * kFinThreads) {
    float2 v[kB];
#pragma unroll
    for (int k = 0; k < kB; ++k) {
      const int i = i0 + k * kFinThreads + tid;
      v[k] = p2[min(i, nparts - 1)];   // unconditional (clamped), zeroed below: no wait at a join
      if (i >= nparts) v[k] = make_float2(0.f, 0.f);
    }
#pragma unroll
    for (int k = 0; k < kB; ++k) {
      const bool f = fx_foldable(v[k].x) && fx_foldable(v[k].y);
      ok = ok && f;
      fc = fx128_add(fc, to_fx128(f ? v[k].x : 0.f));
      fl = fx128_add(fl, to_fx128(f ? v[k].y : 0.f));
    }
  }
  for (int i = tid; i < nseg; i += kFinThreads) {
    const float v = hnm[i];
    const bool f = fx_foldable(v);
    ok = ok && f;
    fc = fx128_add(fc, to_fx128(f ? v : 0.f));
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    fc = fx128_add(fc, Fx128{shfl_xor_u64(fc.lo, m), shfl_xor_u64(fc.hi, m)});
    fl = fx128_add(fl, Fx128{shfl_xor_u64(fl.lo, m), shfl_xor_u64(fl.hi, m)});
  }
  const bool wave_ok = __ballot(!ok) == 0ull;
  if (lane == 0) {
    s_fx[5 * wv + 0] = fc.lo;
    s_fx[5 * wv + 1] = fc.hi;
    s_fx[5 * wv + 2] = fl.lo;
    s_fx[5 * wv + 3] = fl.hi;
    s_fx[5 * wv + 4] = wave_ok ? 1ull : 0ull;
  }
  __syncthreads();
  bool all_ok = true;
  fc = Fx128{0ull, 0ull};
  fl = Fx128{0ull, 0ull};
  for (int w2 = 0; w2 < kFinThreads / 64; ++w2) {
    fc = fx128_add(fc, Fx128{s_fx[5 * w2 + 0], s_fx[5 * w2 + 1]});
    fl = fx128_add(fl, Fx128{s_fx[5 * w2 + 2], s_fx[5 * w2 + 3]});
    all_ok = all_ok && s_fx[5 * w2 + 4] != 0ull;
  }
  double c = fx128_value(fc.lo, fc.hi), l = fx128_value(fl.lo, fl.hi);
  if (!all_ok) {   // a non-finite or huge value: the double sum
    c = 0.0;
    l = 0.0;
    for (int i = tid; i < nparts; i += kFinThreads) {
      c += partials[2 * i];
      l += partials[2 * i + 1];
    }
    for (int i = tid; i < nseg; i += kFinThreads) c += hnm[i];
    c = block_sum(c, s_red);
    __syncthreads();
    l = block_sum(l, s_red);
  }
  if (tid == 0) loss_outputs(c, l, static_cast<float>(*npos_total), reg, cls, flags, reg_weight, out);
  STAMP_END(6, 1);
}

// The launch takes ONE by-value argument: this runtime's host cost of a launch grows with the
// argument count (≈ 0.5 µs more for sixteen arguments than for one struct of the same bytes,
// scripts/micro/launch_cost.hip), and this kernel is on every step's criterion submit.
struct LossFinalArgs {
  const float *partials;
  int nparts;
  const float *hnm;
  int nseg;
  const int32_t *npos_total;
  int reg, cls, flags;
  float reg_weight;
  float *out;
};
__global__ __launch_bounds__(kFinThreads) void k_loss_final(const LossFinalArgs a) {
  loss_final_body(a.partials, a.nparts, a.hnm, a.nseg, a.npos_total, a.reg, a.cls, a.flags, a.reg_weight, a.out);
}

// ----------------------------------------------------------------------------- standalone
__global__ __launch_bounds__(256) void k_aligned(int kind, const float *__restrict__ b1,
                                                 const float *__restrict__ b2, int64_t n,
                                                 float *__restrict__ ov, float *__restrict__ g,
                                                 float *__restrict__ g2) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  OvOut r = aligned_overlap<true>(kind, ld4(b1 + 4 * i), ld4(b2 + 4 * i), g != nullptr || g2 != nullptr);
  ov[i] = r.v;
  if (g2) st4(g2 + 4 * i, Box4{r.g2[0], r.g2[1], r.g2[2], r.g2[3]});
  if (g) st4(g + 4 * i, Box4{r.g[0], r.g[1], r.g[2], r.g[3]});
}

__global__ __launch_bounds__(256) void k_smooth_l1(const float *__restrict__ a,
                                                   const float *__restrict__ b, int64_t n,
                                                   float beta, float *__restrict__ loss,
                                                   float *__restrict__ g) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float d = a[i] - b[i], x = fabsf(d);
  const float sg = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
  const bool big = x >= beta;
  loss[i] = big ? x - 0.5f * beta : 0.5f * (x * x) / beta;
  if (g) g[i] = big ? sg : (x / beta) * sg;
}

__global__ __launch_bounds__(256) void k_focal_rows(int kind, const float *__restrict__ z,
                                                    const int64_t *__restrict__ tgt, int64_t rows,
                                                    int C, float afg, float abg, float gamma,
                                                    float *__restrict__ loss, float *__restrict__ g) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  const float *x = z + r * C;
  float *gr = g ? g + r * C : nullptr;
  const int t = static_cast<int>(tgt[r]);
  float L = 0.f;
  if (kind == SBOD_FOCAL_SOFTMAX) {
    float m = x[0];
    for (int c = 1; c < C; ++c) m = fmaxf(m, x[c]);
    float s = 0.f;
    for (int c = 0; c < C; ++c) s += expf(x[c] - m);
    const float inv = 1.f / s;
    float pmin = 1.f;
    for (int c = 0; c < C; ++c) pmin = fminf(pmin, expf(x[c] - m) * inv);
    const float q = expf(x[t] - m) * inv, lq = logf(q);
    float dq;
    if (t == 0) {
      L = abg * powg(q, gamma) * -lq;
      dq = abg * (gamma * powg1(q, gamma) * -lq - powg1(q, gamma));
    } else {
      const float om = 1.f - q;
      L = afg * powg(om, gamma) * -lq;
      dq = afg * (-gamma * powg1(om, gamma) * -lq - powg(om, gamma) / q);
    }
    if (!(pmin > 0.f)) L = __builtin_nanf("");
    if (gr)
      for (int c = 0; c < C; ++c)
        gr[c] = L != L ? L : dq * q * ((c == t ? 1.f : 0.f) - expf(x[c] - m) * inv);
  } else if (kind == SBOD_FOCAL_SIGMOID) {  // Loss.py:48-80, column 0 excluded
    if (gr) gr[0] = 0.f;
    for (int c = 1; c < C; ++c) {
      const float p = 1.f / (1.f + expf(-x[c]));
      const float lp = logf(p), l1p = logf(1.f - p);
      const float t1 = powg(1.f - p, gamma) * lp, t2 = powg(p, gamma) * l1p;
      const float m1 = t == c ? 1.f : 0.f, m2 = (t != c && t > 0) ? 1.f : 0.f;
      L += -(m1 * afg * t1) - (m2 * (1.f - afg) * t2);
      if (gr) {
        const float dp = p * (1.f - p);
        const float d1 = -gamma * powg1(1.f - p, gamma) * lp + powg(1.f - p, gamma) / p;
        const float d2 = gamma * powg1(p, gamma) * l1p - powg(p, gamma) / (1.f - p);
        gr[c] = -(m1 * afg * d1 * dp) - (m2 * (1.f - afg) * d2 * dp);
      }
    }
  } else {  // FocalLoss (Loss.py:91-103): BCE-with-logits, prediction clamped to [1e-4, 1-1e-4]
    for (int c = 0; c < C; ++c) {
      const float zc = x[c];
      const float y = t == c ? 1.f : 0.f;
      const float sg = 1.f / (1.f + expf(-zc));
      const float pred = fminf(fmaxf(sg, 1e-4f), 1.f - 1e-4f);
      const float mx = fmaxf(-zc, 0.f);
      const float ce = (1.f - y) * zc + mx + logf(expf(-mx) + expf(-zc - mx));
      const float al = y * afg + (1.f - y) * (1.f - afg);
      const float pt = y == 1.f ? pred : 1.f - pred;
      const float w = powg(1.f - pt, gamma);
      L += al * w * ce;
      if (gr) {
        const float dpred = (sg >= 1e-4f && sg <= 1.f - 1e-4f) ? sg * (1.f - sg) : 0.f;
        const float dpt = y == 1.f ? dpred : -dpred;
        gr[c] = al * (-gamma * powg1(1.f - pt, gamma) * dpt * ce + w * (sg - y));
      }
    }
  }
  loss[r] = L;
}

}  // namespace sbod

using namespace sbod;

namespace {
struct LossWs {
  float *partials, *pool, *hnm;
  unsigned long long *fin;
  void *recs;
  size_t pool_off;     // byte offset of `pool` (sbod_loss_pool_offset)
  size_t zero_bytes;   // the fused finish's state: its words (`fin`) and records, left zero
  size_t bytes;
};
// Rows per k_multibox tile (balanced_rows, sbod_common.h); the workspaces are sized for
// kLMinRows-row tiles.
constexpr int kLMinRows = 64;
inline int mb_rows(int B, int P) { return balanced_rows(B, P, kLTile, kLMinRows); }
LossWs carve(void *w, int B, int P) {
  const size_t nblk = static_cast<size_t>(B) * ((P + kLMinRows - 1) / kLMinRows);   // the most tiles mb_rows makes
  LossWs r;
  // the fused finish's state first (zero on entry, SBOD_LOSS_WS_ZEROED): its words, then one
  // record per workgroup; no other pass writes them
  r.fin = ws_at<unsigned long long>(w, 0);
  size_t o = align_up(kFinBytes);
  r.recs = ws_at<char>(w, o);
  o += align_up(nblk * 16);
  r.zero_bytes = o;
  r.partials = ws_at<float>(w, o);
  o += align_up(nblk * 2 * sizeof(float));
  r.pool = ws_at<float>(w, o);
  r.pool_off = o;
  o += align_up(static_cast<size_t>(B) * P * sizeof(float));
  r.hnm = ws_at<float>(w, o);
  o += align_up((B + 1) * sizeof(float));
  r.bytes = o;
  return r;
}
// Hard-negative mining (CE) and the loss finaliser, after the fused pass: per-image pools, or
// the global pool over `n_all` gathered values of which this caller owns [local_off, +B*P).
int mine_and_finish(const void *scores, int dtype, int B, int P, int C, const int32_t *n_pos,
                    const int32_t *npos_total, int reg, int cls, int flags, int neg_pos_ratio,
                    float reg_weight, const float *pool, int64_t n_all, int64_t local_off,
                    void *grad_scores, float *loss_out, const LossWs &ws, hipStream_t s) {
  const int rows = mb_rows(B, P);
  const int nblk = B * ((P + rows - 1) / rows);
  int nseg = 0;
  if (cls == SBOD_CLS_CE) {
    const int global = (flags & SBOD_POOL_GLOBAL_NEG) ? 1 : 0;
    nseg = global ? 1 : B;
    const int64_t segn = global ? n_all : P;
    const bool staged = segn <= kHStage;
    const size_t hl = staged ? segn * sizeof(float) : 0;
#define SBOD_HNM(T, ST)                                                                         \
  do {                                                                                          \
    KernelTimer kt("k_hnm", s, true);                                                                 \
    tlaunch(kt, (k_hnm<T, ST>), dim3(nseg), dim3(kHBlock), hl, s, pool, P, B, global,    \
                       n_pos, neg_pos_ratio, static_cast<const T *>(scores), static_cast<T *>(grad_scores), C, \
                       npos_total, ws.hnm, n_all, local_off);                                   \
  } while (0)
    if (dtype == SBOD_DT_F32) {
      if (staged) SBOD_HNM(float, true); else SBOD_HNM(float, false);
    } else {
      if (staged) SBOD_HNM(uint16_t, true); else SBOD_HNM(uint16_t, false);
    }
#undef SBOD_HNM
    SBOD_LAUNCHED("k_hnm");
  }
  {
    KernelTimer kt("k_loss_final", s, true);
    tlaunch(kt, k_loss_final, dim3(1), dim3(kFinThreads), 0, s,
            LossFinalArgs{static_cast<const float *>(ws.partials), static_cast<int>(nblk),
                          static_cast<const float *>(ws.hnm), nseg, npos_total, reg, cls, flags, reg_weight,
                          loss_out});
  }
  SBOD_LAUNCHED("k_loss_final");
  return SBOD_OK;
}
// The one-launch criterion's workspace: [done, status | arrivals [B] | matcher workspace (keys
// first) | loss workspace (the finish's accumulators first) | forced lists [B][Gmax] | their
// counts [B]].  Everything up to the end of the finish's accumulators must be zero on entry and
// is left zero by every successful call (zero_bytes); the matcher and loss workspaces are also
// what the two-launch form of the same call uses.
struct CritWs {
  unsigned long long *done, *arrive, *forced;
  unsigned *status;
  int32_t *nforced;
  char *match_ws, *loss_ws;
  size_t match_bytes, loss_bytes, zero_bytes, bytes;
};
CritWs carve_crit(void *w, int B, int Gmax, int P) {
  CritWs r;
  r.done = ws_at<unsigned long long>(w, 0);
  r.status = ws_at<unsigned>(w, 8);
  size_t o = 256;
  r.arrive = ws_at<unsigned long long>(w, o);
  o += align_up(static_cast<size_t>(B) * 8);
  r.match_ws = ws_at<char>(w, o);
  r.match_bytes = sbod_match_workspace_bytes_p(B, Gmax, P);
  o += align_up(r.match_bytes);
  r.loss_ws = ws_at<char>(w, o);
  const LossWs lw = carve(nullptr, B, P);
  r.loss_bytes = lw.bytes;
  r.zero_bytes = o + lw.zero_bytes;
  o += align_up(r.loss_bytes);
  r.forced = ws_at<unsigned long long>(w, o);
  o += align_up(static_cast<size_t>(B) * Gmax * 8);
  r.nforced = ws_at<int32_t>(w, o);
  o += align_up(static_cast<size_t>(B) * 4);
  r.bytes = o;
  return r;
}

#ifdef SBOD_VARIANT_ONE_LAUNCH
// Workgroups of `kernel` (kLTile threads, `lds` dynamic bytes) resident at once on the current
// device: the occupancy query times the CU count, cached per (device, kernel, lds).  The
// one-launch criterion needs its whole grid resident (its workgroups wait for each other).  The
// query ignores the SGPR file: 256-thread blocks are admitted per CU up to
// floor(800 / (ceil(sgpr / 16) * 16 + 16)) (MI355X_MICROARCH.md, residency), which is 6 for the
// k_multibox<..., true> instantiations (TotalSGPRs <= 112 in the build's resource table;
// tests/test_cpu_host.py checks it), so the count per CU is capped at kCritBlocksPerCU.
constexpr int kCritBlocksPerCU = 6;
int resident_capacity(const void *kernel, size_t lds) {
  struct Entry { int dev; const void *k; size_t lds; int cap; };
  static std::mutex mu;
  static std::vector<Entry> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  std::lock_guard<std::mutex> g(mu);
  for (const Entry &e : cache)
    if (e.dev == dev && e.k == kernel && e.lds == lds) return e.cap;
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kLTile, lds) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
    (void)hipGetLastError();
    per_cu = cus = 0;
  }
  if (per_cu > kCritBlocksPerCU) per_cu = kCritBlocksPerCU;
  cache.push_back(Entry{dev, kernel, lds, per_cu * cus});
  return per_cu * cus;
}
#endif  // SBOD_VARIANT_ONE_LAUNCH
}  // namespace

extern "C" {

size_t sbod_loss_workspace_bytes(int B, int P) { return carve(nullptr, B, P).bytes; }

size_t sbod_criterion_workspace_bytes(int B, int Gmax, int P) {
  return carve_crit(nullptr, B > 0 ? B : 1, Gmax > 0 ? Gmax : 1, P > 0 ? P : 1).bytes;
}
size_t sbod_criterion_zero_bytes(int B, int Gmax, int P) {
  return carve_crit(nullptr, B > 0 ? B : 1, Gmax > 0 ? Gmax : 1, P > 0 ? P : 1).zero_bytes;
}

int sbod_criterion_focal(const void *locs, const void *scores, int dtype, int B, int P, int C,
                         const float *priors_cxcy, const float *priors_xy, const float *gt_boxes,
                         const int64_t *gt_labels, const int32_t *gt_offsets, int Gmax, float threshold,
                         float neg_threshold, int reg, int flags, float reg_weight, float focal_alpha,
                         float focal_gamma, int32_t *obj, float *ovl, int32_t *n_pos, void *grad_locs,
                         void *grad_scores, float *loss_out, void *workspace, size_t workspace_bytes,
                         void *stream) {
  SBOD_REQUIRE(B > 0 && P > 0 && C >= 2 && Gmax > 0 && locs && scores && priors_cxcy && priors_xy && gt_boxes &&
                   gt_labels && gt_offsets && obj && ovl && n_pos && loss_out,
               "sbod_criterion_focal: bad arguments (B=%d P=%d C=%d Gmax=%d)", B, P, C, Gmax);
  SBOD_REQUIRE(dtype == SBOD_DT_F32 || dtype == SBOD_DT_BF16, "sbod_criterion_focal: dtype %d", dtype);
  SBOD_REQUIRE(reg >= 0 && reg <= 2, "sbod_criterion_focal: reg %d", reg);
  SBOD_REQUIRE(Gmax <= 4096, "sbod_criterion_focal: Gmax %d > 4096 unsupported", Gmax);
  SBOD_REQUIRE(C * kLTile * 4 <= 160 * 1024, "sbod_criterion_focal: C=%d too large for one LDS tile", C);
  SBOD_REQUIRE((flags & ~(SBOD_LOSS_FOCAL_NORM | SBOD_CRIT_WS_ZEROED | SBOD_CRIT_TWO_LAUNCH |
                          SBOD_LOSS_UNFUSED_FINISH)) == 0,
               "sbod_criterion_focal: unknown flags 0x%x", flags);
  const CritWs ws = carve_crit(workspace, B, Gmax, P);
  if (workspace_bytes < ws.bytes) {
    set_error("sbod_criterion_focal: workspace %zu < %zu", workspace_bytes, ws.bytes);
    return SBOD_E_WORKSPACE;
  }
  hipStream_t s = as_stream(stream);
  if ((flags & SBOD_CRIT_WS_ZEROED) == 0 && hipMemsetAsync(workspace, 0, ws.zero_bytes, s) != hipSuccess)
    return launch_status("hipMemsetAsync(criterion)");
  const int lflags = flags & (SBOD_LOSS_FOCAL_NORM | SBOD_LOSS_UNFUSED_FINISH);
  const dim3 grid((P + kLTile - 1) / kLTile, B);
  const size_t nblk = static_cast<size_t>(grid.x) * B;
#ifdef SBOD_VARIANT_ONE_LAUNCH
  // the tile's rows (+ 8 floats, as k_multibox), the match phase's key rows, and the forced
  // match's LDS form beyond 64 objects: one dynamic region, used in turn
  size_t lds = (static_cast<size_t>(kLTile) * C + 8) * sizeof(float);
  const size_t keys_lds = (kLTile / 64) * kSlots * (64 + 1) * sizeof(uint32_t);
  if (lds < keys_lds) lds = keys_lds;
  if (Gmax > 64 && lds < static_cast<size_t>(Gmax) * 24) lds = static_cast<size_t>(Gmax) * 24;
  const void *kfused = nullptr;
#define SBOD_CRIT_K(T, CM) kfused = reinterpret_cast<const void *>(&k_multibox<T, CM, SBOD_CLS_FOCAL, true>)
#define SBOD_CRIT_C(T)                 \
  do {                                 \
    if (C <= 8) SBOD_CRIT_K(T, 8);     \
    else if (C <= 16) SBOD_CRIT_K(T, 16); \
    else if (C <= 24) SBOD_CRIT_K(T, 24); \
    else if (C <= 32) SBOD_CRIT_K(T, 32); \
    else SBOD_CRIT_K(T, 0);            \
  } while (0)
  if (dtype == SBOD_DT_F32) SBOD_CRIT_C(float);
  else SBOD_CRIT_C(uint16_t);
#undef SBOD_CRIT_C
#undef SBOD_CRIT_K
  const bool one = (flags & (SBOD_CRIT_TWO_LAUNCH | SBOD_LOSS_UNFUSED_FINISH)) == 0 &&
                   nblk <= static_cast<size_t>(resident_capacity(kfused, lds));
#else
  // the one-launch form (k_multibox<..., true>: workgroups that wait for each other) is built into
  // the variant library only (scripts/build_variant_lib.sh); the product library always runs the
  // matcher and the loss pass as separate launches
  (void)nblk;
  const bool one = false;
#endif
  if (!one) {   // the two-launch form on the same workspace (both parts are zero on entry)
    const int st = sbod_match_f32(gt_boxes, gt_labels, gt_offsets, B, Gmax, priors_xy, nullptr, nullptr, P, threshold,
                                  0.01f, SBOD_MATCH_WS_ZEROED, obj, ovl, n_pos, ws.match_ws, ws.match_bytes, stream);
    if (st != SBOD_OK) return st;
    return sbod_multibox_loss(locs, scores, dtype, B, P, C, priors_cxcy, nullptr, nullptr, gt_boxes, gt_labels,
                              gt_offsets, obj, ovl, n_pos, n_pos + B, threshold, neg_threshold, 0.01f, reg,
                              SBOD_CLS_FOCAL, lflags | SBOD_LOSS_WS_ZEROED, 3, reg_weight, focal_alpha, focal_gamma,
                              grad_locs, grad_scores, loss_out, ws.loss_ws, ws.loss_bytes, stream);
  }
#ifdef SBOD_VARIANT_ONE_LAUNCH
  const LossWs lw = carve(ws.loss_ws, B, P);
  LossArgs a{B, P, C, priors_cxcy, nullptr, nullptr, gt_boxes, gt_labels, gt_offsets, nullptr, nullptr, nullptr,
             threshold, neg_threshold, 0.01f, reg, SBOD_CLS_FOCAL, lflags, reg_weight, focal_alpha,
             1.f - focal_alpha, focal_gamma, lw.partials, lw.pool, nullptr, lw.fin, loss_out};
  a.anchors = priors_xy;
  a.Gmax = Gmax;
  a.obj_out = obj;
  a.ovl_out = ovl;
  a.npos_out = n_pos;
  a.keys = reinterpret_cast<unsigned long long *>(ws.match_ws);   // the matcher workspace's keys
  a.arrive = ws.arrive;
  a.done = ws.done;
  a.status = ws.status;
  a.forced = ws.forced;
  a.nforced = ws.nforced;
  {
    KernelTimer kt("k_criterion", s, true);
    a.span = kt.span();
#define SBOD_CRIT(T, CM)                                                                                  \
  tlaunch(kt, (k_multibox<T, CM, SBOD_CLS_FOCAL, true>), grid, dim3(kLTile), lds, s, a,                  \
          static_cast<const T *>(locs), static_cast<const T *>(scores), static_cast<T *>(grad_locs),      \
          static_cast<T *>(grad_scores))
#define SBOD_CRIT_C(T)                 \
  do {                                 \
    if (C <= 8) SBOD_CRIT(T, 8);       \
    else if (C <= 16) SBOD_CRIT(T, 16); \
    else if (C <= 24) SBOD_CRIT(T, 24); \
    else if (C <= 32) SBOD_CRIT(T, 32); \
    else SBOD_CRIT(T, 0);              \
  } while (0)
    if (dtype == SBOD_DT_F32) SBOD_CRIT_C(float);
    else SBOD_CRIT_C(uint16_t);
#undef SBOD_CRIT_C
#undef SBOD_CRIT
  }
  SBOD_LAUNCHED("k_criterion");
  return SBOD_OK;
#else
  return SBOD_OK;
#endif
}

int sbod_criterion_focal_lists(const void *const *box_ptrs, const void *const *label_ptrs, const int32_t *counts,
                               int64_t capacity, const void *locs, const void *scores, int dtype, int B, int P,
                               int C, const float *priors_cxcy, const float *priors_xy, float *gt_boxes,
                               int64_t *gt_labels, int32_t *gt_offsets, int Gmax, float threshold,
                               float neg_threshold, int reg, int flags, float reg_weight, float focal_alpha,
                               float focal_gamma, int32_t *obj, float *ovl, int32_t *n_pos, void *grad_locs,
                               void *grad_scores, float *loss_out, void *workspace, size_t workspace_bytes,
                               void *stream) {
  SBOD_REQUIRE(B > 0 && P > 0 && C >= 2 && Gmax > 0 && locs && scores && priors_cxcy && priors_xy && gt_boxes &&
                   gt_labels && gt_offsets && obj && ovl && n_pos && loss_out,
               "sbod_criterion_focal_lists: bad arguments (B=%d P=%d C=%d Gmax=%d)", B, P, C, Gmax);
  SBOD_REQUIRE(dtype == SBOD_DT_F32 || dtype == SBOD_DT_BF16, "sbod_criterion_focal_lists: dtype %d", dtype);
  SBOD_REQUIRE(reg >= 0 && reg <= 2, "sbod_criterion_focal_lists: reg %d", reg);
  SBOD_REQUIRE((flags & ~(SBOD_LOSS_FOCAL_NORM | SBOD_CRIT_WS_ZEROED | SBOD_CRIT_TWO_LAUNCH |
                          SBOD_LOSS_UNFUSED_FINISH)) == 0,
               "sbod_criterion_focal_lists: unknown flags 0x%x", flags);
  const CritWs ws = carve_crit(workspace, B, Gmax, P);
  if (workspace_bytes < ws.bytes) {
    set_error("sbod_criterion_focal_lists: workspace %zu < %zu", workspace_bytes, ws.bytes);
    return SBOD_E_WORKSPACE;
  }
  hipStream_t s = as_stream(stream);
  if ((flags & SBOD_CRIT_WS_ZEROED) == 0 && hipMemsetAsync(workspace, 0, ws.zero_bytes, s) != hipSuccess)
    return launch_status("hipMemsetAsync(criterion)");
  const int st = sbod_match_lists_f32(box_ptrs, label_ptrs, counts, capacity, gt_boxes, gt_labels, gt_offsets, B,
                                      Gmax, priors_xy, nullptr, nullptr, P, threshold, 0.01f, SBOD_MATCH_WS_ZEROED,
                                      obj, ovl, n_pos, ws.match_ws, ws.match_bytes, stream);
  if (st != SBOD_OK) return st;
  const int lflags = flags & (SBOD_LOSS_FOCAL_NORM | SBOD_LOSS_UNFUSED_FINISH);
  return sbod_multibox_loss(locs, scores, dtype, B, P, C, priors_cxcy, nullptr, nullptr, gt_boxes, gt_labels,
                            gt_offsets, obj, ovl, n_pos, n_pos + B, threshold, neg_threshold, 0.01f, reg,
                            SBOD_CLS_FOCAL, lflags | SBOD_LOSS_WS_ZEROED, 3, reg_weight, focal_alpha, focal_gamma,
                            grad_locs, grad_scores, loss_out, ws.loss_ws, ws.loss_bytes, stream);
}

int sbod_criterion_status(const void *workspace, void *stream) {
  // diagnostics: the one-launch criterion's sticky wait-timeout word (nonzero: a wait gave up in
  // some call on this workspace; the per-call word is cleared by each call's finish), read with a
  // stream synchronisation
  SBOD_REQUIRE(workspace != nullptr, "sbod_criterion_status: null workspace");
  unsigned v = 0;
  hipStream_t s = as_stream(stream);
  if (hipMemcpyAsync(&v, static_cast<const char *>(workspace) + 12, 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return launch_status("sbod_criterion_status");
  return static_cast<int>(v);
}

int sbod_loss_finish_status(const void *workspace, int B, int Gmax, int P, void *stream) {
  // diagnostics: the fused loss finish's sticky word (nonzero: a gather wait gave up in some
  // call on this workspace, so every later loss from it is NaN until its zero-on-entry prefix is
  // zeroed again — call without the *_WS_ZEROED flag once).  Gmax == 0: a sbod_multibox_loss
  // workspace; Gmax > 0: a sbod_criterion_focal workspace of (B, Gmax, P).  Synchronises.
  SBOD_REQUIRE(workspace != nullptr && B > 0 && P > 0 && Gmax >= 0, "sbod_loss_finish_status: bad arguments");
  const char *lw = static_cast<const char *>(workspace);
  if (Gmax > 0) lw = carve_crit(const_cast<void *>(workspace), B, Gmax, P).loss_ws;
  unsigned long long v = 0;
  hipStream_t s = as_stream(stream);
  if (hipMemcpyAsync(&v, lw + kFinSticky * sizeof(unsigned long long), 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return launch_status("sbod_loss_finish_status");
  return v != 0ull ? 1 : 0;
}

int sbod_multibox_loss(const void *locs, const void *scores, int dtype, int B, int P, int C,
                       const float *priors_cxcy, const float *odm_arm_locs,
                       const float *arm_scores, const float *gt_boxes, const int64_t *gt_labels,
                       const int32_t *gt_offsets, const int32_t *obj, const float *ovl,
                       const int32_t *n_pos, const int32_t *npos_total, float threshold,
                       float neg_threshold, float theta, int reg, int cls, int flags,
                       int neg_pos_ratio, float reg_weight, float focal_alpha, float focal_gamma,
                       void *grad_locs, void *grad_scores, float *loss_out, void *workspace,
                       size_t workspace_bytes, void *stream) {
  SBOD_REQUIRE(B > 0 && P > 0 && C >= 2 && locs && scores && priors_cxcy && gt_boxes &&
                   gt_labels && gt_offsets && obj && ovl && n_pos && npos_total && loss_out,
               "sbod_multibox_loss: bad arguments (B=%d P=%d C=%d)", B, P, C);
  SBOD_REQUIRE(dtype == SBOD_DT_F32 || dtype == SBOD_DT_BF16, "sbod_multibox_loss: dtype %d", dtype);
  SBOD_REQUIRE(reg >= 0 && reg <= 2 && (cls == 0 || cls == 1), "sbod_multibox_loss: reg/cls");
  SBOD_REQUIRE(C * kLTile * 4 <= 160 * 1024, "sbod_multibox_loss: C=%d too large for one LDS tile", C);
  const bool odm = (flags & SBOD_MATCH_ODM) != 0;
  SBOD_REQUIRE(!odm || (odm_arm_locs && arm_scores), "sbod_multibox_loss: ODM needs ARM locs/scores");
  SBOD_REQUIRE(!(flags & SBOD_LOSS_DEFER_MINING) || (cls == SBOD_CLS_CE && (flags & SBOD_POOL_GLOBAL_NEG)),
               "sbod_multibox_loss: DEFER_MINING applies to the CE global pool only");
  LossWs ws = carve(workspace, B, P);
  if (workspace_bytes < ws.bytes) {
    set_error("sbod_multibox_loss: workspace %zu < %zu", workspace_bytes, ws.bytes);
    return SBOD_E_WORKSPACE;
  }
  hipStream_t s = as_stream(stream);
  // no mining pass (focal, without SBOD_LOSS_UNFUSED_FINISH): the fused pass finishes the loss
  // itself (loss_gather), so the step has no k_loss_final launch; its state (sticky word, records)
  // is zero on entry and left zero (SBOD_LOSS_WS_ZEROED); every call without the flag zeroes it,
  // fused or not, and no other pass writes it
  const bool fused = cls == SBOD_CLS_FOCAL && !(flags & (SBOD_LOSS_DEFER_MINING | SBOD_LOSS_UNFUSED_FINISH));
  if ((flags & SBOD_LOSS_WS_ZEROED) == 0 &&
      hipMemsetAsync(ws.fin, 0, ws.zero_bytes, s) != hipSuccess)
    return launch_status("hipMemsetAsync(loss)");
  LossArgs a{B, P, C, priors_cxcy, odm_arm_locs, arm_scores, gt_boxes, gt_labels, gt_offsets, obj,
             npos_total, ovl, threshold, neg_threshold, theta, reg, cls, flags, reg_weight,
             focal_alpha, 1.f - focal_alpha, focal_gamma, ws.partials, ws.pool, nullptr,
             fused ? ws.fin : nullptr, loss_out};
  a.recs = ws.recs;
  a.rows = mb_rows(B, P);
  dim3 grid((P + a.rows - 1) / a.rows, B);
  // + 8 floats: the register path's constant-offset row reads may run up to 7 past the last row
  const size_t lds = (static_cast<size_t>(a.rows) * C + 8) * sizeof(float);
  {
    KernelTimer kt("k_multibox", s, true);
    a.span = kt.span();
#define SBOD_MB(T, CM, CLS)                                                                       \
  tlaunch(kt, (k_multibox<T, CM, CLS, false>), grid, dim3(kLTile), lds, s, a, static_cast<const T *>(locs), \
                     static_cast<const T *>(scores), static_cast<T *>(grad_locs), static_cast<T *>(grad_scores))
    // VOC's 21 classes: the exact-width rows (no padding slots)
#define SBOD_MB21(T, CLS)                                                                          \
  tlaunch(kt, (k_multibox<T, 24, CLS, false, 21>), grid, dim3(kLTile), lds, s, a,                  \
          static_cast<const T *>(locs), static_cast<const T *>(scores), static_cast<T *>(grad_locs),    \
          static_cast<T *>(grad_scores))
    // rows of C <= CM classes in registers; wider rows take the LDS path
#define SBOD_MB_C(T)                                                  \
  do {                                                                \
    if (cls == SBOD_CLS_FOCAL) {                                      \
      if (C == 21) SBOD_MB21(T, SBOD_CLS_FOCAL);                      \
      else if (C <= 8) SBOD_MB(T, 8, SBOD_CLS_FOCAL);                 \
      else if (C <= 16) SBOD_MB(T, 16, SBOD_CLS_FOCAL);               \
      else if (C <= 24) SBOD_MB(T, 24, SBOD_CLS_FOCAL);               \
      else if (C <= 32) SBOD_MB(T, 32, SBOD_CLS_FOCAL);               \
      else SBOD_MB(T, 0, SBOD_CLS_FOCAL);                             \
    } else {                                                          \
      if (C == 21) SBOD_MB21(T, SBOD_CLS_CE);                         \
      else if (C <= 8) SBOD_MB(T, 8, SBOD_CLS_CE);                    \
      else if (C <= 16) SBOD_MB(T, 16, SBOD_CLS_CE);                  \
      else if (C <= 24) SBOD_MB(T, 24, SBOD_CLS_CE);                  \
      else if (C <= 32) SBOD_MB(T, 32, SBOD_CLS_CE);                  \
      else SBOD_MB(T, 0, SBOD_CLS_CE);                                \
    }                                                                 \
  } while (0)
    if (dtype == SBOD_DT_F32) SBOD_MB_C(float);
    else SBOD_MB_C(uint16_t);
#undef SBOD_MB_C
#undef SBOD_MB21
#undef SBOD_MB
  }
  SBOD_LAUNCHED("k_multibox");
  if (fused) return SBOD_OK;
  if (flags & SBOD_LOSS_DEFER_MINING) return SBOD_OK;   // the caller exchanges the pool first
  return mine_and_finish(scores, dtype, B, P, C, n_pos, npos_total, reg, cls, flags, neg_pos_ratio,
                         reg_weight, ws.pool, static_cast<int64_t>(B) * P, 0, grad_scores, loss_out, ws, s);
}

size_t sbod_loss_zero_bytes(int B, int P) { return carve(nullptr, B > 0 ? B : 1, P > 0 ? P : 1).zero_bytes; }

size_t sbod_loss_pool_offset(int B, int P) {
  return carve(nullptr, B, P).pool_off;
}

int sbod_multibox_mine_global(const void *scores, int dtype, int B, int P, int C,
                              const int32_t *npos_total, int reg, int cls, int flags,
                              int neg_pos_ratio, float reg_weight, const float *pool_all,
                              int64_t n_all, int64_t local_off, void *grad_scores,
                              float *loss_out, void *workspace, size_t workspace_bytes,
                              void *stream) {
  SBOD_REQUIRE(B > 0 && P > 0 && C >= 2 && scores && npos_total && pool_all && loss_out,
               "sbod_multibox_mine_global: bad arguments (B=%d P=%d C=%d)", B, P, C);
  SBOD_REQUIRE(cls == SBOD_CLS_CE && (flags & SBOD_POOL_GLOBAL_NEG),
               "sbod_multibox_mine_global: only the CE global pool (SSD300) is mined across ranks");
  SBOD_REQUIRE(local_off >= 0 && local_off + static_cast<int64_t>(B) * P <= n_all,
               "sbod_multibox_mine_global: rows [%lld, %lld) outside the gathered pool of %lld",
               static_cast<long long>(local_off), static_cast<long long>(local_off + static_cast<int64_t>(B) * P),
               static_cast<long long>(n_all));
  SBOD_REQUIRE(dtype == SBOD_DT_F32 || dtype == SBOD_DT_BF16, "sbod_multibox_mine_global: dtype %d", dtype);
  LossWs ws = carve(workspace, B, P);
  if (workspace_bytes < ws.bytes) {
    set_error("sbod_multibox_mine_global: workspace %zu < %zu", workspace_bytes, ws.bytes);
    return SBOD_E_WORKSPACE;
  }
  return mine_and_finish(scores, dtype, B, P, C, nullptr, npos_total, reg, cls, flags, neg_pos_ratio,
                         reg_weight, pool_all, n_all, local_off, grad_scores, loss_out, ws, as_stream(stream));
}

int sbod_aligned_overlap_f32(int kind, const float *b1, const float *b2, int64_t n,
                             float *overlap, float *grad_b1, float *grad_b2, void *stream) {
  SBOD_REQUIRE(kind >= 0 && kind <= 3 && n >= 0 && (n == 0 || (b1 && b2 && overlap)),
               "sbod_aligned_overlap_f32: bad arguments");
  if (n == 0) return SBOD_OK;
  hipLaunchKernelGGL(k_aligned, dim3((n + 255) / 256), dim3(256), 0, as_stream(stream), kind, b1,
                     b2, n, overlap, grad_b1, grad_b2);
  SBOD_LAUNCHED("k_aligned");
  return SBOD_OK;
}

int sbod_smooth_l1_f32(const float *pred, const float *target, int64_t n, float beta,
                       float *loss, float *grad, void *stream) {
  SBOD_REQUIRE(n >= 0 && (n == 0 || (pred && target && loss)), "sbod_smooth_l1_f32: bad arguments");
  if (n == 0) return SBOD_OK;
  hipLaunchKernelGGL(k_smooth_l1, dim3((n + 255) / 256), dim3(256), 0, as_stream(stream), pred,
                     target, n, beta, loss, grad);
  SBOD_LAUNCHED("k_smooth_l1");
  return SBOD_OK;
}

int sbod_focal_f32(int kind, const float *logits, const int64_t *target, int64_t rows, int C,
                   float alpha_fg, float alpha_bg, float gamma, float *row_loss, float *grad,
                   void *stream) {
  SBOD_REQUIRE(kind >= 0 && kind <= 2 && rows >= 0 && C >= 1 &&
                   (rows == 0 || (logits && target && row_loss)),
               "sbod_focal_f32: bad arguments");
  if (rows == 0) return SBOD_OK;
  hipLaunchKernelGGL(k_focal_rows, dim3((rows + 255) / 256), dim3(256), 0, as_stream(stream), kind,
                     logits, target, rows, C, alpha_fg, alpha_bg, gamma, row_loss, grad);
  SBOD_LAUNCHED("k_focal_rows");
  return SBOD_OK;
}

}  // extern "C"

SBOD_STAMP_EXPORT(loss)

#ifdef SBOD_BLOCK_STAMPS
// k_multibox's per-workgroup marks (diagnostic build): copies the first n workgroups' 8 marks out,
// then clears them.
extern "C" int sbod_debug_fin_marks(unsigned long long *seen, int n, unsigned long long *marks) {
  const int cap = static_cast<int>(SBOD_STAMP_REGION);
  if (seen && n > 0) hipMemcpyFromSymbol(seen, HIP_SYMBOL(g_fin_seen), sizeof(unsigned long long) * (n < cap ? n : cap));
  if (marks) hipMemcpyFromSymbol(marks, HIP_SYMBOL(g_fin_marks), sizeof(unsigned long long) * 8);
  void *sym = nullptr;
  if (hipGetSymbolAddress(&sym, HIP_SYMBOL(g_fin_seen)) == hipSuccess) hipMemset(sym, 0, sizeof(unsigned long long) * cap);
  if (hipGetSymbolAddress(&sym, HIP_SYMBOL(g_fin_marks)) == hipSuccess) hipMemset(sym, 0, sizeof(unsigned long long) * 8);
  return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}
extern "C" int sbod_debug_mb_marks(unsigned long long *host, int n) {
  const int cap = static_cast<int>(SBOD_STAMP_REGION);
  if (host && n > 0)
    hipMemcpyFromSymbol(host, HIP_SYMBOL(g_mb_marks), sizeof(unsigned long long) * 8 * (n < cap ? n : cap));
  void *sym = nullptr;
  if (hipGetSymbolAddress(&sym, HIP_SYMBOL(g_mb_marks)) == hipSuccess)
    hipMemset(sym, 0, sizeof(unsigned long long) * 8 * cap);
  return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}
#endif

// VOC 11-point mAP (metrics.calculate_mAP, metrics.py:8-145) on the device.
//
// The reference walks every class, sorts its detections by score and assigns TP/FP one detection
// at a time against the class's ground truth.  A detection only interacts with ground truth of
// its own (class, image), so:
//   1. keys: detections by (class, score desc) and by (class, image, score desc); ground truth
//      by (class, image) — three stable radix sorts (ties keep input order);
//   2. k_map_match: one thread per (class, image) detection group runs the reference's greedy
//      assignment in score order (max IoU with first-index ties, > threshold in double, the
//      difficult / already-detected rules) and writes TP/FP/none per detection;
//   3. k_map_ap: one block per class scans TP/FP in class score order (exact integer counts, the
//      reference's float32 precision / recall arithmetic), max-reduces precision for each of the
//      11 recall thresholds and averages them;  k_map_mean averages the class APs.
#include <hipcub/hipcub.hpp>

#include "sbod_common.h"

namespace sbod {

constexpr int kMapThreads = 256;
constexpr uint32_t kNoClass = 0xffu;

__device__ __forceinline__ int image_of(const int32_t *off, int B, int64_t i) {
  int lo = 0, hi = B - 1;   // largest b with off[b] <= i
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (off[mid] <= i) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

__global__ __launch_bounds__(kMapThreads) void k_map_det_keys(
    const int64_t *__restrict__ labels, const float *__restrict__ scores, const int32_t *__restrict__ off,
    int B, int C, int64_t D, unsigned long long *__restrict__ key_a, unsigned long long *__restrict__ key_b,
    int32_t *__restrict__ idx) {
  const int64_t d = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (d >= D) return;
  const int64_t l = labels[d];
  const bool valid = l >= 1 && l < C;
  const uint32_t cls = valid ? static_cast<uint32_t>(l) : kNoClass;
  const uint32_t sdesc = 0xffffffffu - f2ord(scores[d]);
  const uint32_t img = static_cast<uint32_t>(image_of(off, B, d));
  key_a[d] = (static_cast<unsigned long long>(cls) << 32) | sdesc;
  key_b[d] = (static_cast<unsigned long long>(cls) << 56) | (static_cast<unsigned long long>(img) << 32) | sdesc;
  idx[d] = static_cast<int32_t>(d);
}

__global__ __launch_bounds__(kMapThreads) void k_map_true_keys(
    const int64_t *__restrict__ labels, const int32_t *__restrict__ off, int B, int C, int64_t T,
    uint32_t *__restrict__ key_g, int32_t *__restrict__ idx) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= T) return;
  const int64_t l = labels[t];
  const uint32_t cls = (l >= 1 && l < C) ? static_cast<uint32_t>(l) : kNoClass;
  key_g[t] = (cls << 24) | static_cast<uint32_t>(image_of(off, B, t));
  idx[t] = static_cast<int32_t>(t);
}

// first index in a sorted u32 array with value >= v
__device__ __forceinline__ int64_t lower_u32(const uint32_t *a, int64_t n, uint32_t v) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ int64_t lower_u64(const unsigned long long *a, int64_t n, unsigned long long v) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// metrics.find_jaccard_overlap(detection [1,4], objects [n,4]) element (metrics.py:208-252)
__device__ __forceinline__ float det_iou(const Box4 &d, const Box4 &o) {
  float iw = fminf(d.c, o.c) - fmaxf(d.a, o.a);
  iw = iw < 0.f ? 0.f : iw;
  float ih = fminf(d.d, o.d) - fmaxf(d.b, o.b);
  ih = ih < 0.f ? 0.f : ih;
  const float dx = d.c - d.a, dy = d.d - d.b;
  const float ox = o.c - o.a, oy = o.d - o.b;
  const float inner = iw * ih;
  float ov = inner / (dx * dy + ox * oy - inner + kIouEps);
  if (fabsf(dx) < kIouEps && fabsf(dy) < kIouEps) ov = 0.f;
  if (ox < kIouEps && oy < kIouEps) ov = -1.f;
  return ov;
}

// One thread per (class, image) group of the (class, image, score desc) order.
__global__ __launch_bounds__(kMapThreads) void k_map_match(
    const unsigned long long *__restrict__ key_b, const int32_t *__restrict__ idx_b, int64_t D,
    const float *__restrict__ det_boxes, const uint32_t *__restrict__ key_g, const int32_t *__restrict__ idx_g,
    int64_t T, const float *__restrict__ true_boxes, const uint8_t *__restrict__ diff, double threshold,
    uint8_t *__restrict__ detected, uint8_t *__restrict__ flag) {
  const int64_t p = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (p >= D) return;
  const unsigned long long grp = key_b[p] >> 32;
  if (p > 0 && (key_b[p - 1] >> 32) == grp) return;       // not the first of its group
  const uint32_t cls = static_cast<uint32_t>(grp >> 24);
  if (cls == kNoClass) return;
  const uint32_t gkey = (cls << 24) | static_cast<uint32_t>(grp & 0xffffffu);
  const int64_t g0 = lower_u32(key_g, T, gkey);
  const int64_t g1 = lower_u32(key_g, T, gkey + 1u);
  for (int64_t q = p; q < D && (key_b[q] >> 32) == grp; ++q) {
    const int32_t d = idx_b[q];
    if (g0 == g1) {                                   // no object of this class in the image
      flag[d] = 2;
      continue;
    }
    const Box4 db = ld4(det_boxes + 4 * static_cast<int64_t>(d));
    float best = 0.f;
    int64_t bi = -1;
    for (int64_t g = g0; g < g1; ++g) {
      const float ov = det_iou(db, ld4(true_boxes + 4 * static_cast<int64_t>(idx_g[g])));
      if (bi < 0 || ov > best) {                      // torch.max: first index on ties
        best = ov;
        bi = g;
      }
    }
    const int32_t t = idx_g[bi];
    if (static_cast<double>(best) > threshold) {      // max_overlap.item() > threshold (:108)
      if (diff[t] == 0) {
        if (detected[t] == 0) {
          flag[d] = 1;
          detected[t] = 1;
        } else {
          flag[d] = 2;
        }
      } else {
        flag[d] = 0;                                  // difficult: neither TP nor FP
      }
    } else {
      flag[d] = 2;
    }
  }
}

// One block per class c = blockIdx.x + 1.
__global__ __launch_bounds__(kMapThreads) void k_map_ap(
    const unsigned long long *__restrict__ key_a, const int32_t *__restrict__ idx_a, int64_t D,
    const uint32_t *__restrict__ key_g, const int32_t *__restrict__ idx_g, int64_t T,
    const uint8_t *__restrict__ diff, const uint8_t *__restrict__ flag, const float *__restrict__ rthr,
    float *__restrict__ ap) {
  __shared__ uint32_t s_tp[kMapThreads], s_fp[kMapThreads];
  __shared__ float s_max[11][kMapThreads / 64];
  __shared__ uint32_t s_easy[kMapThreads / 64];
  __shared__ uint32_t s_carry[2];
  const int c = blockIdx.x + 1, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const unsigned long long cls = static_cast<unsigned long long>(c) << 32;
  const int64_t a0 = lower_u64(key_a, D, cls), a1 = lower_u64(key_a, D, cls + (1ull << 32));
  const int64_t g0 = lower_u32(key_g, T, static_cast<uint32_t>(c) << 24);
  const int64_t g1 = lower_u32(key_g, T, static_cast<uint32_t>(c + 1) << 24);
  if (a0 == a1) {                                    // no detection of this class: AP stays 0
    if (tid == 0) ap[c - 1] = 0.f;
    return;
  }
  // easy objects of the class
  uint32_t easy = 0;
  for (int64_t g = g0 + tid; g < g1; g += kMapThreads) easy += diff[idx_g[g]] == 0 ? 1u : 0u;
  for (int o = 32; o > 0; o >>= 1) easy += __shfl_xor(easy, o, 64);
  if (lane == 0) s_easy[wv] = easy;
  if (tid == 0) s_carry[0] = s_carry[1] = 0;
  __syncthreads();
  const float n_easy = static_cast<float>(s_easy[0] + s_easy[1] + s_easy[2] + s_easy[3]);
  float rt[11], pmax[11];
#pragma unroll
  for (int t = 0; t < 11; ++t) {
    rt[t] = rthr[t];
    pmax[t] = -1.f;          // "no recall >= t yet" (precision is never negative)
  }
  for (int64_t base = a0; base < a1; base += kMapThreads) {
    const int64_t p = base + tid;
    const uint8_t f = p < a1 ? flag[idx_a[p]] : 0;
    s_tp[tid] = f == 1 ? 1u : 0u;
    s_fp[tid] = f == 2 ? 1u : 0u;
    __syncthreads();
    for (int o = 1; o < kMapThreads; o <<= 1) {       // inclusive block scan (Hillis-Steele)
      const uint32_t vt = tid >= o ? s_tp[tid - o] : 0u, vf = tid >= o ? s_fp[tid - o] : 0u;
      __syncthreads();
      s_tp[tid] += vt;
      s_fp[tid] += vf;
      __syncthreads();
    }
    const uint32_t ctp_i = s_carry[0] + s_tp[tid], cfp_i = s_carry[1] + s_fp[tid];
    if (p < a1) {
      // float32 arithmetic of metrics.py:121-125
      const float ctp = static_cast<float>(ctp_i), cfp = static_cast<float>(cfp_i);
      const float prec = ctp / ((ctp + cfp) + 1e-10f);
      const float rec = ctp / n_easy;
#pragma unroll
      for (int t = 0; t < 11; ++t)
        if (rec >= rt[t]) pmax[t] = fmaxf(pmax[t], prec);
    }
    __syncthreads();
    if (tid == kMapThreads - 1) {
      s_carry[0] = ctp_i;
      s_carry[1] = cfp_i;
    }
    __syncthreads();
  }
#pragma unroll
  for (int t = 0; t < 11; ++t) {
    float v = pmax[t];
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    if (lane == 0) s_max[t][wv] = v;
  }
  __syncthreads();
  if (tid == 0) {
    float sum = 0.f;
    for (int t = 0; t < 11; ++t) {
      const float m = fmaxf(fmaxf(s_max[t][0], s_max[t][1]), fmaxf(s_max[t][2], s_max[t][3]));
      sum += m < 0.f ? 0.f : m;      // no recall >= t: precision 0 (:133)
    }
    ap[c - 1] = sum / 11.f;
  }
}

__global__ void k_map_mean(const float *__restrict__ ap, int n, float *__restrict__ out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    float s = 0.f;
    for (int i = 0; i < n; ++i) s += ap[i];
    *out = s / static_cast<float>(n);
  }
}

struct MapWs {
  unsigned long long *ka, *kb, *ka_s, *kb_s;
  int32_t *ia, *ib, *ia_s, *ib_s, *ig, *ig_s;
  uint32_t *kg, *kg_s;
  uint8_t *flag, *detected;
  void *temp;
  size_t temp_bytes, bytes;
};

size_t map_temp_bytes(int64_t D, int64_t T) {
  size_t a = 0, b = 0;
  // size queries only; a failed query makes the workspace requirement unsatisfiable (loud) rather than small
  const hipError_t ea = hipcub::DeviceRadixSort::SortPairs(nullptr, a, static_cast<unsigned long long *>(nullptr),
                                     static_cast<unsigned long long *>(nullptr), static_cast<int32_t *>(nullptr),
                                     static_cast<int32_t *>(nullptr), static_cast<int>(D > 0 ? D : 1), 0, 64);
  const hipError_t eb = hipcub::DeviceRadixSort::SortPairs(nullptr, b, static_cast<uint32_t *>(nullptr), static_cast<uint32_t *>(nullptr),
                                     static_cast<int32_t *>(nullptr), static_cast<int32_t *>(nullptr),
                                     static_cast<int>(T > 0 ? T : 1), 0, 32);
  if (ea != hipSuccess || eb != hipSuccess) return SIZE_MAX / 2;
  return a > b ? a : b;
}

MapWs map_carve(void *base, int64_t D, int64_t T) {
  MapWs w{};
  char *p = static_cast<char *>(base);
  size_t off = 0;
  auto take = [&](size_t bytes) { char *r = p ? p + off : nullptr; off += align_up(bytes > 0 ? bytes : 1); return r; };
  const size_t d = static_cast<size_t>(D > 0 ? D : 1), t = static_cast<size_t>(T > 0 ? T : 1);
  w.ka = reinterpret_cast<unsigned long long *>(take(d * 8));
  w.kb = reinterpret_cast<unsigned long long *>(take(d * 8));
  w.ka_s = reinterpret_cast<unsigned long long *>(take(d * 8));
  w.kb_s = reinterpret_cast<unsigned long long *>(take(d * 8));
  w.ia = reinterpret_cast<int32_t *>(take(d * 4));
  w.ib = reinterpret_cast<int32_t *>(take(d * 4));
  w.ia_s = reinterpret_cast<int32_t *>(take(d * 4));
  w.ib_s = reinterpret_cast<int32_t *>(take(d * 4));
  w.kg = reinterpret_cast<uint32_t *>(take(t * 4));
  w.kg_s = reinterpret_cast<uint32_t *>(take(t * 4));
  w.ig = reinterpret_cast<int32_t *>(take(t * 4));
  w.ig_s = reinterpret_cast<int32_t *>(take(t * 4));
  w.flag = reinterpret_cast<uint8_t *>(take(d));
  w.detected = reinterpret_cast<uint8_t *>(take(t));
  w.temp_bytes = map_temp_bytes(D, T);
  w.temp = take(w.temp_bytes);
  w.bytes = off;
  return w;
}

}  // namespace sbod

using namespace sbod;

extern "C" {

size_t sbod_map_workspace_bytes(int64_t n_det, int64_t n_true) { return map_carve(nullptr, n_det, n_true).bytes; }

int sbod_map_f32(const float *det_boxes, const int64_t *det_labels, const float *det_scores,
                 const int32_t *det_offsets, const float *true_boxes, const int64_t *true_labels,
                 const uint8_t *true_difficulties, const int32_t *true_offsets, int B, int C,
                 int64_t n_det, int64_t n_true, double threshold, const float *recall_thresholds,
                 float *ap, float *mean_ap, void *workspace, size_t workspace_bytes, void *stream) {
  SBOD_REQUIRE(B > 0 && C >= 2 && C < 255 && n_det >= 0 && n_true >= 0 && det_offsets && true_offsets &&
                   recall_thresholds && ap && mean_ap,
               "sbod_map_f32: bad arguments (B=%d C=%d D=%lld T=%lld)", B, C, static_cast<long long>(n_det),
               static_cast<long long>(n_true));
  SBOD_REQUIRE(B < (1 << 24) && n_det < (1ll << 31) && n_true < (1ll << 31), "sbod_map_f32: sizes too large");
  SBOD_REQUIRE(n_det == 0 || (det_boxes && det_labels && det_scores), "sbod_map_f32: detections are NULL");
  SBOD_REQUIRE(n_true == 0 || (true_boxes && true_labels && true_difficulties), "sbod_map_f32: ground truth is NULL");
  MapWs w = map_carve(workspace, n_det, n_true);
  if (workspace == nullptr || workspace_bytes < w.bytes) {
    set_error("sbod_map_f32: workspace %zu < %zu", workspace_bytes, w.bytes);
    return SBOD_E_WORKSPACE;
  }
  hipStream_t s = as_stream(stream);
  const int nb_d = static_cast<int>((n_det + kMapThreads - 1) / kMapThreads);
  const int nb_t = static_cast<int>((n_true + kMapThreads - 1) / kMapThreads);
  if (n_det > 0) {
    hipLaunchKernelGGL(k_map_det_keys, dim3(nb_d), dim3(kMapThreads), 0, s, det_labels, det_scores, det_offsets,
                       B, C, n_det, w.ka, w.kb, w.ia);
    SBOD_LAUNCHED("k_map_det_keys");
    if (hipMemcpyAsync(w.ib, w.ia, static_cast<size_t>(n_det) * 4, hipMemcpyDeviceToDevice, s) != hipSuccess)
      return launch_status("hipMemcpyAsync(map idx)");
  }
  if (n_true > 0) {
    hipLaunchKernelGGL(k_map_true_keys, dim3(nb_t), dim3(kMapThreads), 0, s, true_labels, true_offsets, B, C,
                       n_true, w.kg, w.ig);
    SBOD_LAUNCHED("k_map_true_keys");
  }
  size_t tb = w.temp_bytes;
  if (n_det > 0) {
    if (hipcub::DeviceRadixSort::SortPairs(w.temp, tb, w.ka, w.ka_s, w.ia, w.ia_s, static_cast<int>(n_det), 0, 64,
                                           s) != hipSuccess)
      return launch_status("map sort (class, score)");
    tb = w.temp_bytes;
    if (hipcub::DeviceRadixSort::SortPairs(w.temp, tb, w.kb, w.kb_s, w.ib, w.ib_s, static_cast<int>(n_det), 0, 64,
                                           s) != hipSuccess)
      return launch_status("map sort (class, image, score)");
  }
  if (n_true > 0) {
    tb = w.temp_bytes;
    if (hipcub::DeviceRadixSort::SortPairs(w.temp, tb, w.kg, w.kg_s, w.ig, w.ig_s, static_cast<int>(n_true), 0, 32,
                                           s) != hipSuccess)
      return launch_status("map sort (ground truth)");
    if (hipMemsetAsync(w.detected, 0, static_cast<size_t>(n_true), s) != hipSuccess)
      return launch_status("hipMemsetAsync(map detected)");
  }
  if (n_det > 0) {
    hipLaunchKernelGGL(k_map_match, dim3(nb_d), dim3(kMapThreads), 0, s, w.kb_s, w.ib_s, n_det, det_boxes, w.kg_s,
                       w.ig_s, n_true, true_boxes, true_difficulties, threshold, w.detected, w.flag);
    SBOD_LAUNCHED("k_map_match");
  }
  hipLaunchKernelGGL(k_map_ap, dim3(C - 1), dim3(kMapThreads), 0, s, w.ka_s, w.ia_s, n_det, w.kg_s, w.ig_s, n_true,
                     true_difficulties, w.flag, recall_thresholds, ap);
  SBOD_LAUNCHED("k_map_ap");
  hipLaunchKernelGGL(k_map_mean, dim3(1), dim3(64), 0, s, ap, C - 1, mean_ap);
  SBOD_LAUNCHED("k_map_mean");
  return SBOD_OK;
}

}  // extern "C"

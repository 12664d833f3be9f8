// Shared device/host helpers for libsbod_hip.so (gfx950 only).
//
// Numerics contract: the library is compiled with -ffp-contract=off and IEEE division, and
// every expression that feeds an integer decision (IoU -> argmax, NMS suppression, label
// thresholds) is written in the reference's evaluation order, so those decisions are the
// reference CPU path's bit for bit.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdint>
#include <cstdio>
#include <tuple>

#include "sbod.h"

namespace sbod {

void set_error(const char *fmt, ...);
int launch_status(const char *what);  // hipGetLastError -> SBOD_OK / SBOD_E_HIP
// Rows per tile of a one-round kernel over B images x P rows (k_multibox, k_det_prepare): every
// workgroup of such a launch loads, computes and stores in lockstep, so it lasts as long as its
// busiest CU.  The tile is sized for the fewest workgroups that give every CU the same count (k
// per CU, k <= 6) as long as a tile stays within max_rows — SSD512 (P = 10,248) at B = 32: 1,536
// tiles of 216 rows, six per CU, instead of 1,312 of 256 (five or six per CU); at B = 16: 768
// (three per CU) instead of 656 (two or three) — else max_rows.  A multiple of 8 rows (whole
// 16-byte chunks of fp32 and bf16 rows when P % 8 == 0), at least min_rows.
int balanced_rows(int B, int P, int max_rows, int min_rows);

constexpr int kWave = 64;
constexpr float kIouEps = 1e-5f;  // metrics.py:233 EPS (compared as float32, like torch)

#define SBOD_REQUIRE(cond, ...)            \
  do {                                      \
    if (!(cond)) {                          \
      ::sbod::set_error(__VA_ARGS__);       \
      return SBOD_E_INVALID;                \
    }                                       \
  } while (0)

#define SBOD_LAUNCHED(what)                       \
  do {                                            \
    int _st = ::sbod::launch_status(what);        \
    if (_st != SBOD_OK) return _st;               \
  } while (0)

inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

struct SpanRing;

// Brackets a launch with HIP events on its stream when sbod_timing_enable() selected it.
// With `attached` the scope's launch carries the two events itself (hipExtLaunchKernelGGL(...,
// kt.start(), kt.stop(), 0, ...)): the runtime stamps them at the dispatch's own start and end, so
// the measured time is the kernel's, without the gap between a separately recorded event and
// the dispatch.  Without it the events are recorded around the scope's launches.
class KernelTimer {
 public:
  KernelTimer(const char *name, hipStream_t s, bool attached = false);
  ~KernelTimer();
  KernelTimer(const KernelTimer &) = delete;
  KernelTimer &operator=(const KernelTimer &) = delete;
  hipEvent_t start() const { return attached_ ? start_ : nullptr; }
  hipEvent_t stop() const { return attached_ ? stop_ : nullptr; }
  // Under hipGraph capture (where a dispatch cannot carry events and this runtime refuses
  // external event nodes) a selected kernel instead gets a device span ring (SpanRing, below)
  // that the kernel itself writes on every replay; nullptr when not selected.
  SpanRing *span() const { return span_; }

 private:
  const char *name_;
  hipStream_t stream_;
  bool attached_;
  hipEvent_t start_ = nullptr, stop_ = nullptr;
  SpanRing *span_ = nullptr;
};

// Kernel-side span recording (see KernelTimer::span).  A captured kernel is replayed many
// times and the host never writes the record between replays: every launch overwrites, per
// workgroup, its own {start, end} pair (plain stores by thread 0, no atomics — thousands of
// same-address atomics would themselves stretch the kernel), and workgroup 0 the grid size; the
// host reduces min(start) / max(end) after the replay.
constexpr int kSpanBlocks = 16384;   // workgroups recorded per launch (ids beyond are not)
struct SpanRing {
  unsigned long long nblocks;
  unsigned long long t[kSpanBlocks][2];
};

__device__ __forceinline__ unsigned span_block_id() {
  return blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
}
// (The grid values are read outside the thread-0 branch: a uniform value first read inside a
// divergent branch becomes a per-lane phi at the join, and every later use of it — blockIdx,
// gridDim, addresses built from them — is demoted from scalar to vector registers and loads.)
__device__ __forceinline__ void span_begin(SpanRing *r) {
  if (r == nullptr) return;
  const unsigned blk = span_block_id();
  const unsigned long long nb = static_cast<unsigned long long>(gridDim.x) * gridDim.y * gridDim.z;
  if (threadIdx.x == 0) {
    if (blk == 0) r->nblocks = nb;
    if (blk < kSpanBlocks) r->t[blk][0] = __builtin_amdgcn_s_memrealtime();
  }
}
// Synchronises the workgroup; must be reached by all of its threads.  Each thread first waits
// for its own outstanding memory operations (s_waitcnt 0: stores acknowledged by L2), so the end
// stamp follows the block's stores.  (Not __threadfence(): a device-scope release writes the
// XCD's L2 back on every block, ~10x the kernel's own time on MI355X.)
__device__ __forceinline__ void span_end(SpanRing *r) {
  if (r == nullptr) return;
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  const unsigned blk = span_block_id();
  if (threadIdx.x == 0 && blk < kSpanBlocks) r->t[blk][1] = __builtin_amdgcn_s_memrealtime();
}

// Launch through a KernelTimer: a timed launch carries the timer's events on the dispatch
// (hipExtLaunchKernel); an untimed one is a plain hipLaunchKernel, the form stream capture
// records into a hipGraph kernel node.  Arguments are converted to the kernel's parameter types
// first, as the triple-chevron launch does.
template <typename... KArgs, typename... Args>
inline void tlaunch(const KernelTimer &kt, void (*kernel)(KArgs...), dim3 grid, dim3 block,
                    size_t lds, hipStream_t s, Args... args) {
  static_assert(sizeof...(KArgs) == sizeof...(Args), "tlaunch: argument count");
  auto conv = std::tuple<KArgs...>{static_cast<KArgs>(args)...};
  void *a[sizeof...(KArgs) > 0 ? sizeof...(KArgs) : 1];
  std::apply([&a](auto &...v) {
    int i = 0;
    ((a[i++] = static_cast<void *>(&v)), ...);
  }, conv);
  const void *k = reinterpret_cast<const void *>(kernel);
  if (kt.start())
    (void)hipExtLaunchKernel(k, grid, block, a, lds, s, kt.start(), kt.stop(), 0);
  else
    (void)hipLaunchKernel(k, grid, block, a, lds, s);
}

inline size_t align_up(size_t x, size_t a = 256) { return (x + a - 1) / a * a; }

// Address `off` bytes into a caller workspace, or nullptr in a size-only query (base == nullptr):
// the carve functions never do pointer arithmetic on a null base.
template <typename T>
inline T *ws_at(void *base, size_t off) {
  return base ? reinterpret_cast<T *>(static_cast<char *>(base) + off) : nullptr;
}

inline int next_pow2_host(int x) {
  int p = 1;
  while (p < x) p <<= 1;
  return p;
}

// Monotone float <-> uint32 mapping: a < b  <=>  ord(a) < ord(b) (for non-NaN floats).
__device__ __forceinline__ uint32_t f2ord(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(uint32_t k) {
  uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
  return __uint_as_float(u);
}

__device__ __forceinline__ unsigned long long shfl_xor_u64(unsigned long long v, int m) {
  uint32_t lo = __shfl_xor(static_cast<uint32_t>(v), m, kWave);
  uint32_t hi = __shfl_xor(static_cast<uint32_t>(v >> 32), m, kWave);
  return (static_cast<unsigned long long>(hi) << 32) | lo;
}

__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    unsigned long long o = shfl_xor_u64(v, m);
    v = o > v ? o : v;
  }
  return v;
}

// Wave-wide max of a u32, valid in every lane: DPP quad swaps and mirrors inside each row of 16,
// then row broadcasts (gfx9 DPP) — no LDS traffic, a few cycles per step.
template <int kCtrl, int kRowMask>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t x) {
  return static_cast<uint32_t>(
      __builtin_amdgcn_update_dpp(static_cast<int>(x), static_cast<int>(x), kCtrl, kRowMask, 0xf, false));
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  v = max(v, dpp_u32<0xB1, 0xf>(v));    // quad_perm [1,0,3,2]
  v = max(v, dpp_u32<0x4E, 0xf>(v));    // quad_perm [2,3,0,1]
  v = max(v, dpp_u32<0x141, 0xf>(v));   // row_half_mirror
  v = max(v, dpp_u32<0x140, 0xf>(v));   // row_mirror: every lane of a row holds the row max
  v = max(v, dpp_u32<0x142, 0xa>(v));   // row_bcast:15 -> rows 1, 3
  v = max(v, dpp_u32<0x143, 0xc>(v));   // row_bcast:31 -> rows 2, 3: lane 63 holds the wave max
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), 63));
}

// Sum over each 32-lane half of the wave with DPP (no LDS): quad swaps and mirrors give every
// lane its row-of-16 sum, then row_bcast:15 adds row 0 into row 1 and row 2 into row 3 (rows 0
// and 2 add 0).  The lower half's total is in lanes 16..31, the upper half's in lanes 48..63.
template <int kCtrl, int kRowMask>
__device__ __forceinline__ float dpp_f32_or0(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), kCtrl, kRowMask, 0xf, false));
}
__device__ __forceinline__ float half_sum_f32(float v) {
  v += dpp_f32_or0<0xB1, 0xf>(v);    // quad_perm [1,0,3,2]
  v += dpp_f32_or0<0x4E, 0xf>(v);    // quad_perm [2,3,0,1]
  v += dpp_f32_or0<0x141, 0xf>(v);   // row_half_mirror
  v += dpp_f32_or0<0x140, 0xf>(v);   // row_mirror
  return v + dpp_f32_or0<0x142, 0xa>(v);   // row_bcast:15 -> rows 1, 3
}

__device__ __forceinline__ float wave_sum_f32(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, kWave);
  return v;
}

__device__ __forceinline__ int wave_sum_i32(int v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, kWave);
  return v;
}

// Block-wide sum (blockDim.x multiple of 64, <= 1024); result valid in every thread.
template <typename T>
__device__ __forceinline__ T block_sum(T v, T *scratch /* >= 16 */) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, kWave);
  __syncthreads();
  if (lane == 0) scratch[w] = v;
  __syncthreads();
  T s = 0;
  for (int i = 0; i < nw; ++i) s += scratch[i];
  return s;
}

// ----------------------------------------------------------------------------- box codecs
// dataset/transforms.py:37-45 / 69-83 in the reference's evaluation order.
struct Box4 {
  float a, b, c, d;
};

// cxcy_to_xy(gcxgcy_to_cxcy(g, prior)).  c = g_xy * p_wh / 10 + p_xy; wh = exp(g_wh / 5) * p_wh.
__device__ __forceinline__ Box4 decode_tenfive_xy(Box4 g, Box4 p) {
  float cx = g.a * p.c / 10.f + p.a;
  float cy = g.b * p.d / 10.f + p.b;
  float w = expf(g.c / 5.f) * p.c;
  float h = expf(g.d / 5.f) * p.d;
  return Box4{cx - w / 2.f, cy - h / 2.f, cx + w / 2.f, cy + h / 2.f};
}

// xy_to_cxcy (transforms.py:26-34).
__device__ __forceinline__ Box4 xy_to_cxcy(Box4 x) {
  return Box4{(x.c + x.a) / 2.f, (x.d + x.b) / 2.f, x.c - x.a, x.d - x.b};
}

// cxcy_to_gcxgcy (transforms.py:48-66): (c - pc) / (pwh / 10), log(wh / pwh) * 5.
__device__ __forceinline__ Box4 encode_tenfive(Box4 c, Box4 p) {
  return Box4{(c.a - p.a) / (p.c / 10.f), (c.b - p.b) / (p.d / 10.f), logf(c.c / p.c) * 5.f,
              logf(c.d / p.d) * 5.f};
}

__device__ __forceinline__ Box4 ld4(const float *p) {
  float4 v = *reinterpret_cast<const float4 *>(p);
  return Box4{v.x, v.y, v.z, v.w};
}
// A uniform load through the constant address space: becomes a scalar (s_load) when the address
// is wave-uniform.  Only for data no workgroup writes during the kernel.
__device__ __forceinline__ Box4 ld4_uniform(const float *p) {
  const __attribute__((address_space(4))) float *q = (const __attribute__((address_space(4))) float *)(p);
  return Box4{q[0], q[1], q[2], q[3]};
}
__device__ __forceinline__ int32_t ld_i32_uniform(const int32_t *p) {
  return *(const __attribute__((address_space(4))) int32_t *)(p);
}
__device__ __forceinline__ void st4(float *p, Box4 b) {
  *reinterpret_cast<float4 *>(p) = make_float4(b.a, b.b, b.c, b.d);
}
// Streaming (non-temporal) stores for large one-shot outputs: written through instead of left
// dirty in the XCD's L2, so the write-back overlaps the kernel instead of following it.
typedef float f32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st4_nt(float *p, Box4 b) {
  f32x4_t v = {b.a, b.b, b.c, b.d};
  __builtin_nontemporal_store(v, reinterpret_cast<f32x4_t *>(p));
}
__device__ __forceinline__ void st4_nt(float *p, float4 b) { st4_nt(p, Box4{b.x, b.y, b.z, b.w}); }
__device__ __forceinline__ void st_nt(unsigned long long *p, unsigned long long v) { __builtin_nontemporal_store(v, p); }

// Write-through (sc1) stores and L1-bypassing (sc1) loads for in-launch hand-offs between
// workgroups (MI355X_MICROARCH.md, inter-workgroup visibility: every handed-off byte stored sc1
// and drained by its storing wave before the signalling add; every load of it sc1).  <= 8 bytes:
// agent-scope relaxed atomics on global pointers (global_store/load ... sc1); 16 bytes: a raw
// buffer store with the sc1 cache-policy bit over a wave-uniform descriptor.
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned int gu32;
__device__ __forceinline__ void st_wt_u64(unsigned long long *p, unsigned long long v) {
  __hip_atomic_store((gu64 *)(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_wt_u64(const unsigned long long *p) {
  return __hip_atomic_load((gu64 *)(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt_u32(int32_t *p, uint32_t v) {
  __hip_atomic_store((gu32 *)(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_wt_u32(const int32_t *p) {
  return __hip_atomic_load((gu32 *)(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Wait for every outstanding vector-memory operation of the calling wave (stores acknowledged,
// atomics performed) with a compiler memory barrier: no memory access moves across it (a bare
// __builtin_amdgcn_s_waitcnt is not a compiler barrier).
// Per-image ground-truth lists travelling in kernel arguments (the collate_fn batch, one device
// tensor pair per image): k_gt_pack copies them into the packed layout, the list form of the
// matcher reads them in place.  kPackImgs images per launch (1,284 B of kernel arguments).
constexpr int kPackImgs = 64;
struct GtPackArgs {
  const float *boxes[kPackImgs];
  const int64_t *labels[kPackImgs];
  int32_t off[kPackImgs + 1];    // destination row offsets (absolute)
};

__device__ __forceinline__ void drain_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
constexpr int kCpolSc1 = 16;   // gfx950 cache-policy bit SC1 in the buffer intrinsics' aux word
// 16 bytes written through at byte offset `off` of the wave-uniform region [base, base + bytes).
__device__ __forceinline__ void st_wt_b128(void *base, uint32_t bytes, uint32_t off, u32x4_t v) {
  const auto r = __builtin_amdgcn_make_buffer_rsrc(base, static_cast<short>(0), static_cast<int>(bytes), 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(v, r, static_cast<int>(off), 0, kCpolSc1);
}

// [n] floats global -> LDS, 16 bytes per lane when the source is 16-byte aligned.
// Global -> LDS copy of n floats by the whole block.  Loads are issued in batches of 8 per
// thread into registers before any LDS store, so a thread has 8 HBM requests in flight instead
// of one round trip per element (the compiler cannot reorder loads past stores to `dst`).
// kBatch = loads per thread per batch: a caller that knows its tile (256 rows x C <= 4 kBatch
// floats per thread) passes the exact count, so no lane issues clamped duplicate requests.
template <int kBatch = 8>
__device__ __forceinline__ void tile_load_f32(float *__restrict__ dst, const float *__restrict__ src, int n) {
  const int nt = blockDim.x;
  if ((reinterpret_cast<uintptr_t>(src) & 15) == 0) {
    const int n4 = n >> 2;
    const float4 *s4 = reinterpret_cast<const float4 *>(src);
    float4 *d4 = reinterpret_cast<float4 *>(dst);
    // loads AND stores are unconditional (index clamped; an out-of-range lane rewrites the last
    // element with the value it holds): a guarded store lets the compiler sink each load into
    // its store's branch, which serialises the batch into one memory round trip per element
    for (int base = 0; base < n4; base += kBatch * nt) {
      float4 r[kBatch];
#pragma unroll
      for (int k = 0; k < kBatch; ++k) r[k] = s4[min(base + k * nt + static_cast<int>(threadIdx.x), n4 - 1)];
#pragma unroll
      for (int k = 0; k < kBatch; ++k) d4[min(base + k * nt + static_cast<int>(threadIdx.x), n4 - 1)] = r[k];
    }
    for (int i = (n4 << 2) + threadIdx.x; i < n; i += nt) dst[i] = src[i];
  } else {
    for (int base = 0; base < n; base += kBatch * nt) {
      float r[kBatch];
#pragma unroll
      for (int k = 0; k < kBatch; ++k) r[k] = src[min(base + k * nt + static_cast<int>(threadIdx.x), n - 1)];
#pragma unroll
      for (int k = 0; k < kBatch; ++k) dst[min(base + k * nt + static_cast<int>(threadIdx.x), n - 1)] = r[k];
    }
  }
}

}  // namespace sbod

// ----------------------------------------------------------------------------- debug timeline
// -DSBOD_BLOCK_STAMPS (diagnostic builds only; scripts/build_stamps_lib.sh): the kernel armed
// by sbod_debug_stamps_<tu>(arm) records, per workgroup, its wall-clock start and end
// (s_memrealtime, 100 MHz) and the CU it ran on, so launch ramp, per-block duration and tail
// can be read off one dispatch.  Compiles to nothing otherwise.
// Debug aid (off by default): -DSBOD_PHASE_CLOCKS prints per-phase cycle stamps of a few blocks.
#ifdef SBOD_PHASE_CLOCKS
// (wall clock: s_memrealtime, 100 MHz; every 8th tile of every 4th image)
#define SEG_PHASE(i) do { __syncthreads(); if (threadIdx.x == 0) ph[i] = __builtin_amdgcn_s_memrealtime(); } while (0)
#define PHASE_DECL long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0}
#define PHASE_PRINT_SEL (threadIdx.x == 0 && (blockIdx.x % 8) == 0 && (blockIdx.y % 4) == 0)
#else
#define SEG_PHASE(i) do { } while (0)
#define PHASE_DECL do { } while (0)
#endif

#ifdef SBOD_BLOCK_STAMPS
// Per-workgroup wall-clock stamps (diagnostic build): kernel ID (0..15) owns the region
// [ID * kStampRegion, +kStampRegion) workgroups of its translation unit's buffer and records only
// while bit ID of g_stamp_armed is set, so the kernels of one step (both graphs) can be recorded
// together and lined up on one clock (scripts/step_timeline.py).
#define SBOD_STAMP_REGION 4096u
#define SBOD_STAMP_CAP (16u * SBOD_STAMP_REGION)
#define SBOD_STAMP_DECL                                                  \
  static __device__ unsigned long long g_stamps[2 * SBOD_STAMP_CAP]; \
  static __device__ int g_stamp_armed = 0;
#define STAMP_BEGIN() const unsigned long long _st0 = __builtin_amdgcn_s_memrealtime()
// SYNC: 1 = the whole workgroup is still running (barrier first), 0 = the caller is the last wave
#define STAMP_END(ID, SYNC)                                                                      \
  do {                                                                                           \
    if (g_stamp_armed & (1 << (ID))) {                                                           \
      if (SYNC) __syncthreads();                                                                 \
      if ((threadIdx.x & 63) == 0 && ((SYNC) == 0 || threadIdx.x == 0)) {                        \
        const unsigned _blk = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);    \
        if (_blk < SBOD_STAMP_REGION) {                                                          \
          const unsigned _i = (ID) * SBOD_STAMP_REGION + _blk;                                   \
          g_stamps[2 * _i] = _st0;                                                               \
          g_stamps[2 * _i + 1] = (__builtin_amdgcn_s_memrealtime() & 0xffffffffffffull) |       \
                                 (static_cast<unsigned long long>(__smid() & 0xffff) << 48);    \
        }                                                                                        \
      }                                                                                          \
    }                                                                                            \
  } while (0)
// arm = bit mask of kernel IDs to record from now on; host (n > 0): copy the first n stamp pairs
// of the buffer out BEFORE clearing it.
#define SBOD_STAMP_EXPORT(TU)                                                                    \
  extern "C" int sbod_debug_stamps_##TU(int arm, unsigned long long *host, int n) {              \
    if (host && n > 0)                                                                           \
      hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 2 *           \
                          (n < static_cast<int>(SBOD_STAMP_CAP) ? n : SBOD_STAMP_CAP));     \
    void *_sym = nullptr;                                                                        \
    if (hipGetSymbolAddress(&_sym, HIP_SYMBOL(g_stamps)) == hipSuccess)                          \
      hipMemset(_sym, 0, sizeof(unsigned long long) * 2 * SBOD_STAMP_CAP);                       \
    hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_armed), &arm, sizeof(int));                             \
    return hipDeviceSynchronize() == hipSuccess ? 0 : -1;                                        \
  }
#else
#define SBOD_STAMP_DECL
#define STAMP_BEGIN() do { } while (0)
#define STAMP_END(ID, SYNC) do { } while (0)
#define SBOD_STAMP_EXPORT(TU)
#endif

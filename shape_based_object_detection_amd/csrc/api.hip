// Library plumbing: version, thread-local error string, launch checks, device-side grad scale.
#include <cstdarg>
#include <cstring>
#include <mutex>
#include <unordered_map>
#include <string>
#include <vector>

#include "sbod_common.h"

namespace sbod {

static thread_local char g_err[512] = "";

void set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int balanced_rows(int B, int P, int max_rows, int min_rows) {
  static int ncu = 0;   // CUs of the device (one model per process)
  if (ncu <= 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      return max_rows;
    ncu = n;
  }
  for (int k = 1; k <= 6; ++k) {
    const int tpi = (k * ncu + B - 1) / B;   // tiles per image
    const int rows = (((P + tpi - 1) / tpi) + 7) & ~7;
    if (rows <= max_rows) return rows < min_rows ? min_rows : rows;
  }
  return max_rows;
}

int launch_status(const char *what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return SBOD_E_HIP;
  }
  return SBOD_OK;
}

// An empty kernel (profiling calibration: the fixed per-dispatch cost a tool adds, MEASUREMENT
// in DESIGN.md / scripts/rocprof_overhead.py).
__global__ __launch_bounds__(64) void k_null() {}

// grad *= *scale unless *scale == 1 (every block reads the scalar and exits early).
template <typename T>
__global__ __launch_bounds__(256) void k_scale(T *__restrict__ g, int64_t n, const float *scale) {
  const float s = *scale;
  if (s == 1.0f) return;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    if constexpr (sizeof(T) == 4) {
      g[i] = g[i] * s;
    } else {
      float v = __uint_as_float(static_cast<uint32_t>(g[i]) << 16) * s;
      uint32_t u = __float_as_uint(v);
      u += 0x7fffu + ((u >> 16) & 1u);
      g[i] = static_cast<T>(u >> 16);
    }
  }
}

// Two buffers in one launch (the fused criterion's grad_locs and grad_scores).
template <typename T>
__global__ __launch_bounds__(256) void k_scale2(T *__restrict__ a, int64_t na, T *__restrict__ b,
                                                int64_t nb, const float *scale) {
  const float s = *scale;
  if (s == 1.0f) return;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < na + nb; i += stride) {
    T *p = i < na ? a + i : b + (i - na);
    if constexpr (sizeof(T) == 4) {
      *p = *p * s;
    } else {
      float v = __uint_as_float(static_cast<uint32_t>(*p) << 16) * s;
      uint32_t u = __float_as_uint(v);
      u += 0x7fffu + ((u >> 16) & 1u);
      *p = static_cast<T>(u >> 16);
    }
  }
}

// ---------------------------------------------------------------- kernel timing (bench aid)
// When a filter is set, KernelTimer brackets matching launches with HIP events recorded on the
// launch stream; sbod_timing_query() synchronises them and sums the elapsed times.  Events are
// pooled, so steady-state cost is two hipEventRecord calls per timed launch.
namespace {
std::mutex g_tmu;
std::string g_filter;
struct TimingRec {
  const char *name;
  hipEvent_t a, b;
  bool graph;   // captured into a hipGraph: the kernel writes span slot `slot` on every replay
  int slot;
};
// Span rings for kernels captured into graphs (SpanRing: per-launch {start, end} in
// s_memrealtime ticks, written by the kernel).  Allocated and initialised by
// sbod_timing_enable, never under capture; the host only reads them afterwards.
constexpr int kSpanSlots = 8;   // captured timed kernels (each record ~256 KB)
double g_realtime_hz = 100.0e6;   // replaced by hipDeviceAttributeWallClockRate at allocation
SpanRing *g_span_dev = nullptr;
int g_span_next = 0;
std::vector<TimingRec> g_recs;
int g_every = 1;                                  // time one launch in g_every (per kernel name)
std::unordered_map<std::string, long long> g_seen;
std::vector<hipEvent_t> g_pool;

hipEvent_t pooled_event() {
  if (!g_pool.empty()) {
    hipEvent_t e = g_pool.back();
    g_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}
}  // namespace

KernelTimer::KernelTimer(const char *name, hipStream_t s, bool attached)
    : name_(name), stream_(s), attached_(attached) {
  std::lock_guard<std::mutex> g(g_tmu);
  if (g_filter.empty() || (g_filter != "*" && g_filter != name)) return;
  if (g_every > 1 && (g_seen[name]++ % g_every) != 0) return;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) == hipSuccess && cs == hipStreamCaptureStatusActive) {
    attached_ = false;
    if (g_span_dev != nullptr && g_span_next < kSpanSlots) {
      const int slot = g_span_next++;
      span_ = g_span_dev + slot;
      g_recs.push_back({name, nullptr, nullptr, true, slot});
    }
    return;
  }
  start_ = pooled_event();
  if (attached_) {
    stop_ = pooled_event();
    if (!start_ || !stop_) start_ = stop_ = nullptr;
    return;
  }
  if (start_ && hipEventRecord(start_, s) != hipSuccess) start_ = nullptr;
}

KernelTimer::~KernelTimer() {
  if (!start_) return;
  std::lock_guard<std::mutex> g(g_tmu);
  if (attached_) {
    g_recs.push_back({name_, start_, stop_, false, -1});
    return;
  }
  hipEvent_t e = pooled_event();
  if (e && hipEventRecord(e, stream_) == hipSuccess) g_recs.push_back({name_, start_, e, false, -1});
}

}  // namespace sbod

extern "C" {

int sbod_timing_enable(const char *kernel_filter) {
  std::lock_guard<std::mutex> g(sbod::g_tmu);
  // eager records go back to the pool; records inside captured graphs stay (their events belong
  // to graph nodes) until sbod_timing_reset_graphs()
  std::vector<sbod::TimingRec> keep;
  for (auto &r : sbod::g_recs) {
    if (r.graph) {
      keep.push_back(r);
      continue;
    }
    sbod::g_pool.push_back(r.a);
    sbod::g_pool.push_back(r.b);
  }
  sbod::g_recs.swap(keep);
  sbod::g_seen.clear();
  sbod::g_filter = kernel_filter ? kernel_filter : "";
  if (!sbod::g_filter.empty() && sbod::g_span_dev == nullptr &&
      (hipMalloc(reinterpret_cast<void **>(&sbod::g_span_dev), sizeof(sbod::SpanRing) * sbod::kSpanSlots) != hipSuccess ||
       hipMemset(sbod::g_span_dev, 0, sizeof(sbod::SpanRing) * sbod::kSpanSlots) != hipSuccess)) {
    sbod::g_span_dev = nullptr;
    return sbod::launch_status("sbod_timing_enable(span records)");
  }
  if (!sbod::g_filter.empty()) {
    int dev = 0, khz = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) == hipSuccess && khz > 0)
      sbod::g_realtime_hz = 1e3 * khz;
  }
  return SBOD_OK;
}

double sbod_timing_clock_hz(void) { return sbod::g_realtime_hz; }

int sbod_timing_reset_graphs(void) {
  std::lock_guard<std::mutex> g(sbod::g_tmu);
  std::vector<sbod::TimingRec> keep;
  for (auto &r : sbod::g_recs)
    if (!r.graph) keep.push_back(r);
  sbod::g_recs.swap(keep);
  sbod::g_span_next = 0;   // the graphs holding the span pointers must be gone
  if (sbod::g_span_dev != nullptr &&   // no stale record can be read for a slot handed out again
      hipMemset(sbod::g_span_dev, 0, sizeof(sbod::SpanRing) * sbod::kSpanSlots) != hipSuccess)
    return sbod::launch_status("sbod_timing_reset_graphs");
  return SBOD_OK;
}

int sbod_timing_every(int n) {
  SBOD_REQUIRE(n >= 1, "sbod_timing_every: n must be >= 1");
  std::lock_guard<std::mutex> g(sbod::g_tmu);
  sbod::g_every = n;
  sbod::g_seen.clear();
  return SBOD_OK;
}

int sbod_timing_query(const char *kernel, int *launches, double *total_ms) {
  SBOD_REQUIRE(kernel && launches && total_ms, "sbod_timing_query: bad arguments");
  std::lock_guard<std::mutex> g(sbod::g_tmu);
  int n = 0;
  double tot = 0.0;
  for (auto &r : sbod::g_recs) {
    if (std::strcmp(r.name, kernel) != 0) continue;
    if (r.graph) {   // the latest completed launch of the captured kernel (read only)
      sbod::SpanRing *d = sbod::g_span_dev + r.slot;
      unsigned long long nb = 0;
      if (hipMemcpy(&nb, &d->nblocks, 8, hipMemcpyDeviceToHost) != hipSuccess)
        return sbod::launch_status("sbod_timing_query(span)");
      if (nb == 0 || nb > (1ull << 31)) continue;   // never replayed
      const size_t nr = nb < static_cast<unsigned long long>(sbod::kSpanBlocks) ? nb : sbod::kSpanBlocks;
      std::vector<unsigned long long> t(2 * nr);
      if (hipMemcpy(t.data(), d->t, 16 * nr, hipMemcpyDeviceToHost) != hipSuccess)
        return sbod::launch_status("sbod_timing_query(span)");
      unsigned long long lo = ~0ull, hi = 0ull;
      for (size_t i = 0; i < nr; ++i) {
        lo = t[2 * i] < lo ? t[2 * i] : lo;
        hi = t[2 * i + 1] > hi ? t[2 * i + 1] : hi;
      }
      if (hi <= lo) continue;
      tot += static_cast<double>(hi - lo) / sbod::g_realtime_hz * 1e3;
      ++n;
      continue;
    }
    float ms = 0.f;
    if (hipEventSynchronize(r.b) != hipSuccess || hipEventElapsedTime(&ms, r.a, r.b) != hipSuccess)
      return sbod::launch_status("sbod_timing_query");
    tot += ms;
    ++n;
  }
  *launches = n;
  *total_ms = tot;
  return SBOD_OK;
}

const char *sbod_version(void) { return "sbod-hip 0.1.0 (gfx950)"; }
int sbod_abi_version(void) { return SBOD_ABI_VERSION; }

int sbod_build_variants(void) {
#ifdef SBOD_VARIANT_ONE_LAUNCH
  return SBOD_VARIANT_ONE_LAUNCH_CRITERION;
#else
  return 0;
#endif
}

int sbod_null_kernel(int blocks, void *stream) {
  SBOD_REQUIRE(blocks > 0, "sbod_null_kernel: blocks %d", blocks);
  sbod::KernelTimer kt("k_null", sbod::as_stream(stream), true);
  sbod::tlaunch(kt, sbod::k_null, dim3(blocks), dim3(64), 0, sbod::as_stream(stream));
  SBOD_LAUNCHED("k_null");
  return SBOD_OK;
}
const char *sbod_last_error(void) { return sbod::g_err; }

int sbod_memcpy_d2h_async(void *dst_host, const void *src_dev, size_t bytes, void *stream) {
  SBOD_REQUIRE(bytes == 0 || (dst_host != nullptr && src_dev != nullptr), "sbod_memcpy_d2h_async: bad arguments");
  if (bytes == 0) return SBOD_OK;
  if (hipMemcpyAsync(dst_host, src_dev, bytes, hipMemcpyDeviceToHost, sbod::as_stream(stream)) != hipSuccess)
    return sbod::launch_status("sbod_memcpy_d2h_async");
  return SBOD_OK;
}

int sbod_graph_launch(void *graph_exec, void *stream) {
  SBOD_REQUIRE(graph_exec != nullptr, "sbod_graph_launch: null graph");
  if (hipGraphLaunch(reinterpret_cast<hipGraphExec_t>(graph_exec), sbod::as_stream(stream)) != hipSuccess)
    return sbod::launch_status("sbod_graph_launch");
  return SBOD_OK;
}

int sbod_event_record(void *event, void *stream) {
  SBOD_REQUIRE(event != nullptr, "sbod_event_record: null event");
  if (hipEventRecord(reinterpret_cast<hipEvent_t>(event), sbod::as_stream(stream)) != hipSuccess)
    return sbod::launch_status("sbod_event_record");
  return SBOD_OK;
}

int sbod_stream_wait(void *waiting_stream, void *on_stream) {
  if (waiting_stream == on_stream) return SBOD_OK;
  // one event per host thread and device: hipStreamWaitEvent binds to the record current at the
  // time of the call, so re-recording the same event for the next wait is safe
  thread_local hipEvent_t ev[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return sbod::launch_status("sbod_stream_wait");
  if (ev[dev] == nullptr && hipEventCreateWithFlags(&ev[dev], hipEventDisableTiming) != hipSuccess) {
    ev[dev] = nullptr;
    return sbod::launch_status("sbod_stream_wait(create)");
  }
  if (hipEventRecord(ev[dev], sbod::as_stream(on_stream)) != hipSuccess ||
      hipStreamWaitEvent(sbod::as_stream(waiting_stream), ev[dev], 0) != hipSuccess)
    return sbod::launch_status("sbod_stream_wait");
  return SBOD_OK;
}

int sbod_stream_abort_capture(void *stream) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(sbod::as_stream(stream), &cs) != hipSuccess)
    return sbod::launch_status("sbod_stream_abort_capture");
  if (cs == hipStreamCaptureStatusNone) return SBOD_OK;
  hipGraph_t g = nullptr;
  (void)hipStreamEndCapture(sbod::as_stream(stream), &g);   // an invalidated capture ends with an error
  if (g != nullptr) (void)hipGraphDestroy(g);
  (void)hipGetLastError();
  cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(sbod::as_stream(stream), &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
    sbod::set_error("sbod_stream_abort_capture: the stream is still capturing (status %d): use another stream",
                    static_cast<int>(cs));
    return SBOD_E_HIP;
  }
  return SBOD_OK;
}

int sbod_scale_inplace(void *grad, int dtype, int64_t n, const float *scale, void *stream) {
  SBOD_REQUIRE(n >= 0 && scale != nullptr, "sbod_scale_inplace: bad arguments");
  if (n == 0) return SBOD_OK;
  int64_t blocks = (n + 255) / 256;
  // the usual upstream gradient is 1 and every block exits at once: the grid is kept small,
  // since even an empty workgroup costs its dispatch (a 4096-block grid ~2 us more per step)
  if (blocks > 1024) blocks = 1024;
  if (dtype == SBOD_DT_F32)
    hipLaunchKernelGGL(sbod::k_scale<float>, dim3(blocks), dim3(256), 0, sbod::as_stream(stream),
                       static_cast<float *>(grad), n, scale);
  else
    hipLaunchKernelGGL(sbod::k_scale<uint16_t>, dim3(blocks), dim3(256), 0,
                       sbod::as_stream(stream), static_cast<uint16_t *>(grad), n, scale);
  SBOD_LAUNCHED("sbod_scale_inplace");
  return SBOD_OK;
}

int sbod_scale2_inplace(void *a, int64_t na, void *b, int64_t nb, int dtype, const float *scale,
                        void *stream) {
  SBOD_REQUIRE(na >= 0 && nb >= 0 && scale != nullptr, "sbod_scale2_inplace: bad arguments");
  const int64_t n = na + nb;
  if (n == 0) return SBOD_OK;
  int64_t blocks = (n + 255) / 256;
  // the usual upstream gradient is 1 and every block exits at once: the grid is kept small,
  // since even an empty workgroup costs its dispatch (a 4096-block grid ~2 us more per step)
  if (blocks > 1024) blocks = 1024;
  if (dtype == SBOD_DT_F32)
    hipLaunchKernelGGL(sbod::k_scale2<float>, dim3(blocks), dim3(256), 0, sbod::as_stream(stream),
                       static_cast<float *>(a), na, static_cast<float *>(b), nb, scale);
  else
    hipLaunchKernelGGL(sbod::k_scale2<uint16_t>, dim3(blocks), dim3(256), 0, sbod::as_stream(stream),
                       static_cast<uint16_t *>(a), na, static_cast<uint16_t *>(b), nb, scale);
  SBOD_LAUNCHED("sbod_scale2_inplace");
  return SBOD_OK;
}

}  // extern "C"

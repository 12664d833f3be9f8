// _sbodhost: the per-step host work of the ground-truth packing in C++ (a CPython extension over
// ATen's tensor handles), so staging a batch costs one launch and a loop over pointers:
//
//   pack_device_lists(boxes, labels, capacity, per_image_cap, device, out_boxes, out_labels,
//                     out_offsets, stream, allow_empty) -> list | None | int
//       The collate_fn batch (dataset/Datasets.py:58-86: LISTS of per-image [G_i,4] f32 boxes and
//       [G_i] int64 labels, already on the device, train_anchor.py:266-268) checked and packed
//       by ONE sbod_gt_pack launch.  Returns the per-image counts on success; None when any item
//       is irregular (not a device tensor, another device, dtype/shape/contiguity needing a
//       conversion, an empty image when not allowed, more objects than the capacity) — the
//       caller (core._pack_lists) then takes the Python path, which converts or raises the
//       reference's errors, so error behaviour lives in one place; an int = sbod_gt_pack's
//       failing status (the caller raises SbodError with sbod_last_error()).
//       capacity = rows of the output buffers; per_image_cap < 0 = no per-image limit;
//       device < 0 = any (one device for the whole batch either way).
//
//   stage_and_replay(...): the same packing, then captured graphs and an event (below).
//
//   criterion_focal_fast(...): a focal criterion call of the reference-named classes
//       (MultiBoxLoss512 / 300 / RetinaFocalLoss, models/SSD512.py:525-623) in one call: the GT
//       list checks + packing, sbod_criterion_focal, and the loss tensor's autograd node — a C++
//       node (FusedLossFn), so loss.backward() runs no Python on autograd's device thread.
#include <Python.h>

#include <ATen/ATen.h>
#include <torch/csrc/autograd/custom_function.h>
#include <torch/csrc/autograd/python_variable.h>

#include <chrono>
#include <cstdint>
#include <vector>

#include "sbod.h"

namespace {

// Row pointers of one checked batch (check_lists' output).
struct ListRows {
  std::vector<const void *> bp, lp;
  std::vector<int32_t> cnt;
};

// Checks the lists and, with `launch`, launches sbod_gt_pack.  Returns 1 on success (rows
// filled), 0 when the batch needs the Python path (nothing launched), or a negative sbod status.
int pack_lists(PyObject *boxes, PyObject *labels, long long capacity, long long per_image,
               int want_dev, void *ob, void *ol, void *oo, void *stream, int allow_empty,
               ListRows &rows, void *src_stream, bool launch = true) {
  if (!PyList_Check(boxes) || !PyList_Check(labels)) return 0;
  const Py_ssize_t B = PyList_GET_SIZE(boxes);
  if (B != PyList_GET_SIZE(labels) || B == 0) return 0;
  std::vector<const void *> &bp = rows.bp, &lp = rows.lp;
  std::vector<int32_t> &cnt = rows.cnt;
  bp.assign(B, nullptr);
  lp.assign(B, nullptr);
  cnt.assign(B, 0);
  long long total = 0;
  int dev = want_dev;
  for (Py_ssize_t i = 0; i < B; ++i) {
    PyObject *ob_i = PyList_GET_ITEM(boxes, i), *ol_i = PyList_GET_ITEM(labels, i);
    if (!THPVariable_Check(ob_i) || !THPVariable_Check(ol_i)) return 0;
    const at::Tensor &tb = THPVariable_Unpack(ob_i);
    const at::Tensor &tl = THPVariable_Unpack(ol_i);
    if (!tb.is_cuda() || !tl.is_cuda()) return 0;
    const int d = tb.get_device();
    if ((dev >= 0 && d != dev) || tl.get_device() != d) return 0;
    dev = d;
    if (tb.scalar_type() != at::kFloat || tl.scalar_type() != at::kLong || tb.dim() != 2 ||
        tb.size(1) != 4 || tl.dim() != 1 || tl.size(0) != tb.size(0) || !tb.is_contiguous() ||
        !tl.is_contiguous())
      return 0;
    const int64_t g = tb.size(0);
    if ((g == 0 && !allow_empty) || (per_image >= 0 && g > per_image)) return 0;
    bp[i] = tb.data_ptr();
    lp[i] = tl.data_ptr();
    cnt[i] = static_cast<int32_t>(g);
    total += g;
  }
  if (total > capacity) return 0;
  if (!launch) return 1;
  if (src_stream != stream) {   // fork: the pack waits for the stream that produced the GT
    const int sw = sbod_stream_wait(stream, src_stream);
    if (sw != SBOD_OK) return sw;
  }
  const int st = sbod_gt_pack(bp.data(), lp.data(), cnt.data(), static_cast<int>(B), capacity,
                              static_cast<float *>(ob), static_cast<int64_t *>(ol),
                              static_cast<int32_t *>(oo), stream);
  return st == SBOD_OK ? 1 : st;
}

PyObject *counts_list(const std::vector<int32_t> &cnt) {
  PyObject *counts = PyList_New(static_cast<Py_ssize_t>(cnt.size()));
  if (!counts) return nullptr;
  for (size_t i = 0; i < cnt.size(); ++i) PyList_SET_ITEM(counts, i, PyLong_FromLong(cnt[i]));
  return counts;
}

void *opt_ptr(PyObject *o) { return o == Py_None ? nullptr : PyLong_AsVoidPtr(o); }

PyObject *pack_device_lists(PyObject *, PyObject *const *a, Py_ssize_t n) {
  if (n != 10) {
    PyErr_SetString(PyExc_TypeError, "pack_device_lists: expected 10 arguments");
    return nullptr;
  }
  const long long capacity = PyLong_AsLongLong(a[2]);
  const long long per_image = PyLong_AsLongLong(a[3]);
  const int want_dev = static_cast<int>(PyLong_AsLong(a[4]));
  void *ob = PyLong_AsVoidPtr(a[5]), *ol = PyLong_AsVoidPtr(a[6]), *oo = PyLong_AsVoidPtr(a[7]);
  void *stream = opt_ptr(a[8]);
  const int allow_empty = PyObject_IsTrue(a[9]);
  if (PyErr_Occurred()) return nullptr;
  ListRows rows;
  const int r = pack_lists(a[0], a[1], capacity, per_image, want_dev, ob, ol, oo, stream, allow_empty, rows,
                           stream);
  if (r == 0) Py_RETURN_NONE;
  if (r < 0) return PyLong_FromLong(r);
  return counts_list(rows.cnt);
}

// stage_and_replay(boxes, labels, capacity, per_image_cap, device, out_boxes, out_labels,
//                  out_offsets, stream, allow_empty, launches, event, event_stream, src_stream)
//   pack_device_lists' packing on `stream`, then every (graph_exec, stream) pair of `launches`
//   (a tuple) launched in order (sbod_graph_launch), then `event` (hipEvent_t or None) recorded
//   on `event_stream`: one call submits a captured step.  Returns as pack_device_lists; None
//   means nothing was launched.
//   Ordering contract: the GT tensors were produced on `src_stream` (the caller's current
//   stream, e.g. by a non_blocking .to(device)).  When the packing stream differs, it first
//   waits for `src_stream`, and `src_stream` then waits for the packing launch (not for the
//   graphs): the pack never reads a copy that has not landed, and the caching allocator —
//   which hands a freed block out again only to work on its allocation stream — cannot give
//   the source memory to later work on `src_stream` before the pack has read it.
PyObject *stage_and_replay(PyObject *, PyObject *const *a, Py_ssize_t n) {
  if (n != 14) {
    PyErr_SetString(PyExc_TypeError, "stage_and_replay: expected 14 arguments");
    return nullptr;
  }
  const long long capacity = PyLong_AsLongLong(a[2]);
  const long long per_image = PyLong_AsLongLong(a[3]);
  const int want_dev = static_cast<int>(PyLong_AsLong(a[4]));
  void *ob = PyLong_AsVoidPtr(a[5]), *ol = PyLong_AsVoidPtr(a[6]), *oo = PyLong_AsVoidPtr(a[7]);
  void *stream = opt_ptr(a[8]);
  const int allow_empty = PyObject_IsTrue(a[9]);
  PyObject *launches = a[10];
  void *event = opt_ptr(a[11]);
  void *ev_stream = opt_ptr(a[12]);
  void *src_stream = opt_ptr(a[13]);
  if (PyErr_Occurred()) return nullptr;
  if (!PyTuple_Check(launches)) {
    PyErr_SetString(PyExc_TypeError, "stage_and_replay: launches must be a tuple of (exec, stream)");
    return nullptr;
  }
  const Py_ssize_t nl = PyTuple_GET_SIZE(launches);
  std::vector<void *> ex(nl), st(nl);
  for (Py_ssize_t i = 0; i < nl; ++i) {
    PyObject *pr = PyTuple_GET_ITEM(launches, i);
    if (!PyTuple_Check(pr) || PyTuple_GET_SIZE(pr) != 2) {
      PyErr_SetString(PyExc_TypeError, "stage_and_replay: launches must be a tuple of (exec, stream)");
      return nullptr;
    }
    ex[i] = PyLong_AsVoidPtr(PyTuple_GET_ITEM(pr, 0));
    st[i] = opt_ptr(PyTuple_GET_ITEM(pr, 1));
  }
  if (PyErr_Occurred()) return nullptr;
  ListRows rows;
  const int r = pack_lists(a[0], a[1], capacity, per_image, want_dev, ob, ol, oo, stream, allow_empty, rows,
                           src_stream);
  if (r == 0) Py_RETURN_NONE;
  if (r < 0) return PyLong_FromLong(r);
  if (src_stream != stream) {
    const int sj = sbod_stream_wait(src_stream, stream);   // join: after the pack only
    if (sj != SBOD_OK) return PyLong_FromLong(sj);
  }
  for (Py_ssize_t i = 0; i < nl; ++i) {
    const int s2 = sbod_graph_launch(ex[i], st[i]);
    if (s2 != SBOD_OK) return PyLong_FromLong(s2);
  }
  if (event) {
    const int s3 = sbod_event_record(event, ev_stream);
    if (s3 != SBOD_OK) return PyLong_FromLong(s3);
  }
  return counts_list(rows.cnt);
}

// ---------------------------------------------------------------------------- step programs
// A recorded step, submitted natively: the GT packing's fixed destination, the criterion's and
// detect's entry-point calls with the arguments recorded from one eager call
// (_lib.record_calls: their outputs, the streams' warm workspaces, the zero-on-entry flags), and
// detect's event.  One C++ call per step then does the list checks + sbod_gt_pack,
// sbod_criterion_focal, sbod_detect_f32 and sbod_event_record — what a hipGraph replay does,
// without two hipGraphLaunch calls and without Python between the launches.
//   make_step_program(pack, crit_args, det_args, event, event_stream[, lists]) -> capsule
//     pack = (capacity, per_image_cap, device, out_boxes, out_labels, out_offsets, stream);
//     crit_args / det_args = the recorded argument tuples of sbod_criterion_focal /
//     sbod_detect_f32 (include/sbod.h order; pointers as int or None).
//   submit_step_program(capsule, boxes, labels[, parts]) -> True | None | int
//     None: the lists need the Python path (nothing launched); int: a failing sbod status.
//     parts (default 3): bit 0 the GT packing + criterion, bit 1 the detect + event — one chain
//     alone is a diagnostic (scripts/gpu_interval.py), the step submits both.
//   The lists are taken as ready on the packing stream (resident device tensors), which is the
//   criterion's stream.  With `lists` true the packing is folded into the matcher's first launch
//   (sbod_criterion_focal_lists) whenever the batch allows it (<= 64 images, each 1..Gmax
//   objects, aligned rows); other batches take sbod_gt_pack + sbod_criterion_focal.
struct StepProgram {
  long long capacity, per_image;
  int dev;
  void *ob, *ol, *oo, *pack_stream;
  // sbod_criterion_focal
  const void *c_locs, *c_scores;
  int c_dtype, c_B, c_P, c_C;
  const float *c_pcxcy, *c_pxy, *c_gtb;
  const int64_t *c_gtl;
  const int32_t *c_gto;
  int c_Gmax;
  float c_thr, c_nthr;
  int c_reg, c_flags;
  float c_rw, c_fa, c_fg;
  int32_t *c_obj;
  float *c_ovl;
  int32_t *c_npos;
  void *c_gl, *c_gs;
  float *c_out;
  void *c_ws;
  size_t c_wsb;
  void *c_stream;
  // sbod_detect_f32
  void *d_locs;
  const void *d_scores;
  int d_B, d_P, d_C;
  const float *d_pri;
  const uint8_t *d_pm;
  int d_box, d_act;
  float d_min, d_ovl;
  int d_topk;
  float d_fnms;
  int d_window, d_flags;
  float *d_boxes;
  int64_t *d_labels;
  float *d_scores_out;
  int32_t *d_count, *d_count_host;
  float *d_dbg_p, *d_dbg_b;
  void *d_ws;
  size_t d_wsb;
  void *d_stream;
  void *event, *ev_stream;
  bool lists;
};

struct ArgReader {   // the recorded tuple, item by item, in signature order
  PyObject *t;
  Py_ssize_t i = 0;
  PyObject *next() { return i < PyTuple_GET_SIZE(t) ? PyTuple_GET_ITEM(t, i++) : nullptr; }
  void *ptr() { PyObject *o = next(); return (o == nullptr || o == Py_None) ? nullptr : PyLong_AsVoidPtr(o); }
  int i32() { PyObject *o = next(); return o ? static_cast<int>(PyLong_AsLong(o)) : 0; }
  float f32() { PyObject *o = next(); return o ? static_cast<float>(PyFloat_AsDouble(o)) : 0.f; }
  size_t sz() { PyObject *o = next(); return o ? PyLong_AsSize_t(o) : 0; }
};

void free_program(PyObject *cap) { delete static_cast<StepProgram *>(PyCapsule_GetPointer(cap, "sbod.StepProgram")); }

PyObject *make_step_program(PyObject *, PyObject *const *a, Py_ssize_t n) {
  if ((n != 5 && n != 6) || !PyTuple_Check(a[0]) || PyTuple_GET_SIZE(a[0]) != 7 || !PyTuple_Check(a[1]) ||
      PyTuple_GET_SIZE(a[1]) != 28 || !PyTuple_Check(a[2]) || PyTuple_GET_SIZE(a[2]) != 25) {
    PyErr_SetString(PyExc_TypeError,
                    "make_step_program(pack[7], criterion_focal args[28], detect_f32 args[25], event, event_stream)");
    return nullptr;
  }
  auto *p = new StepProgram();
  ArgReader k{a[0]};
  p->capacity = PyLong_AsLongLong(k.next());
  p->per_image = PyLong_AsLongLong(k.next());
  p->dev = k.i32();
  p->ob = k.ptr(); p->ol = k.ptr(); p->oo = k.ptr(); p->pack_stream = k.ptr();
  ArgReader c{a[1]};
  p->c_locs = c.ptr(); p->c_scores = c.ptr();
  p->c_dtype = c.i32(); p->c_B = c.i32(); p->c_P = c.i32(); p->c_C = c.i32();
  p->c_pcxcy = static_cast<const float *>(c.ptr()); p->c_pxy = static_cast<const float *>(c.ptr());
  p->c_gtb = static_cast<const float *>(c.ptr()); p->c_gtl = static_cast<const int64_t *>(c.ptr());
  p->c_gto = static_cast<const int32_t *>(c.ptr());
  p->c_Gmax = c.i32(); p->c_thr = c.f32(); p->c_nthr = c.f32(); p->c_reg = c.i32(); p->c_flags = c.i32();
  p->c_rw = c.f32(); p->c_fa = c.f32(); p->c_fg = c.f32();
  p->c_obj = static_cast<int32_t *>(c.ptr()); p->c_ovl = static_cast<float *>(c.ptr());
  p->c_npos = static_cast<int32_t *>(c.ptr()); p->c_gl = c.ptr(); p->c_gs = c.ptr();
  p->c_out = static_cast<float *>(c.ptr()); p->c_ws = c.ptr(); p->c_wsb = c.sz(); p->c_stream = c.ptr();
  ArgReader d{a[2]};
  p->d_locs = d.ptr(); p->d_scores = d.ptr();
  p->d_B = d.i32(); p->d_P = d.i32(); p->d_C = d.i32();
  p->d_pri = static_cast<const float *>(d.ptr()); p->d_pm = static_cast<const uint8_t *>(d.ptr());
  p->d_box = d.i32(); p->d_act = d.i32(); p->d_min = d.f32(); p->d_ovl = d.f32(); p->d_topk = d.i32();
  p->d_fnms = d.f32(); p->d_window = d.i32(); p->d_flags = d.i32();
  p->d_boxes = static_cast<float *>(d.ptr()); p->d_labels = static_cast<int64_t *>(d.ptr());
  p->d_scores_out = static_cast<float *>(d.ptr()); p->d_count = static_cast<int32_t *>(d.ptr());
  p->d_count_host = static_cast<int32_t *>(d.ptr()); p->d_dbg_p = static_cast<float *>(d.ptr());
  p->d_dbg_b = static_cast<float *>(d.ptr()); p->d_ws = d.ptr(); p->d_wsb = d.sz(); p->d_stream = d.ptr();
  p->event = opt_ptr(a[3]);
  p->ev_stream = opt_ptr(a[4]);
  p->lists = n == 6 && PyObject_IsTrue(a[5]) == 1;
  if (PyErr_Occurred()) {
    delete p;
    return nullptr;
  }
  PyObject *cap = PyCapsule_New(p, "sbod.StepProgram", free_program);
  if (!cap) delete p;
  return cap;
}

// Host time of submit_step_program by phase (steady clock, summed over calls; read and reset by
// submit_profile()): list checks + packing launch, criterion launches, detect launches, event.
double g_sub_ns[5];
long long g_sub_calls;
constexpr int kSubFirst = 8;   // the first calls after a reset, phase by phase (the pipeline's fill)
double g_sub_first[kSubFirst][4];
using SteadyClock = std::chrono::steady_clock;
inline double ns_since(SteadyClock::time_point &t) {
  const auto n = SteadyClock::now();
  const double d = std::chrono::duration<double, std::nano>(n - t).count();
  t = n;
  return d;
}

PyObject *submit_profile(PyObject *, PyObject *const *a, Py_ssize_t n) {
  const bool reset = n > 0 && PyObject_IsTrue(a[0]) == 1;
  PyObject *first = PyList_New(0);
  for (long long i = 0; first && i < g_sub_calls && i < kSubFirst; ++i) {
    PyObject *e = Py_BuildValue("[d,d,d,d]", g_sub_first[i][0] / 1e3, g_sub_first[i][1] / 1e3,
                                g_sub_first[i][2] / 1e3, g_sub_first[i][3] / 1e3);
    if (!e || PyList_Append(first, e) != 0) Py_CLEAR(first);
    Py_XDECREF(e);
  }
  if (!first) return nullptr;
  PyObject *r = Py_BuildValue("{s:L,s:d,s:d,s:d,s:d,s:d,s:N}", "calls", g_sub_calls, "pack_us", g_sub_ns[0] / 1e3,
                              "criterion_us", g_sub_ns[1] / 1e3, "detect_us", g_sub_ns[2] / 1e3, "event_us",
                              g_sub_ns[3] / 1e3, "total_us", g_sub_ns[4] / 1e3, "first_calls_us", first);
  if (reset) {
    for (double &v : g_sub_ns) v = 0.0;
    g_sub_calls = 0;
  }
  return r;
}

PyObject *submit_step_program(PyObject *, PyObject *const *a, Py_ssize_t n) {
  if (n != 3 && n != 4) {
    PyErr_SetString(PyExc_TypeError, "submit_step_program(program, boxes, labels[, parts])");
    return nullptr;
  }
  auto *p = static_cast<StepProgram *>(PyCapsule_GetPointer(a[0], "sbod.StepProgram"));
  if (!p) return nullptr;
  const long parts = n == 4 ? PyLong_AsLong(a[3]) : 3;
  if (parts < 1 || parts > 3) {
    if (!PyErr_Occurred()) PyErr_SetString(PyExc_ValueError, "submit_step_program: parts must be 1, 2 or 3");
    return nullptr;
  }
  if (!(parts & 1)) {   // detect (+ event) alone: no lists, no packing
    auto t = SteadyClock::now();
    const int sd = sbod_detect_f32(p->d_locs, p->d_scores, p->d_B, p->d_P, p->d_C, p->d_pri, p->d_pm, p->d_box,
                                   p->d_act, p->d_min, p->d_ovl, p->d_topk, p->d_fnms, p->d_window, p->d_flags,
                                   p->d_boxes, p->d_labels, p->d_scores_out, p->d_count, p->d_count_host,
                                   p->d_dbg_p, p->d_dbg_b, p->d_ws, p->d_wsb, p->d_stream);
    if (sd != SBOD_OK) return PyLong_FromLong(sd);
    if (p->event) {
      const int se = sbod_event_record(p->event, p->ev_stream);
      if (se != SBOD_OK) return PyLong_FromLong(se);
    }
    g_sub_ns[2] += ns_since(t);
    Py_RETURN_TRUE;
  }
  auto t_start = SteadyClock::now(), t = t_start;
  double ph[4] = {0.0, 0.0, 0.0, 0.0};
  ListRows rows;
  const int r = pack_lists(a[1], a[2], p->capacity, p->per_image, p->dev, p->ob, p->ol, p->oo, p->pack_stream, 0,
                           rows, p->pack_stream, !p->lists);
  if (r == 0) Py_RETURN_NONE;
  if (r < 0) return PyLong_FromLong(r);
  bool folded = false;
  if (p->lists) {
    const size_t B = rows.cnt.size();
    folded = B <= 64 && static_cast<int>(B) == p->c_B && p->ob == p->c_gtb && p->pack_stream == p->c_stream;
    for (size_t i = 0; folded && i < B; ++i)
      folded = rows.cnt[i] >= 1 && rows.cnt[i] <= p->c_Gmax &&
               (reinterpret_cast<uintptr_t>(rows.bp[i]) & 15) == 0 && (reinterpret_cast<uintptr_t>(rows.lp[i]) & 7) == 0;
    if (!folded) {   // this batch takes the packing launch
      const int sp = sbod_gt_pack(rows.bp.data(), rows.lp.data(), rows.cnt.data(), static_cast<int>(B), p->capacity,
                                  static_cast<float *>(p->ob), static_cast<int64_t *>(p->ol),
                                  static_cast<int32_t *>(p->oo), p->pack_stream);
      if (sp != SBOD_OK) return PyLong_FromLong(sp);
    }
  }
  g_sub_ns[0] += ph[0] = ns_since(t);
  int st;
  if (folded)
    st = sbod_criterion_focal_lists(rows.bp.data(), rows.lp.data(), rows.cnt.data(), p->capacity, p->c_locs,
                                    p->c_scores, p->c_dtype, p->c_B, p->c_P, p->c_C, p->c_pcxcy, p->c_pxy,
                                    static_cast<float *>(p->ob), static_cast<int64_t *>(p->ol),
                                    static_cast<int32_t *>(p->oo), p->c_Gmax, p->c_thr, p->c_nthr, p->c_reg,
                                    p->c_flags, p->c_rw, p->c_fa, p->c_fg, p->c_obj, p->c_ovl, p->c_npos, p->c_gl,
                                    p->c_gs, p->c_out, p->c_ws, p->c_wsb, p->c_stream);
  else
    st = sbod_criterion_focal(p->c_locs, p->c_scores, p->c_dtype, p->c_B, p->c_P, p->c_C, p->c_pcxcy, p->c_pxy,
                              p->c_gtb, p->c_gtl, p->c_gto, p->c_Gmax, p->c_thr, p->c_nthr, p->c_reg, p->c_flags,
                              p->c_rw, p->c_fa, p->c_fg, p->c_obj, p->c_ovl, p->c_npos, p->c_gl, p->c_gs, p->c_out,
                              p->c_ws, p->c_wsb, p->c_stream);
  if (st != SBOD_OK) return PyLong_FromLong(st);
  g_sub_ns[1] += ph[1] = ns_since(t);
  if (!(parts & 2)) Py_RETURN_TRUE;   // the criterion alone
  st = sbod_detect_f32(p->d_locs, p->d_scores, p->d_B, p->d_P, p->d_C, p->d_pri, p->d_pm, p->d_box, p->d_act,
                       p->d_min, p->d_ovl, p->d_topk, p->d_fnms, p->d_window, p->d_flags, p->d_boxes, p->d_labels,
                       p->d_scores_out, p->d_count, p->d_count_host, p->d_dbg_p, p->d_dbg_b, p->d_ws, p->d_wsb,
                       p->d_stream);
  if (st != SBOD_OK) return PyLong_FromLong(st);
  g_sub_ns[2] += ph[2] = ns_since(t);
  if (p->event) {
    st = sbod_event_record(p->event, p->ev_stream);
    if (st != SBOD_OK) return PyLong_FromLong(st);
  }
  g_sub_ns[3] += ph[3] = ns_since(t);
  g_sub_ns[4] += std::chrono::duration<double, std::nano>(t - t_start).count();
  if (g_sub_calls < kSubFirst)
    for (int k = 0; k < 4; ++k) g_sub_first[g_sub_calls][k] = ph[k];
  ++g_sub_calls;
  Py_RETURN_TRUE;
}

// ---------------------------------------------------------------------------- criterion_focal_fast
// The criterion launch inside the autograd node's forward, so the node owns the gradients the
// fused pass writes (core._FusedLoss's contract): backward hands them over as they are when the
// upstream gradient is core.unit_grad(), else scales them in place on the forward's stream
// (sbod_scale2_inplace: no host sync), and drops its own references first so AccumulateGrad
// adopts them as .grad instead of cloning them.
struct CritCall {
  int dtype, B, P, C, gmax, reg, flags;
  const void *pcxcy, *pxy, *gtb, *gtl, *gto;
  float thr, nthr, reg_weight, alpha, gamma;
  void *obj, *ovl, *npos, *ws, *stream;
  size_t ws_bytes;
  bool want;
  int64_t unit;      // data pointer of core.unit_grad(device), 0 if none yet
  at::Tensor out;    // {total, conf, loc, n_pos_total}
  int status = 0;
};

struct FusedLossFn : public torch::autograd::Function<FusedLossFn> {
  static at::Tensor forward(torch::autograd::AutogradContext *ctx, const at::Tensor &locs, const at::Tensor &scores,
                            CritCall *c) {
    at::Tensor out = at::empty({4}, locs.options().dtype(at::kFloat));
    at::Tensor gl, gs;
    if (c->want) {
      gl = at::empty_like(locs);
      gs = at::empty_like(scores);
    }
    c->status = sbod_criterion_focal(locs.data_ptr(), scores.data_ptr(), c->dtype, c->B, c->P, c->C,
                                     static_cast<const float *>(c->pcxcy), static_cast<const float *>(c->pxy),
                                     static_cast<const float *>(c->gtb), static_cast<const int64_t *>(c->gtl),
                                     static_cast<const int32_t *>(c->gto), c->gmax, c->thr, c->nthr, c->reg, c->flags,
                                     c->reg_weight, c->alpha, c->gamma, static_cast<int32_t *>(c->obj),
                                     static_cast<float *>(c->ovl), static_cast<int32_t *>(c->npos),
                                     gl.defined() ? gl.data_ptr() : nullptr, gs.defined() ? gs.data_ptr() : nullptr,
                                     out.data_ptr<float>(), c->ws, c->ws_bytes, c->stream);
    c->out = out;
    ctx->saved_data["gl"] = gl;
    ctx->saved_data["gs"] = gs;
    ctx->saved_data["stream"] = reinterpret_cast<int64_t>(c->stream);
    ctx->saved_data["unit"] = c->unit;
    ctx->saved_data["dt"] = static_cast<int64_t>(c->dtype);
    ctx->set_materialize_grads(false);
    return out.select(0, 0);
  }
  static torch::autograd::variable_list backward(torch::autograd::AutogradContext *ctx,
                                                 torch::autograd::variable_list go) {
    auto &sd = ctx->saved_data;
    if (sd.find("gl") == sd.end())
      throw std::runtime_error("sbod fused criterion: backward through the same graph twice is not supported "
                               "(its gradients are produced in forward)");
    at::Tensor gl = sd["gl"].toTensor(), gs = sd["gs"].toTensor();
    void *stream = reinterpret_cast<void *>(sd["stream"].toInt());
    const int64_t unit = sd["unit"].toInt();
    const int dt = static_cast<int>(sd["dt"].toInt());
    sd.erase("gl");
    sd.erase("gs");
    if (go.empty() || !go[0].defined() || !gl.defined()) return {at::Tensor(), at::Tensor(), at::Tensor()};
    at::Tensor g = go[0];
    if (unit == 0 || reinterpret_cast<int64_t>(g.data_ptr()) != unit) {
      if (g.scalar_type() != at::kFloat || !g.is_contiguous()) g = g.detach().to(at::kFloat).contiguous();
      const int st = sbod_scale2_inplace(gl.data_ptr(), gl.numel(), gs.data_ptr(), gs.numel(), dt,
                                         g.data_ptr<float>(), stream);
      if (st != SBOD_OK) throw std::runtime_error(std::string("sbod_scale2_inplace: ") + sbod_last_error());
    }
    return {std::move(gl), std::move(gs), at::Tensor()};
  }
};

// criterion_focal_fast(locs, scores, boxes, labels, priors_cxcy_ptr, priors_xy_ptr, gt_boxes_ptr,
//                      gt_labels_ptr, gt_offsets_ptr, gt_capacity, reg, flags, threshold,
//                      neg_threshold, reg_weight, alpha, gamma, obj_ptr, ovl_ptr, npos_ptr, ws_ptr,
//                      ws_bytes, clean_bytes, stream, unit_ptr)
//   -> (loss, components, zero_bytes) | None (the batch or the cached buffers need the Python
//      path: it re-packs) | int (a failing sbod status; the caller raises)
//   locs / scores: [B,P,4] / [B,P,C] contiguous, both float32 or both bfloat16, on the device of
//   the GT lists.  flags: SBOD_LOSS_FOCAL_NORM / SBOD_LOSS_UNFUSED_FINISH / SBOD_CRIT_TWO_LAUNCH;
//   SBOD_CRIT_WS_ZEROED is added here when the workspace's first clean_bytes cover the call's
//   zero-on-entry prefix (returned, for the caller's bookkeeping).
PyObject *criterion_focal_fast(PyObject *, PyObject *const *a, Py_ssize_t n) {
  if (n != 25) {
    PyErr_SetString(PyExc_TypeError, "criterion_focal_fast: expected 25 arguments");
    return nullptr;
  }
  if (!THPVariable_Check(a[0]) || !THPVariable_Check(a[1])) Py_RETURN_NONE;
  const at::Tensor &locs = THPVariable_Unpack(a[0]);
  const at::Tensor &scores = THPVariable_Unpack(a[1]);
  const auto dt = locs.scalar_type();
  if (!locs.is_cuda() || !scores.is_cuda() || (dt != at::kFloat && dt != at::kBFloat16) || scores.scalar_type() != dt ||
      locs.dim() != 3 || scores.dim() != 3 || locs.size(2) != 4 || locs.size(0) != scores.size(0) ||
      locs.size(1) != scores.size(1) || !locs.is_contiguous() || !scores.is_contiguous() ||
      locs.get_device() != scores.get_device())
    Py_RETURN_NONE;
  CritCall c;
  c.dtype = dt == at::kFloat ? SBOD_DT_F32 : SBOD_DT_BF16;
  c.B = static_cast<int>(locs.size(0));
  c.P = static_cast<int>(locs.size(1));
  c.C = static_cast<int>(scores.size(2));
  c.pcxcy = PyLong_AsVoidPtr(a[4]);
  c.pxy = PyLong_AsVoidPtr(a[5]);
  void *gb = PyLong_AsVoidPtr(a[6]), *gl = PyLong_AsVoidPtr(a[7]), *go = PyLong_AsVoidPtr(a[8]);
  const long long cap = PyLong_AsLongLong(a[9]);
  c.reg = static_cast<int>(PyLong_AsLong(a[10]));
  c.flags = static_cast<int>(PyLong_AsLong(a[11]));
  c.thr = static_cast<float>(PyFloat_AsDouble(a[12]));
  c.nthr = static_cast<float>(PyFloat_AsDouble(a[13]));
  c.reg_weight = static_cast<float>(PyFloat_AsDouble(a[14]));
  c.alpha = static_cast<float>(PyFloat_AsDouble(a[15]));
  c.gamma = static_cast<float>(PyFloat_AsDouble(a[16]));
  c.obj = PyLong_AsVoidPtr(a[17]);
  c.ovl = PyLong_AsVoidPtr(a[18]);
  c.npos = PyLong_AsVoidPtr(a[19]);
  c.ws = PyLong_AsVoidPtr(a[20]);
  c.ws_bytes = static_cast<size_t>(PyLong_AsUnsignedLongLong(a[21]));
  const unsigned long long clean = PyLong_AsUnsignedLongLong(a[22]);
  c.stream = opt_ptr(a[23]);
  c.unit = static_cast<int64_t>(reinterpret_cast<intptr_t>(opt_ptr(a[24])));
  if (PyErr_Occurred()) return nullptr;
  ListRows rows;
  const int r = pack_lists(a[2], a[3], cap, -1, locs.get_device(), gb, gl, go, c.stream, 0, rows, c.stream);
  if (r == 0) Py_RETURN_NONE;
  if (r < 0) return PyLong_FromLong(r);
  if (static_cast<int>(rows.cnt.size()) != c.B) Py_RETURN_NONE;   // (the caller's error path names it)
  int gmax = 1;
  for (int32_t g : rows.cnt) gmax = g > gmax ? g : gmax;
  c.gmax = gmax;
  if (sbod_criterion_workspace_bytes(c.B, gmax, c.P) > c.ws_bytes) Py_RETURN_NONE;   // the Python path grows it
  const size_t zb = sbod_criterion_zero_bytes(c.B, gmax, c.P);
  if (zb <= clean) c.flags |= SBOD_CRIT_WS_ZEROED;
  c.gtb = gb;
  c.gtl = gl;
  c.gto = go;
  c.want = at::GradMode::is_enabled() && (locs.requires_grad() || scores.requires_grad());
  at::Tensor loss;
  try {
    loss = FusedLossFn::apply(locs, scores, &c);
  } catch (const std::exception &e) {
    PyErr_SetString(PyExc_RuntimeError, e.what());
    return nullptr;
  }
  if (c.status != SBOD_OK) return PyLong_FromLong(c.status);
  PyObject *res = PyTuple_New(4);
  if (!res) return nullptr;
  PyTuple_SET_ITEM(res, 0, THPVariable_Wrap(std::move(loss)));
  PyTuple_SET_ITEM(res, 1, THPVariable_Wrap(std::move(c.out)));
  PyTuple_SET_ITEM(res, 2, PyLong_FromSize_t(zb));
  PyTuple_SET_ITEM(res, 3, PyLong_FromLong(gmax));   // the workspace's layout (sbod_loss_finish_status)
  return res;
}

PyMethodDef methods[] = {
    {"criterion_focal_fast",
     reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(criterion_focal_fast)),
     METH_FASTCALL, "GT packing + sbod_criterion_focal + a C++ autograd node for the loss."},
    {"make_step_program",
     reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(make_step_program)),
     METH_FASTCALL, "Parse a recorded step (GT packing target, criterion and detect calls, event) once."},
    {"submit_profile", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(submit_profile)), METH_FASTCALL,
     "submit_profile([reset]) -> host time of submit_step_program by phase (us, summed over calls)."},
    {"submit_step_program",
     reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(submit_step_program)),
     METH_FASTCALL, "GT packing + the recorded criterion and detect calls + the event, natively (parts: 1 criterion, 2 detect, 3 both)."},
    {"pack_device_lists",
     reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(pack_device_lists)),
     METH_FASTCALL, "Check and pack per-image device GT lists with one sbod_gt_pack launch."},
    {"stage_and_replay",
     reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(stage_and_replay)),
     METH_FASTCALL, "GT packing, then captured graphs launched on their streams, then an event."},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef mod = {PyModuleDef_HEAD_INIT, "_sbodhost", nullptr, -1, methods};

}  // namespace

PyMODINIT_FUNC PyInit__sbodhost(void) { return PyModule_Create(&mod); }

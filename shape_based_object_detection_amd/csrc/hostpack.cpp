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
#include <Python.h>

#include <torch/csrc/autograd/python_variable.h>

#include <cstdint>
#include <vector>

#include "sbod.h"

namespace {

// Checks the lists and launches sbod_gt_pack.  Returns 1 on success (cnt filled), 0 when the
// batch needs the Python path (nothing launched), or a negative sbod status.
int pack_lists(PyObject *boxes, PyObject *labels, long long capacity, long long per_image,
               int want_dev, void *ob, void *ol, void *oo, void *stream, int allow_empty,
               std::vector<int32_t> &cnt, void *src_stream) {
  if (!PyList_Check(boxes) || !PyList_Check(labels)) return 0;
  const Py_ssize_t B = PyList_GET_SIZE(boxes);
  if (B != PyList_GET_SIZE(labels) || B == 0) return 0;
  std::vector<const void *> bp(B), lp(B);
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
  std::vector<int32_t> cnt;
  const int r = pack_lists(a[0], a[1], capacity, per_image, want_dev, ob, ol, oo, stream, allow_empty, cnt,
                           stream);
  if (r == 0) Py_RETURN_NONE;
  if (r < 0) return PyLong_FromLong(r);
  return counts_list(cnt);
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
  std::vector<int32_t> cnt;
  const int r = pack_lists(a[0], a[1], capacity, per_image, want_dev, ob, ol, oo, stream, allow_empty, cnt,
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
  return counts_list(cnt);
}

PyMethodDef methods[] = {
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

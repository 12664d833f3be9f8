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
#include <Python.h>

#include <torch/csrc/autograd/python_variable.h>

#include <cstdint>
#include <vector>

#include "sbod.h"

namespace {

PyObject *pack_device_lists(PyObject *, PyObject *const *a, Py_ssize_t n) {
  if (n != 10) {
    PyErr_SetString(PyExc_TypeError, "pack_device_lists: expected 10 arguments");
    return nullptr;
  }
  PyObject *boxes = a[0], *labels = a[1];
  if (!PyList_Check(boxes) || !PyList_Check(labels)) Py_RETURN_NONE;
  const Py_ssize_t B = PyList_GET_SIZE(boxes);
  if (B != PyList_GET_SIZE(labels) || B == 0) Py_RETURN_NONE;
  const long long capacity = PyLong_AsLongLong(a[2]);
  const long long per_image = PyLong_AsLongLong(a[3]);
  const int want_dev = static_cast<int>(PyLong_AsLong(a[4]));
  void *ob = PyLong_AsVoidPtr(a[5]), *ol = PyLong_AsVoidPtr(a[6]), *oo = PyLong_AsVoidPtr(a[7]);
  void *stream = a[8] == Py_None ? nullptr : PyLong_AsVoidPtr(a[8]);
  const int allow_empty = PyObject_IsTrue(a[9]);
  if (PyErr_Occurred()) return nullptr;

  std::vector<const void *> bp(B), lp(B);
  std::vector<int32_t> cnt(B);
  long long total = 0;
  int dev = want_dev;
  for (Py_ssize_t i = 0; i < B; ++i) {
    PyObject *ob_i = PyList_GET_ITEM(boxes, i), *ol_i = PyList_GET_ITEM(labels, i);
    if (!THPVariable_Check(ob_i) || !THPVariable_Check(ol_i)) Py_RETURN_NONE;
    const at::Tensor &tb = THPVariable_Unpack(ob_i);
    const at::Tensor &tl = THPVariable_Unpack(ol_i);
    if (!tb.is_cuda() || !tl.is_cuda()) Py_RETURN_NONE;
    const int d = tb.get_device();
    if ((dev >= 0 && d != dev) || tl.get_device() != d) Py_RETURN_NONE;
    dev = d;
    if (tb.scalar_type() != at::kFloat || tl.scalar_type() != at::kLong || tb.dim() != 2 ||
        tb.size(1) != 4 || tl.dim() != 1 || tl.size(0) != tb.size(0) || !tb.is_contiguous() ||
        !tl.is_contiguous())
      Py_RETURN_NONE;
    const int64_t g = tb.size(0);
    if ((g == 0 && !allow_empty) || (per_image >= 0 && g > per_image)) Py_RETURN_NONE;
    bp[i] = tb.data_ptr();
    lp[i] = tl.data_ptr();
    cnt[i] = static_cast<int32_t>(g);
    total += g;
  }
  if (total > capacity) Py_RETURN_NONE;
  const int st = sbod_gt_pack(bp.data(), lp.data(), cnt.data(), static_cast<int>(B), capacity,
                              static_cast<float *>(ob), static_cast<int64_t *>(ol),
                              static_cast<int32_t *>(oo), stream);
  if (st != SBOD_OK) return PyLong_FromLong(st);
  PyObject *counts = PyList_New(B);
  if (!counts) return nullptr;
  for (Py_ssize_t i = 0; i < B; ++i) PyList_SET_ITEM(counts, i, PyLong_FromLong(cnt[i]));
  return counts;
}

PyMethodDef methods[] = {
    {"pack_device_lists",
     reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(pack_device_lists)),
     METH_FASTCALL, "Check and pack per-image device GT lists with one sbod_gt_pack launch."},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef mod = {PyModuleDef_HEAD_INIT, "_sbodhost", nullptr, -1, methods};

}  // namespace

PyMODINIT_FUNC PyInit__sbodhost(void) { return PyModule_Create(&mod); }

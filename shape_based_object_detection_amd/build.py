"""Build libsbod_hip.so in-tree with hipcc for gfx950 (no JIT cache, no setup.py install).

    python -m shape_based_object_detection_amd.build [--force] [-j N]

Compile flags that matter for parity: ``-ffp-contract=off`` (no FMA contraction: every
IoU / threshold expression rounds like the reference's separate torch kernels) and the
default IEEE fp32 division.

Also builds ``lib/_sbodcall*.so``: a CPython extension (gcc, generated from ``_lib.SIGNATURES``)
with one METH_FASTCALL wrapper per int-returning entry point of include/sbod.h.  It calls the
same C ABI as the ctypes binding, minus ctypes' per-argument conversion (~5-15 us per launch
call on the host, which is most of the hot path's step time at SSD512 B=32).
"""
import argparse
import concurrent.futures as cf
import glob
import hashlib
import json
import os
import re
import shutil
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, 'csrc')
INCLUDE = os.path.join(REPO, 'include')
OBJDIR = os.path.join(PKG, 'build')
LIB = os.path.join(PKG, 'lib', 'libsbod_hip.so')
RESOURCES = os.path.join(PKG, 'lib', 'kernel_resources.json')
ARCH = os.environ.get('SBOD_OFFLOAD_ARCH', 'gfx950')

CXXFLAGS = ['-O3', '-std=c++17', '-fPIC', '--offload-arch=' + ARCH, '-ffp-contract=off',
            '-munsafe-fp-atomics', '-Wall', '-Wno-unused-function', '-I', INCLUDE, '-I', CSRC]


def hipcc():
    for c in (os.environ.get('HIPCC'), shutil.which('hipcc'), '/opt/rocm/bin/hipcc'):
        if c and os.path.exists(c):
            return c
    raise RuntimeError('hipcc not found (ROCm toolchain required to build libsbod_hip.so)')


def _deps():
    return glob.glob(os.path.join(CSRC, '*.h')) + glob.glob(os.path.join(INCLUDE, '*.h'))


STAMP = os.path.join(PKG, 'lib', 'build_stamp.json')


def _digest(paths, extra=()):
    """sha256 over the CONTENT of ``paths`` (+ ``extra`` strings): staleness is decided by what the
    sources say, never by file times (a checkout or a copy to the GPU box changes mtimes, not
    content)."""
    h = hashlib.sha256()
    for p in sorted(paths):
        h.update(os.path.relpath(p, REPO).encode() + b'\0')
        with open(p, 'rb') as f:
            h.update(f.read())
        h.update(b'\0')
    for e in extra:
        e = str(e)
        if os.path.isabs(e):   # include paths: the tree moves (the GPU box runs it elsewhere)
            e = os.path.relpath(e, REPO)
        h.update(e.encode() + b'\0')
    return h.hexdigest()


def source_files():
    """Every file the built libraries are made from."""
    return (sorted(glob.glob(os.path.join(CSRC, '*.hip'))) + [HOSTPACK_SRC] + _deps()
            + [os.path.join(PKG, '_lib.py')])


def source_digest():
    """Digest of the sources, the compile flags and the target arch: ``lib/build_stamp.json``
    records it after a successful build, and ``_lib.lib()`` refuses a library whose stamp differs
    (the box must run exactly the committed sources)."""
    return _digest(source_files(), [ARCH] + CXXFLAGS)


def read_stamp():
    try:
        with open(STAMP) as f:
            return json.load(f).get('digest')
    except (OSError, ValueError):
        return None


def _key_path(target):
    return target + '.sha256'


def _stale(target, key):
    """True unless ``target`` exists and was built from inputs whose digest is ``key``."""
    if not os.path.exists(target) or not os.path.exists(_key_path(target)):
        return True
    with open(_key_path(target)) as f:
        return f.read().strip() != key


def _mark(target, key):
    with open(_key_path(target), 'w') as f:
        f.write(key + '\n')


_RES_RE = re.compile(r'remark: +(Function Name|VGPRs|AGPRs|TotalSGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|'
                     r'LDS Size \[bytes/block\]): (\S+)')


def _resource_usage(stderr):
    """Per-kernel register / scratch / LDS / occupancy figures from -Rpass-analysis remarks."""
    out, cur = {}, None
    for m in _RES_RE.finditer(stderr):
        key, val = m.group(1), m.group(2)
        if key == 'Function Name':
            cur = out.setdefault(val, {})
        elif cur is not None:
            cur[key.split(' ')[0]] = int(val)
    return out


def _compile(src, force):
    obj = os.path.join(OBJDIR, os.path.basename(src) + '.o')
    res = obj + '.resources.json'
    key = _digest([src] + _deps(), [ARCH] + CXXFLAGS)
    if force or _stale(obj, key) or not os.path.exists(res):
        cmd = [hipcc()] + CXXFLAGS + ['-Rpass-analysis=kernel-resource-usage', '-c', src, '-o', obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError('hipcc failed for %s:\n%s\n%s' % (src, ' '.join(cmd), r.stderr))
        with open(res, 'w') as f:
            json.dump(_resource_usage(r.stderr), f, indent=1, sort_keys=True)
        _mark(obj, key)
    return obj


def build(force=False, jobs=8, verbose=True):
    """Compile every csrc/*.hip for gfx950 and link lib/libsbod_hip.so.  Returns its path."""
    os.makedirs(OBJDIR, exist_ok=True)
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, '*.hip')))
    with cf.ThreadPoolExecutor(max_workers=max(1, min(jobs, 16))) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), srcs))
    usage = {}
    for o in objs:
        with open(o + '.resources.json') as f:
            usage.update(json.load(f))
    with open(RESOURCES, 'w') as f:     # kernel resource table (tests assert no scratch use)
        json.dump(usage, f, indent=1, sort_keys=True)
    lib_key = _digest([o + '.sha256' for o in objs], [ARCH])
    if force or _stale(LIB, lib_key):
        cmd = [hipcc(), '-shared', '-fPIC', '--offload-arch=' + ARCH, '-o', LIB] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError('link failed:\n%s\n%s' % (' '.join(cmd), r.stderr))
        _mark(LIB, lib_key)
        if verbose:
            print('built', LIB)
    build_fastcall(force=force, verbose=verbose)
    build_hostpack(force=force, verbose=verbose)
    with open(STAMP, 'w') as f:
        json.dump({'digest': source_digest(), 'arch': ARCH,
                   'sources': [os.path.relpath(p, REPO) for p in source_files()]}, f, indent=1)
    return LIB


FASTCALL_SRC = os.path.join(OBJDIR, '_sbodcall.c')
FASTCALL_LIB = os.path.join(PKG, 'lib', '_sbodcall.so')

# ctypes type name -> (C declaration, converter expression over PyObject *o, error test)
_CONV = {
    'c_void_p': ('void *', 'cv_ptr(o, &ok)'),
    'c_int': ('int', '(int)PyLong_AsLong(o)'),
    'c_long': ('long long', 'PyLong_AsLongLong(o)'),
    'c_float': ('float', '(float)PyFloat_AsDouble(o)'),
    'c_double': ('double', 'PyFloat_AsDouble(o)'),
    'c_ulong': ('size_t', 'PyLong_AsSize_t(o)'),
}


def _fastcall_source(signatures):
    """C source of the _sbodcall extension: a wrapper per entry point returning int or size_t."""
    import ctypes
    out = ['/* generated by build.py from _lib.SIGNATURES: do not edit */',
           '#define PY_SSIZE_T_CLEAN', '#include <Python.h>', '#include "sbod.h"', '',
           'static inline void *cv_ptr(PyObject *o, int *ok) {',
           '  if (o == Py_None) return NULL;',
           '  void *p = PyLong_AsVoidPtr(o);',
           '  if (p == NULL && PyErr_Occurred()) *ok = 0;',
           '  return p;', '}', '']
    names = []
    for name, (res, args) in signatures.items():
        if res not in (ctypes.c_int, ctypes.c_size_t):
            continue
        if any(t.__name__ not in _CONV for t in args):
            continue
        names.append(name)
        n = len(args)
        out.append('static PyObject *w_%s(PyObject *self, PyObject *const *a, Py_ssize_t n) {' % name)
        out.append('  (void)self;')
        out.append('  if (n != %d) { PyErr_SetString(PyExc_TypeError, "%s: expected %d arguments"); '
                   'return NULL; }' % (n, name, n))
        out.append('  int ok = 1;%s' % (' PyObject *o;' if n else ' (void)a;'))
        for i, t in enumerate(args):
            decl, conv = _CONV[t.__name__]
            out.append('  o = a[%d]; %s v%d = %s;' % (i, decl, i, conv))
        out.append('  if (!ok || PyErr_Occurred()) return NULL;')
        call = '%s(%s)' % (name, ', '.join('v%d' % i for i in range(n)))
        if res is ctypes.c_int:
            out.append('  return PyLong_FromLong(%s);' % call)
        else:
            out.append('  return PyLong_FromSize_t(%s);' % call)
        out.append('}')
        out.append('')
    out.append('static PyMethodDef methods[] = {')
    for name in names:
        out.append('  {"%s", (PyCFunction)(void (*)(void))w_%s, METH_FASTCALL, NULL},' % (name, name))
    out.append('  {NULL, NULL, 0, NULL}};')
    out.append('static struct PyModuleDef mod = {PyModuleDef_HEAD_INIT, "_sbodcall", NULL, -1, methods};')
    out.append('PyMODINIT_FUNC PyInit__sbodcall(void) { return PyModule_Create(&mod); }')
    return '\n'.join(out) + '\n'


def build_fastcall(force=False, verbose=True):
    """Generate and compile lib/_sbodcall.so (gcc, CPython headers), linked to libsbod_hip.so."""
    import sysconfig
    from . import _lib
    src = _fastcall_source(_lib.SIGNATURES)
    old = open(FASTCALL_SRC).read() if os.path.exists(FASTCALL_SRC) else None
    if old != src:
        with open(FASTCALL_SRC, 'w') as f:
            f.write(src)
    key = _digest([FASTCALL_SRC, _key_path(LIB)] + _deps())
    if force or _stale(FASTCALL_LIB, key):
        cc = shutil.which('gcc') or 'cc'
        cmd = [cc, '-O2', '-shared', '-fPIC', '-Wall', '-Werror', '-I', sysconfig.get_paths()['include'],
               '-I', INCLUDE, FASTCALL_SRC, '-o', FASTCALL_LIB, '-L', os.path.dirname(LIB), '-lsbod_hip',
               '-Wl,-rpath,$ORIGIN']
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError('fastcall build failed:\n%s\n%s' % (' '.join(cmd), r.stderr))
        _mark(FASTCALL_LIB, key)
        if verbose:
            print('built', FASTCALL_LIB)
    return FASTCALL_LIB


HOSTPACK_SRC = os.path.join(CSRC, 'hostpack.cpp')
HOSTPACK_LIB = os.path.join(PKG, 'lib', '_sbodhost.so')


def build_hostpack(force=False, verbose=True):
    """Compile lib/_sbodhost.so (g++ against the installed torch's headers and libraries):
    the per-step GT list checks + packing launch in C++ (csrc/hostpack.cpp)."""
    import sysconfig
    import torch
    tdir = os.path.dirname(torch.__file__)
    key = _digest([HOSTPACK_SRC, _key_path(LIB)] + _deps(), [torch.__version__])
    if force or _stale(HOSTPACK_LIB, key):
        cxx = shutil.which('g++') or 'c++'
        abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
        tlib = os.path.join(tdir, 'lib')
        cmd = [cxx, '-O2', '-std=c++17', '-shared', '-fPIC', '-Wall', '-Wno-unused-parameter',
               '-D_GLIBCXX_USE_CXX11_ABI=%d' % abi, '-DUSE_ROCM',
               '-I', sysconfig.get_paths()['include'], '-I', INCLUDE,
               '-I', os.path.join(tdir, 'include'),
               '-I', os.path.join(tdir, 'include', 'torch', 'csrc', 'api', 'include'),
               HOSTPACK_SRC, '-o', HOSTPACK_LIB,
               '-L', os.path.dirname(LIB), '-lsbod_hip', '-L', tlib, '-lc10', '-ltorch', '-ltorch_cpu',
               '-ltorch_python', '-Wl,-rpath,$ORIGIN', '-Wl,-rpath,' + tlib]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError('hostpack build failed:\n%s\n%s' % (' '.join(cmd), r.stderr))
        _mark(HOSTPACK_LIB, key)
        if verbose:
            print('built', HOSTPACK_LIB)
    return HOSTPACK_LIB


if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    ap.add_argument('--force', action='store_true')
    ap.add_argument('-j', type=int, default=8)
    a = ap.parse_args()
    build(force=a.force, jobs=a.j)

#!/usr/bin/env python3
"""Host AddressSanitizer + UBSan build of the C ABI's host side, CPU only.

Builds into variants/asan/ (never the product lib/):
  * libsbod_hip.so — every csrc/*.hip with the sanitizers on the HOST code only
    (``-Xarch_host -fsanitize=...``; GPU AddressSanitizer is not available on this pool, and the
    device code is not what these tests reach): the argument / workspace validation every entry
    point runs before its first launch;
  * _sbodhost.so — csrc/hostpack.cpp (the collate_fn list walk, pointer and count tables) with
    clang's sanitizers, so one ASan runtime (clang's) serves both;
  * _sbodcall.so — the generated METH_FASTCALL wrappers, likewise.

Run the host tests under it with scripts/asan_host.sh (LD_PRELOAD of clang's ASan runtime; no
GPU is touched: every case fails validation or works on host memory only).
"""
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)

from shape_based_object_detection_amd import build as B  # noqa: E402

OUT = os.path.join(REPO, 'variants', 'asan')
SAN = ['-fsanitize=address,undefined', '-fno-omit-frame-pointer', '-fno-sanitize-recover=undefined']
CLANG = '/opt/rocm/lib/llvm/bin/clang++'
CLANGC = '/opt/rocm/lib/llvm/bin/clang'


def run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise SystemExit('failed: %s\n%s' % (' '.join(cmd), r.stderr[-4000:]))


def main():
    os.makedirs(OUT, exist_ok=True)
    objs = []
    flags = [f for f in B.CXXFLAGS if f != '-O3'] + ['-O1', '-g']
    for src in sorted(os.listdir(B.CSRC)):
        if not src.endswith('.hip'):
            continue
        o = os.path.join(OUT, src + '.o')
        cmd = [B.hipcc()] + flags + ['-Xarch_host', SAN[0], '-Xarch_host', SAN[1], '-Xarch_host', SAN[2],
                                     '-c', os.path.join(B.CSRC, src), '-o', o]
        run(cmd)
        objs.append(o)
    lib = os.path.join(OUT, 'libsbod_hip.so')
    run([B.hipcc(), '-shared', '-fPIC', '--offload-arch=' + B.ARCH, '-fsanitize=address,undefined',
         '-shared-libsan', '-o', lib] + objs)
    import torch
    from shape_based_object_detection_amd import _lib
    tdir = os.path.dirname(torch.__file__)
    tlib = os.path.join(tdir, 'lib')
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    run([CLANG, '-O1', '-g', '-std=c++17', '-shared', '-fPIC', '-shared-libsan'] + SAN +
        ['-D_GLIBCXX_USE_CXX11_ABI=%d' % abi, '-DUSE_ROCM', '-Wno-unused-parameter',
         '-I', sysconfig.get_paths()['include'], '-I', B.INCLUDE, '-I', os.path.join(tdir, 'include'),
         '-I', os.path.join(tdir, 'include', 'torch', 'csrc', 'api', 'include'), B.HOSTPACK_SRC,
         '-o', os.path.join(OUT, '_sbodhost.so'), '-L', OUT, '-lsbod_hip', '-L', tlib, '-lc10', '-ltorch',
         '-ltorch_cpu', '-ltorch_python', '-Wl,-rpath,$ORIGIN', '-Wl,-rpath,' + tlib])
    csrc = os.path.join(OUT, '_sbodcall.c')
    with open(csrc, 'w') as f:
        f.write(B._fastcall_source(_lib.SIGNATURES))
    run([CLANGC, '-O1', '-g', '-shared', '-fPIC', '-shared-libsan'] + SAN +
        ['-I', sysconfig.get_paths()['include'], '-I', B.INCLUDE, csrc, '-o', os.path.join(OUT, '_sbodcall.so'),
         '-L', OUT, '-lsbod_hip', '-Wl,-rpath,$ORIGIN'])
    print('built', OUT)


if __name__ == '__main__':
    main()

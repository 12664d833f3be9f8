"""Build libsbod_hip.so in-tree with hipcc for gfx950 (no JIT cache, no setup.py install).

    python -m shape_based_object_detection_amd.build [--force] [-j N]

Compile flags that matter for parity: ``-ffp-contract=off`` (no FMA contraction: every
IoU / threshold expression rounds like the reference's separate torch kernels) and the
default IEEE fp32 division.
"""
import argparse
import concurrent.futures as cf
import glob
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


def _stale(target, sources):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


_RES_RE = re.compile(r'remark: +(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|'
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
    if force or _stale(obj, [src] + _deps()) or not os.path.exists(res):
        cmd = [hipcc()] + CXXFLAGS + ['-Rpass-analysis=kernel-resource-usage', '-c', src, '-o', obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError('hipcc failed for %s:\n%s\n%s' % (src, ' '.join(cmd), r.stderr))
        with open(res, 'w') as f:
            json.dump(_resource_usage(r.stderr), f, indent=1, sort_keys=True)
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
    if force or _stale(LIB, objs):
        cmd = [hipcc(), '-shared', '-fPIC', '--offload-arch=' + ARCH, '-o', LIB] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError('link failed:\n%s\n%s' % (' '.join(cmd), r.stderr))
        if verbose:
            print('built', LIB)
    return LIB


if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    ap.add_argument('--force', action='store_true')
    ap.add_argument('-j', type=int, default=8)
    a = ap.parse_args()
    build(force=a.force, jobs=a.j)

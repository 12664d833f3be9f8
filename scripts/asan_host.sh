#!/bin/bash
# Host ASan + UBSan run of the C ABI's host side, CPU only, in this container:
# builds variants/asan/ (scripts/build_asan.py) and runs the host tests against it with clang's
# ASan runtime preloaded (any LD_PRELOAD already set is kept after it).  No GPU is touched.
#   bash scripts/asan_host.sh [log]
set -o pipefail
cd "$(dirname "$0")/.."
LOG=${1:-profiles/r3_asan_host.log}
python scripts/build_asan.py || exit 1
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -n 1)
export ASAN_OPTIONS=detect_leaks=0:alloc_dealloc_mismatch=0:detect_odr_violation=0:halt_on_error=1:abort_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
{
  echo "# $(date -u +%FT%TZ) host ASan+UBSan: $RT"
  echo "# libsbod_hip.so (-Xarch_host sanitizers), _sbodhost.so, _sbodcall.so from variants/asan"
  LD_PRELOAD="$RT${LD_PRELOAD:+:$LD_PRELOAD}" SBOD_LIB=$PWD/variants/asan/libsbod_hip.so \
    timeout -k 10 900 python -m pytest -p no:cacheprovider -s tests/test_cpu_host.py tests/test_host_malformed.py \
    tests/test_host_path.py -q 2>&1
} | tee "$LOG"

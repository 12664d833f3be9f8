#!/bin/bash
# Debug build of the library with -DSBOD_PHASE_CLOCKS (per-phase cycle stamps via printf) as
# variants/libsbod_hip_phase.so; select it with SBOD_LIB=<path>.
set -e
cd "$(dirname "$0")/.."
OUT=variants/build_phase
mkdir -p variants
mkdir -p $OUT
for f in shape_based_object_detection_amd/csrc/*.hip; do
  hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -munsafe-fp-atomics -DSBOD_PHASE_CLOCKS \
    -Iinclude -Ishape_based_object_detection_amd/csrc -c $f -o $OUT/$(basename $f).o &
done
wait
hipcc -shared -fPIC --offload-arch=gfx950 -o variants/libsbod_hip_phase.so $OUT/*.o
echo built phase lib

#!/bin/bash
# Debug build of the library with -DSBOD_BLOCK_STAMPS (per-workgroup wall-clock start/end stamps) as
# variants/libsbod_hip_${NAME:-stamps}.so (extra compile flags in $EXTRA); select it with SBOD_LIB=<path>.
set -e
cd "$(dirname "$0")/.."
NAME=${NAME:-stamps}
OUT=variants/build_$NAME
mkdir -p variants
mkdir -p $OUT
for f in shape_based_object_detection_amd/csrc/*.hip; do
  hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -munsafe-fp-atomics -DSBOD_BLOCK_STAMPS $EXTRA \
    -Iinclude -Ishape_based_object_detection_amd/csrc -c $f -o $OUT/$(basename $f).o &
done
wait
hipcc -shared -fPIC --offload-arch=gfx950 -o variants/libsbod_hip_$NAME.so $OUT/*.o
echo built $NAME lib

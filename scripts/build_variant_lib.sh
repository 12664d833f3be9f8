#!/bin/bash
# Build an A/B variant library from a source tree (e.g. an older commit's csrc/include extracted
# with git archive; EXTRA="-D..." adds compile flags) into variants/libsbod_hip_<name>.so.
#   bash scripts/build_variant_lib.sh <name> <src_root>
set -e
cd "$(dirname "$0")/.."
NAME=$1; SRC=$2
OUT=variants/build_$NAME
mkdir -p variants
mkdir -p $OUT
for f in $SRC/shape_based_object_detection_amd/csrc/*.hip; do
  hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -munsafe-fp-atomics $EXTRA \
    -I$SRC/include -I$SRC/shape_based_object_detection_amd/csrc -c $f -o $OUT/$(basename $f).o &
done
wait
hipcc -shared -fPIC --offload-arch=gfx950 -o variants/libsbod_hip_$NAME.so $OUT/*.o
echo built $NAME

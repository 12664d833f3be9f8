#!/bin/bash
# Build an A/B variant of libsbod_hip.so from THIS tree with extra compile flags into
# shape_based_object_detection_amd/lib/variants/libsbod_hip_<name>.so (travels with the tree to
# the GPU box; loaded only when SBOD_LIB names it).   EXTRA="-D..." bash scripts/build_lib_variant.sh NAME
set -e
cd "$(dirname "$0")/.."
NAME=$1
OUT=gpurun_out/vbuild_$NAME
LIBV=shape_based_object_detection_amd/lib/variants
mkdir -p $OUT $LIBV
for f in shape_based_object_detection_amd/csrc/*.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -munsafe-fp-atomics $EXTRA \
    -Iinclude -Ishape_based_object_detection_amd/csrc -c $f -o $OUT/$(basename $f).o &
done
wait
for f in shape_based_object_detection_amd/csrc/*.hip; do test $OUT/$(basename $f).o -nt $f || { echo "compile failed: $f"; exit 1; }; done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $LIBV/libsbod_hip_$NAME.so $OUT/*.o
echo built $LIBV/libsbod_hip_$NAME.so
# a full variant directory too: the library under its product name next to copies of the two
# CPython extensions (they link libsbod_hip.so through RUNPATH $ORIGIN), so SBOD_LIB=<dir>/libsbod_hip.so
# runs the bench's native submit path against the variant
mkdir -p $LIBV/$NAME
cp $LIBV/libsbod_hip_$NAME.so $LIBV/$NAME/libsbod_hip.so
cp shape_based_object_detection_amd/lib/_sbodcall.so shape_based_object_detection_amd/lib/_sbodhost.so $LIBV/$NAME/ 2>/dev/null || true

#!/bin/bash
# Device assembly of one csrc/*.hip file with the library's flags (diagnostic, CPU only):
#   bash scripts/isa.sh match  -> /tmp/isa/match.s
set -e
cd "$(dirname "$0")/.."
mkdir -p /tmp/isa
FLAGS=$(python3 -c "import sys; sys.path.insert(0,'.'); from shape_based_object_detection_amd import build as b; print(' '.join(b.CXXFLAGS))")
hipcc $FLAGS --cuda-device-only -S shape_based_object_detection_amd/csrc/$1.hip -o /tmp/isa/$1.s

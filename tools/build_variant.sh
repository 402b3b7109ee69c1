#!/bin/bash
# Build libfdf.so of the working tree with extra compile definitions into
# build/libfdf_<NAME>.so, for A/B timing in one process pool:
#   tools/build_variant.sh ring8 "-DFDF_RING_MAXT=8 -DFDF_RING_SAD=8"
#   FDF_LIB_PATH=build/libfdf_ring8.so python tools/ablate.py ...
set -e
NAME=${1:?name}; DEFS=${2:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d /tmp/fdf_var_XXXX)
mkdir -p "$TMP/feature_detector_fast_amd"
cp -r "$ROOT/include" "$ROOT/Makefile" "$TMP/"
cp -r "$ROOT/feature_detector_fast_amd/csrc" "$TMP/feature_detector_fast_amd/"
rm -f "$TMP"/feature_detector_fast_amd/csrc/*.o
make -C "$TMP" -j8 feature_detector_fast_amd/libfdf.so EXTRA_HIPFLAGS="$DEFS" > /dev/null
mkdir -p "$ROOT/build"
cp "$TMP/feature_detector_fast_amd/libfdf.so" "$ROOT/build/libfdf_$NAME.so"
rm -rf "$TMP"
echo "$ROOT/build/libfdf_$NAME.so"

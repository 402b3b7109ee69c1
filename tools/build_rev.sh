#!/bin/bash
# Build libfdf.so of git revision REV into build/libfdf_<REV>.so (for A/B timing against the
# working tree: FDF_LIB_PATH=build/libfdf_<REV>.so python tools/ablate.py ...).
set -e
REV=${1:?revision}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d /tmp/fdf_rev_XXXX)
git -C "$ROOT" worktree add -q --detach "$TMP" "$REV"
make -C "$TMP" -j8 feature_detector_fast_amd/libfdf.so > /dev/null
mkdir -p "$ROOT/build"
cp "$TMP/feature_detector_fast_amd/libfdf.so" "$ROOT/build/libfdf_$REV.so"
git -C "$ROOT" worktree remove --force "$TMP"
echo "$ROOT/build/libfdf_$REV.so"

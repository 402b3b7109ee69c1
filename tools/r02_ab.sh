#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-ab}; shift
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "full_geometry or golden or random or tiers or config4" > $O/pytest_new.log 2>&1 || { echo "new pytest failed"; tail -20 $O/pytest_new.log; exit 1; }
tail -1 $O/pytest_new.log
FDF_LIB_PATH=build/libfdf_sel.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "full_geometry or golden or random or tiers or config4" > $O/pytest_sel.log 2>&1 || { echo "sel pytest failed"; tail -20 $O/pytest_sel.log; }
tail -1 $O/pytest_sel.log
bash tools/ab_interleave.sh $O/ab1080.txt 3 "maxt:0,off:0,sad:0" "" build/libfdf_HEAD.so feature_detector_fast_amd/libfdf.so build/libfdf_sel.so > $O/ab1080.sum || exit 1
cat $O/ab1080.sum
bash tools/ab_interleave.sh $O/ab4k.txt 2 "sad:0,off:0" "--width 3840 --height 2160 --frames 128 --threshold 8 --count 12" build/libfdf_HEAD.so feature_detector_fast_amd/libfdf.so build/libfdf_sel.so > $O/ab4k.sum || exit 1
cat $O/ab4k.sum

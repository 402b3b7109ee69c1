#!/bin/bash
# Session check: HEAD library (in-tree) gpu tests + bench line; candidate build (build/libfdf_new.so)
# parity tests, interleaved A/B against HEAD, single-frame latency of both.
set -o pipefail
O=gpurun_out/s2; mkdir -p $O
NEW=build/libfdf_new.so
timeout -k 10 300 python bench.py > $O/bench_head.json 2> $O/bench_head.err || { tail $O/bench_head.err; exit 1; }
echo bench-head-ok
FDF_LIB_PATH=$NEW timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_new.log 2>&1 || { tail -30 $O/pytest_new.log; exit 1; }
tail -2 $O/pytest_new.log
for r in 1 2; do
  bash tools/ab_libs.sh $O/ab_$r.txt off:0,maxt:0,sad:0 feature_detector_fast_amd/libfdf.so $NEW || exit 1
  cat $O/ab_$r.txt
done
for L in feature_detector_fast_amd/libfdf.so $NEW; do
  for m in off maxt; do
    FDF_LIB_PATH=$L timeout -k 10 120 python3 tools/single_frame.py --nms $m || exit 1
  done
done > $O/single.txt
cat $O/single.txt
echo s2-done

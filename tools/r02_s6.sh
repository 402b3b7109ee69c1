#!/bin/bash
# Candidate build/libfdf_cu8.so (compaction copies 8 points per thread per round): gpu api
# and parity tests, interleaved A/B of the whole step (detector + compaction) against the tree.
set -o pipefail
O=gpurun_out/s6; mkdir -p $O
NEW=build/libfdf_cu8.so
FDF_LIB_PATH=$NEW timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_cu8.log 2>&1 || { tail -30 $O/pytest_cu8.log; exit 1; }
tail -2 $O/pytest_cu8.log
for r in 1 2 3; do
  bash tools/ab_libs.sh $O/ab_$r.txt off:0,maxt:0 feature_detector_fast_amd/libfdf.so $NEW || exit 1
  cat $O/ab_$r.txt
done
echo s6-done

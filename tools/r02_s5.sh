#!/bin/bash
# Candidate build/libfdf_slot4.so (4x slots for grids that cannot fill the chip): gpu parity
# tests, single-frame latency against the in-tree build, batch A/B (unchanged path).
set -o pipefail
O=gpurun_out/s5; mkdir -p $O
NEW=build/libfdf_slot4.so
FDF_LIB_PATH=$NEW timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_slot4.log 2>&1 || { tail -30 $O/pytest_slot4.log; exit 1; }
tail -2 $O/pytest_slot4.log
for r in 1 2; do for L in feature_detector_fast_amd/libfdf.so $NEW; do
  for m in off maxt sad; do
    echo "$L $(FDF_LIB_PATH=$L timeout -k 10 120 python3 tools/single_frame.py --nms $m)" || exit 1
  done
done; done > $O/single.txt
cat $O/single.txt
bash tools/ab_libs.sh $O/ab_1.txt off:0,maxt:0 feature_detector_fast_amd/libfdf.so $NEW || exit 1
cat $O/ab_1.txt
echo s5-done

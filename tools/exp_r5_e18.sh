#!/bin/bash
# Round 5 e18 (variant macro not kept; add "#ifdef FDF_LAT_AGE / #define FDF_MAX_AGE FDF_LAT_AGE" to fdf_sweep_latency.hip
# to rebuild): the latency instances issue partial batches once a candidate is 1 or 2 rows old.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_e18
mkdir -p $O
for r in 1 2 3; do
  for L in feature_detector_fast_amd/libfdf.so build/libfdf_age1.so build/libfdf_age2.so; do
    for nm in maxt off; do
      echo -n "$(basename $L) " >> $O/single.txt
      FDF_LIB_PATH=$L timeout -k 10 60 python3 tools/single_frame.py --nms $nm --iters 300 >> $O/single.txt
    done
  done
done

#!/bin/bash
# Round 5 e17 (variant macro not kept in the source; add "#define FDF_SWEEP_TU_WAVES FDF_LAT_WAVES" to fdf_sweep_latency.hip to rebuild): the latency instances occupancy target (FDF_LAT_WAVES: 4 default, 2, 1 waves
# per SIMD, i.e. 128 / 256 / 512 VGPRs): single device-resident 1080p frames, interleaved.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_e17
mkdir -p $O
for r in 1 2 3; do
  for L in feature_detector_fast_amd/libfdf.so build/libfdf_lat2.so build/libfdf_lat1.so; do
    for nm in maxt off; do
      echo -n "$(basename $L) " >> $O/single.txt
      FDF_LIB_PATH=$L timeout -k 10 60 python3 tools/single_frame.py --nms $nm --iters 300 >> $O/single.txt
    done
  done
done

#!/bin/bash
# Round 5 e15: the sweep stops at a unit's last row instead of finishing its 8-step block
# (FDF_EARLY_EXIT), and a direct launch's ticket round trip runs under the band's LDS setup
# (FDF_TICKET_OVERLAP): single device frames and the batch configurations, interleaved
# against the base build of the same tree.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_e15
mkdir -p $O
LIBS="${LIBS:-feature_detector_fast_amd/libfdf.so build/libfdf_ee.so build/libfdf_to.so build/libfdf_eeto.so}"; O=${OUT:-$O}; mkdir -p $O
for r in 1 2 3; do
  for L in $LIBS; do
    for nm in maxt off; do
      echo -n "$(basename $L) " >> $O/single.txt
      FDF_LIB_PATH=$L timeout -k 10 60 python3 tools/single_frame.py --nms $nm --iters 300 >> $O/single.txt
    done
  done
done
timeout -k 10 600 bash tools/ab_interleave.sh $O/ab_1080.txt 3 "maxt:0,off:0,sad:0" "--frames 512" $LIBS > $O/ab_1080.log 2>&1
tail -4 $O/ab_1080.log
timeout -k 10 600 bash tools/ab_interleave.sh $O/ab_4k.txt 3 "sad:0" "--frames 128 --width 3840 --height 2160 --threshold 8 --count 12" $LIBS > $O/ab_4k.log 2>&1
tail -4 $O/ab_4k.log

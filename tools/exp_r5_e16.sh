#!/bin/bash
# (The latency instances measured here are in commit 3307c16, taken out again: DESIGN.md §7.5.)
# Round 5 e16: latency instances (fdf_sweep_latency.hip: units leave their last 8-step block
# at their last row) for grids whose units end inside a block.  The GPU suite on the new
# library, then single device frames and the batch configurations against the previous build
# (build/libfdf_base.so), interleaved.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_e16
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
LIBS="build/libfdf_base.so feature_detector_fast_amd/libfdf.so"
for r in 1 2 3; do
  for L in $LIBS; do
    for nm in maxt off; do
      echo -n "$(basename $L) " >> $O/single.txt
      FDF_LIB_PATH=$L timeout -k 10 60 python3 tools/single_frame.py --nms $nm --iters 300 >> $O/single.txt
    done
    echo -n "$(basename $L) " >> $O/host.txt
    FDF_LIB_PATH=$L timeout -k 10 120 python3 tools/host_latency.py --iters 300 --modes off,maxt --mem pinned --chunks 0 >> $O/host.txt
  done
done
timeout -k 10 600 bash tools/ab_interleave.sh $O/ab_1080.txt 3 "maxt:0,off:0,sad:0" "--frames 512" $LIBS > $O/ab_1080.log 2>&1
tail -2 $O/ab_1080.log
timeout -k 10 600 bash tools/ab_interleave.sh $O/ab_64.txt 3 "maxt:0,off:0" "--frames 64" $LIBS > $O/ab_64.log 2>&1
tail -2 $O/ab_64.log

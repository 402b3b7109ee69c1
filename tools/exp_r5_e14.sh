#!/bin/bash
# Round 5 e14: the in-launch upload (copier workgroups move the pinned frame into HBM, each
# byte once over the link, the bands wait per chunk): host-path parity, then the end-to-end
# fdf_detect A/B against reading in place (FDF_UP_COPIERS=0) and 16 / 64 copiers, interleaved.
# The copier code is on branch exp-inlaunch-upload (not kept: DESIGN.md §7.5); build the
# variants there with tools/build_variant.sh upN "-DFDF_UP_COPIERS=N".
set -e
OUT=gpurun_out/r5_e14
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -q --timeout 120 --timeout-method thread \
  tests/test_gpu_host_inplace.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
for r in 1 2 3; do
  for lib in build/libfdf_up0.so feature_detector_fast_amd/libfdf.so build/libfdf_up16.so build/libfdf_up64.so; do
    echo -n "$lib " >> $OUT/host_ab.txt
    FDF_LIB_PATH=$lib timeout -k 10 120 python3 tools/host_latency.py --iters 300 \
      --modes off,maxt --mem pinned --chunks 0 >> $OUT/host_ab.txt
  done
done
cat $OUT/host_ab.txt

#!/bin/bash
# parity of the working tree's library (max-t keypoint queue), then an interleaved A/B of
# build/libfdf_base.so (no queue), build/libfdf_new.so (queue) and build/libfdf_new2.so
# (queue + batch codes kept in registers)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_stress.py tests/test_gpu_scored.py > gpurun_out/ab4_tests.log 2>&1 || { tail -30 gpurun_out/ab4_tests.log; exit 1; }
tail -2 gpurun_out/ab4_tests.log
bash tools/ab_interleave.sh gpurun_out/ab4_1080.txt 4 "off:0,maxt:0,sad:0" "" build/libfdf_base.so build/libfdf_new.so build/libfdf_new2.so | tail -3 || exit 1
bash tools/ab_interleave.sh gpurun_out/ab4_4k.txt 3 "sad:0,maxt:0" "--frames 128 --width 3840 --height 2160 --threshold 8 --count 12" build/libfdf_base.so build/libfdf_new.so build/libfdf_new2.so | tail -3

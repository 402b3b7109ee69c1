#!/bin/bash
# parity of the working tree's library, then interleaved A/B of build/libfdf_base.so vs build/libfdf_new.so
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_stress.py > gpurun_out/ab3_tests.log 2>&1 || { tail -30 gpurun_out/ab3_tests.log; exit 1; }
tail -2 gpurun_out/ab3_tests.log
bash tools/ab_interleave.sh gpurun_out/ab3_1080.txt 4 "off:0,maxt:0,sad:0" "" build/libfdf_base.so build/libfdf_new.so | tail -2 || exit 1
bash tools/ab_interleave.sh gpurun_out/ab3_4k.txt 3 "sad:0" "--frames 128 --width 3840 --height 2160 --threshold 8 --count 12" build/libfdf_base.so build/libfdf_new.so | tail -2

#!/bin/bash
# 5 waves per SIMD (96 VGPRs) with <= 32 KB LDS per workgroup vs the default 4-wave build
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
bash tools/ab_interleave.sh gpurun_out/w5_1080.txt 3 "off:0:0,off:0:32000,off:0:30000,maxt:0:0,maxt:0:32000,sad:0:32000" "" build/libfdf_debug.so build/libfdf_w5dbg.so | tail -2

#!/bin/bash
# Round 5 e13: host round trip of a tiny launch (blocking vs polled), and the link's read rate
# for a 1080p frame of pinned host memory read by a kernel, each byte once, by grid size.
set -e
OUT=gpurun_out/r5_e13
mkdir -p $OUT
timeout -k 10 120 ./build/sync_latency > $OUT/sync_latency2.txt

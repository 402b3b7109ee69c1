#!/bin/bash
# Round-2 record on the GPU box: default bench line, rocprofv3 kernel stats + PMC traffic for
# max-t / off (1080p) and config 5 (4K), a 4096-frame batch, single-frame traces.
set -o pipefail
O=gpurun_out/rec
mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
bash tools/profile_round.sh maxt --nms maxt > $O/prof_maxt.log 2>&1 || exit 1
bash tools/profile_round.sh off --nms off > $O/prof_off.log 2>&1 || exit 1
bash tools/profile_round.sh 4k --width 3840 --height 2160 --frames 128 --threshold 8 --count 12 --nms sad > $O/prof_4k.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --frames 4096 --steps 5 --warmup 2 --no-extras --cpu-seconds 0 > $O/bench_4096.json 2> $O/bench_4096.err || exit 1
timeout -k 10 300 python bench.py --frames 4096 --steps 5 --warmup 2 --no-extras --cpu-seconds 0 --nms off > $O/bench_4096_off.json 2> $O/bench_4096_off.err || exit 1
bash tools/r02_single.sh rec/single > $O/single.log 2>&1 || exit 1
echo record-done

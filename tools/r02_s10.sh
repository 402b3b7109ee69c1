#!/bin/bash
# Round-2 extras: PCIe-inclusive streaming pipeline (host frames in, keypoints out) and the
# per-GPU shard of BASELINE config 4 at 8 GPUs (64 frames, rotated through HBM copies).
set -o pipefail
O=gpurun_out/s10; mkdir -p $O
timeout -k 10 300 python3 tools/stream_bench.py > $O/stream_bench.jsonl 2> $O/stream_bench.err || { tail $O/stream_bench.err; exit 1; }
cat $O/stream_bench.jsonl
for m in maxt off; do
  timeout -k 10 200 python3 bench.py --frames 64 --nms $m --cpu-seconds 0 --no-extras > $O/shard64_$m.json 2> $O/shard64_$m.err || exit 1
  cat $O/shard64_$m.json
done
echo s10-done

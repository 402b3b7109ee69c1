#!/bin/bash
# Quick GPU iteration: selected tests (-k EXPR), short bench lines (max-t, off), 4K ablation.
set -o pipefail
O=gpurun_out/${1:-r02q}; K=${2:-"stress or api or parity"}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for m in maxt off; do
  timeout -k 10 200 python bench.py --nms $m --cpu-seconds 0 --no-extras > $O/q_$m.json 2> $O/q_$m.err || exit 1
done
timeout -k 10 200 python tools/ablate.py --width 3840 --height 2160 --frames 128 --threshold 8 --count 12 \
   --variants sad:0,sad:16,off:0,maxt:0 > $O/ablate4k.json 2> $O/ablate4k.err || exit 1
echo done

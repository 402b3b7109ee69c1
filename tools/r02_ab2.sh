#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-ab}; shift
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
bash tools/ab_interleave.sh $O/ab1080.txt 3 "maxt:0,off:0,sad:0" "" "$@" > $O/ab1080.sum || exit 1
cat $O/ab1080.sum
bash tools/ab_interleave.sh $O/ab4k.txt 2 "sad:0,maxt:0" "--width 3840 --height 2160 --frames 128 --threshold 8 --count 12" "$@" > $O/ab4k.sum || exit 1
cat $O/ab4k.sum

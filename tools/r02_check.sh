#!/bin/bash
# GPU check of the working tree: parity/API tests, the default bench line (with extras and
# the CPU baseline), and a 4K config-5 ablation with the debug build.
set -o pipefail
O=gpurun_out/${1:-r02c}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
timeout -k 10 200 python tools/ablate.py --width 3840 --height 2160 --frames 128 --threshold 8 --count 12 \
   --variants sad:0,sad:1,sad:64,sad:16,off:0 > $O/ablate4k.json 2> $O/ablate4k.err || exit 1
echo done

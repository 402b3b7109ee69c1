#!/bin/bash
# Round record on the GPU box: parity tests, default bench line, per-mode bench lines and
# rocprof kernel stats + PMC traffic (tools/profile_round.sh).  Outputs under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/bench_maxt.json 2> gpurun_out/bench_maxt.err || exit 1
timeout -k 10 200 python bench.py --nms off --cpu-seconds 0 > gpurun_out/bench_off.json 2> gpurun_out/bench_off.err || exit 1
timeout -k 10 200 python bench.py --nms sad --cpu-seconds 0 > gpurun_out/bench_sad.json 2> gpurun_out/bench_sad.err || exit 1
bash tools/profile_round.sh maxt --nms maxt > gpurun_out/prof_maxt.log 2>&1 || exit 1
bash tools/profile_round.sh off --nms off > gpurun_out/prof_off.log 2>&1 || exit 1
echo round-done

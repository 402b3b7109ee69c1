#!/bin/bash
# Parity tests + short bench lines for all three modes (no CPU baseline / extras).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 ; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
for m in maxt off sad; do
  timeout -k 10 200 python bench.py --nms $m --cpu-seconds 0 --no-extras > gpurun_out/q_$m.json 2> gpurun_out/q_$m.err || exit 1
done

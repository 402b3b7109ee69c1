#!/bin/bash
# Full GPU check: every -m gpu test, quick bench lines (max-t, off), single-frame timing.
set -o pipefail
O=gpurun_out/${1:-full}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for m in maxt off; do
  timeout -k 10 200 python bench.py --nms $m --cpu-seconds 0 --no-extras > $O/q_$m.json 2> $O/q_$m.err || exit 1
  python -c "import json; d=json.load(open('$O/q_$m.json')); r=d['roofline']; print('$m', d['value'], r['kernel_ms_avg'], r['frac'], r['compaction_kernel_ms_avg'])"
done
for m in off maxt; do
  timeout -k 10 120 python3 tools/single_frame.py --nms $m > $O/single_$m.json 2> $O/single_$m.err || exit 1
  cat $O/single_$m.json
done

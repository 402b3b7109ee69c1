#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-rgb}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "rgb or golden or full_geometry or tiers" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python tools/rgb_bench.py > $O/rgb.json 2> $O/rgb.err || { tail $O/rgb.err; exit 1; }
cat $O/rgb.json

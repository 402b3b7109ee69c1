#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-single}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for m in off maxt; do
  timeout -k 10 120 python3 tools/single_frame.py --nms $m > $O/single_$m.json 2> $O/single_$m.err || exit 1
  cat $O/single_$m.json
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/trace_$m -o p -- python3 tools/single_frame.py --nms $m --iters 50 > $O/trace_$m.json 2> $O/trace_$m.err || exit 1
done
echo done

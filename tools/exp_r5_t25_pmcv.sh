#!/bin/bash
# Round 5 t25: instruction counts per detector launch of the final kernels (VERDICT r04 item 3's
# measure): SQ_INSTS_VALU / SALU / LDS / VMEM and waves, one lane (serialised dispatches), at
# 512 x 1080p max-t / off / SAD and 128 x 4K t=8 n=12 SAD.  One --pmc pass per configuration.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/t25_pmcv
mkdir -p $O
SHORT="--steps 6 --warmup 1 --settle-seconds 0 --cpu-seconds 0 --no-extras --no-parity --lanes 1"
run() {
  local tag=$1; shift
  timeout -k 10 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES \
      --output-format csv -d "$O/$tag" -o p -- python3 bench.py $SHORT "$@" > "$O/$tag.json" 2> "$O/$tag.log"
  python3 tools/pmc_summary.py "$O/$tag" > "$O/${tag}_summary.json"
  rm -rf "$O/$tag"
}
run maxt --nms maxt
run off --nms off
run sad --nms sad
run 4k --width 3840 --height 2160 --frames 128 --threshold 8 --count 12 --nms sad
cat $O/*_summary.json

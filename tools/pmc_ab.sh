#!/bin/bash
# Instruction / cycle counters of one ablation variant for several library builds.
# Usage: tools/pmc_ab.sh OUT VARIANT lib1 lib2 ...
O=$1; V=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$O"
for L in "$@"; do
  n=$(basename "$L" .so)
  i=0
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_BUSY_CYCLES" \
             "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
             "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE"; do
    i=$((i+1)); D="$O/$n/p$i"; mkdir -p "$D"
    FDF_LIB_PATH=$L timeout -k 10 120 rocprofv3 --pmc $set -d "$D" -o p --output-format csv -- \
        python3 tools/ablate.py --rounds 1 --iters 1 --variants "$V" > "$D.log" 2>&1 || echo "pass $i failed $n"
  done
  echo "== $n $V"
  python3 tools/pmc_summary.py "$O/$n"/p* | grep -v '"p[0-9]"\|_dispatches\|^  }'
  rm -rf "$O/$n"
done

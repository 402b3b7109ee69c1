#!/bin/bash
# Three SQ counter passes (mix, cycles, LDS) for each ablation variant given.
# Usage: tools/pmc_quick.sh OUTDIR VARIANT...
O=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for V in "$@"; do
  i=0
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH" \
             "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
             "SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES"; do
    i=$((i+1))
    D="$O/${V//:/_}/p$i"
    mkdir -p "$D"
    timeout -k 10 120 rocprofv3 --pmc $set -d "$D" -o p --output-format csv -- \
        python3 tools/ablate.py --rounds 1 --iters 1 --variants "$V" > "$D.log" 2>&1 || exit 1
  done
  echo "== $V"
  python3 tools/pmc_summary.py "$O/${V//:/_}"/p*
done

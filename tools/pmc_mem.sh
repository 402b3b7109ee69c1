#!/bin/bash
# Memory-pipeline counters (TA / TD / TCP / TCC) per ablation variant, one --pmc set per run.
# Usage: tools/pmc_mem.sh OUTDIR VARIANT...
O=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$O"
timeout -k 10 60 rocprofv3 -L > /tmp/counters.txt 2>&1 || true
grep -o "\bT[ACDP][A-Z]*_[A-Z0-9_]*\|GRBM_[A-Z_]*" /tmp/counters.txt | sort -u > "$O/counters_mem.txt" || true
for V in "$@"; do
  i=0
  for set in "TA_TA_BUSY_sum TA_BUFFER_LOAD_WAVEFRONTS_sum GRBM_GUI_ACTIVE GRBM_COUNT" \
             "TD_TD_BUSY_sum TD_LOAD_WAVEFRONT_sum" \
             "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum" \
             "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum" \
             "SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"; do
    i=$((i+1))
    D="$O/${V//:/_}/p$i"
    mkdir -p "$D"
    timeout -k 10 120 rocprofv3 --pmc $set -d "$D" -o p --output-format csv -- \
        python3 tools/ablate.py --rounds 1 --iters 1 --variants "$V" > "$D.log" 2>&1 || echo "pass $i failed for $V: $(tail -2 $D.log)"
  done
  echo "== $V"
  python3 tools/pmc_summary.py "$O/${V//:/_}"/p*
  rm -rf "$O/${V//:/_}"
done

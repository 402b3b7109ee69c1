#!/bin/bash
# ablation switches live in the debug build only (make debug)
export FDF_LIB_PATH=${FDF_LIB_PATH:-$(cd "$(dirname "$0")/.." && pwd)/build/libfdf_debug.so}
# Instruction-issue and instruction-cache counters for ablation variants (one --pmc set per
# rocprofv3 run).  Usage: tools/pmc_icache.sh OUTDIR VARIANT...
O=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$O"
timeout -k 10 60 rocprofv3 -L > /tmp/counters.txt 2>&1 || true
grep -o "SQC_[A-Z_]*\|SQ_I[A-Z_]*\|SQ_WAIT[A-Z_]*" /tmp/counters.txt | sort -u > "$O/counters_sq.txt" || true
for V in "$@"; do
  i=0
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_INSTS_SMEM" \
             "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY" \
             "SQ_IFETCH SQ_IFETCH_LEVEL SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM" \
             "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ"; do
    i=$((i+1))
    D="$O/${V//:/_}/p$i"
    mkdir -p "$D"
    timeout -k 10 120 rocprofv3 --pmc $set -d "$D" -o p --output-format csv -- \
        python3 tools/ablate.py --rounds 1 --iters 1 $ABL_ARGS --variants "$V" > "$D.log" 2>&1 || echo "pass $i failed for $V"
  done
  echo "== $V"
  python3 tools/pmc_summary.py "$O/${V//:/_}"/p*
  tail -3 "$O/${V//:/_}"/p*.log
  rm -rf "$O/${V//:/_}"
done

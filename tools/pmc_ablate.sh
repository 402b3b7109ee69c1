#!/bin/bash
# ablation switches live in the debug build only (make debug)
export FDF_LIB_PATH=${FDF_LIB_PATH:-$(cd "$(dirname "$0")/.." && pwd)/build/libfdf_debug.so}
# Timing of ablation variants (tools/ablate.py, interleaved rounds) plus one SQ instruction-mix
# --pmc pass per variant.  Usage: tools/pmc_ablate.sh OUTDIR VARIANT,VARIANT,...
O=$1; VS=$2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$O"
timeout -k 10 200 python3 tools/ablate.py --rounds 5 --iters 10 --variants "$VS" > "$O/ablate.json" 2> "$O/ablate.err" || exit 1
cat "$O/ablate.json"
for V in ${VS//,/ }; do
  D="$O/${V//:/_}"
  mkdir -p "$D"
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_BUSY_CYCLES -d "$D" -o p --output-format csv -- \
      python3 tools/ablate.py --rounds 1 --iters 1 --variants "$V" > "$D.log" 2>&1 || { echo "pmc failed $V"; exit 1; }
  echo "== $V"
  python3 tools/pmc_summary.py "$D"
  rm -rf "$D"
done

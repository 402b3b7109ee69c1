#!/bin/bash
# Memory-side counters of the detector per library build: for each lib,
# one FETCH_SIZE pass and one TCC_HIT/TCC_MISS pass over one launch of each workload (own
# rocprofv3 run per counter set, never combined with tracing).
#   tools/pmc_variants.sh OUTDIR "ABLATE_ARGS" VARIANTS lib1 lib2 ...
set -e
O=$1; AA=$2; VS=$3; shift 3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$O"
for L in "$@"; do
  N=$(basename "$L" .so)
  for set in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES"; do
    tag=$(echo "$set" | cut -d' ' -f1)
    FDF_LIB_PATH=$L timeout -k 10 120 rocprofv3 --pmc $set -d "$O/${N}_$tag" -o p --output-format csv -- \
        python3 tools/ablate.py --rounds 1 --iters 1 $AA --variants "$VS" > "$O/${N}_$tag.log" 2>&1
  done
  python3 tools/pmc_summary.py "$O/${N}_FETCH_SIZE" "$O/${N}_TCC_HIT_sum" "$O/${N}_SQ_INSTS_VALU" > "$O/${N}_summary.json"
done

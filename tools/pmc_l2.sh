#!/bin/bash
# L2 (TCC) hit/miss and EA traffic counters per ablation variant.  Usage: tools/pmc_l2.sh OUT VARIANT...
O=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$O"
timeout -k 10 60 rocprofv3 -L > /tmp/counters.txt 2>&1 || true
grep -o "TCC_[A-Z_0-9]*\|MALL[A-Z_0-9]*\|.*MALL.*" /tmp/counters.txt | sort -u | head -200 > "$O/counters_tcc.txt" || true
for V in "$@"; do
  i=0
  for set in "TCC_HIT_sum TCC_MISS_sum" "TCC_REQ_sum TCC_READ_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
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

#!/bin/bash
# Interleaved A/B of library builds on one box: R rounds, each running tools/ablate.py once
# per library (in-process medians of VARIANTS); prints per-library medians over the rounds.
#   tools/ab_interleave.sh OUT ROUNDS "VARIANTS" "ABLATE_ARGS" lib1 lib2 ...
O=$1; R=$2; VS=$3; AA=$4; shift 4
cd "$GRAFT_REPO_ROOT"
: > "$O"
for r in $(seq 1 $R); do
  for L in "$@"; do
    echo -n "$(basename $L) " >> "$O"
    FDF_LIB_PATH=$L timeout -k 10 200 python3 tools/ablate.py --rounds 3 --iters 10 $AA --variants "$VS" 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print(json.dumps({k:v['ms_median'] for k,v in d.items()}))" >> "$O" || exit 1
  done
done
python3 - "$O" <<'PY'
import json, sys, collections
res = collections.defaultdict(lambda: collections.defaultdict(list))
for line in open(sys.argv[1]):
    name, js = line.split(" ", 1)
    for k, v in json.loads(js).items():
        res[name][k].append(v)
for name, d in res.items():
    print(name, {k: round(sorted(v)[len(v) // 2], 4) for k, v in d.items()})
PY

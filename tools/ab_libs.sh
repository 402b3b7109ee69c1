#!/bin/bash
# A/B timing of library builds: tools/ab_libs.sh OUT VARIANTS lib1 lib2 ...  (ablate.py per lib)
O=$1; VS=$2; shift 2
cd "$GRAFT_REPO_ROOT"
for L in "$@"; do
  echo "== $L"
  FDF_LIB_PATH=$L timeout -k 10 200 python3 tools/ablate.py --rounds 5 --iters 10 --variants "$VS" 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print({k:v['ms_median'] for k,v in d.items()})" || exit 1
done > "$O" 2>&1

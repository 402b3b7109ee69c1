#!/bin/bash
# ablation switches live in the debug build only (make debug)
export FDF_LIB_PATH=${FDF_LIB_PATH:-$(cd "$(dirname "$0")/.." && pwd)/build/libfdf_debug.so}
# Calibrates the PMC traffic of the detector kernel: FETCH_SIZE / WRITE_SIZE of the normal
# run and of a run whose full tests are disabled (FDF_DEBUG_FLAGS=1: the row stream alone,
# the access pattern the x2 FETCH_SIZE correction is calibrated for), plus the L2 hit rate.
# Usage: tools/traffic_split.sh OUTDIR [bench args]
set -e
O=$1; shift
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-extras $*"
run() {  # name env counter
  env $2 timeout -k 10 300 rocprofv3 --pmc $3 --output-format csv -d "$O/$1" -o p -- $B > "$O/$1.json" 2> "$O/$1.log"
}
run fetch_full "FDF_DEBUG_FLAGS=0" FETCH_SIZE
run fetch_stream "FDF_DEBUG_FLAGS=1" FETCH_SIZE
run write_full "FDF_DEBUG_FLAGS=0" WRITE_SIZE
run l2 "FDF_DEBUG_FLAGS=0" "TCC_HIT_sum TCC_MISS_sum"
python3 - "$O" <<'PY'
import json, sys, os
sys.path.insert(0, "tools")
from pmc_summary import load
o = sys.argv[1]
res = {}
for name, ctr in (("fetch_full", "FETCH_SIZE"), ("fetch_stream", "FETCH_SIZE"),
                  ("write_full", "WRITE_SIZE"), ("l2", "TCC_HIT_sum"), ("l2", "TCC_MISS_sum")):
    per, _ = load(os.path.join(o, name), "fast_sweep")
    vals = [c[ctr] for c in per.values() if ctr in c]
    res[f"{name}:{ctr}"] = sum(vals) / len(vals) if vals else None
print(json.dumps(res, indent=1))
json.dump(res, open(os.path.join(o, "split.json"), "w"), indent=1)
PY

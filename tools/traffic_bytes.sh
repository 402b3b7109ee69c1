#!/bin/bash
# ablation switches live in the debug build only (make debug)
export FDF_LIB_PATH=${FDF_LIB_PATH:-$(cd "$(dirname "$0")/.." && pwd)/build/libfdf_debug.so}
# Read traffic of the detector kernel from request-size counters (bytes = 32/64/128 x the
# requests of each size), for the normal run and for the row stream alone (full tests
# disabled, FDF_DEBUG_FLAGS=1).  Usage: tools/traffic_bytes.sh OUTDIR [bench args]
set -e
O=$1; shift
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-extras $*"
for mode in 0 1; do
  i=0
  for set in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum" "TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum" \
             "TCC_EA0_RDREQ_DRAM_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
    i=$((i+1))
    env FDF_DEBUG_FLAGS=$mode timeout -k 10 300 rocprofv3 --pmc $set --output-format csv \
        -d "$O/m${mode}_$i" -o p -- $B > "$O/m${mode}_$i.json" 2> "$O/m${mode}_$i.log"
  done
done
python3 - "$O" <<'PY'
import json, sys, os, glob
sys.path.insert(0, "tools")
from pmc_summary import load
o = sys.argv[1]
out = {}
for mode in (0, 1):
    acc = {}
    for d in sorted(glob.glob(os.path.join(o, f"m{mode}_*"))):
        if not os.path.isdir(d):
            continue
        per, _ = load(d, "fast_sweep")
        for c in per.values():
            for k, v in c.items():
                acc.setdefault(k, []).append(v)
    avg = {k: sum(v) / len(v) for k, v in acc.items()}
    n128 = avg.get("TCC_EA0_RDREQ_128B_sum", 0)
    n64 = avg.get("TCC_EA0_RDREQ_64B_sum", 0)
    n32 = avg.get("TCC_EA0_RDREQ_32B_sum", 0)
    avg["read_bytes_by_size"] = 128 * n128 + 64 * n64 + 32 * n32
    out["full" if mode == 0 else "stream_only"] = avg
print(json.dumps(out, indent=1))
json.dump(out, open(os.path.join(o, "bytes.json"), "w"), indent=1)
PY
for d in "$O"/m*_*; do if [ -d "$d" ]; then rm -rf "$d"; fi; done

#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-budget3}
mkdir -p $O
export FDF_LIB_PATH=build/libfdf_debug.so
timeout -k 10 400 python3 tools/ablate.py --rounds 4 --iters 10 \
  --variants off:0:0,off:0:33000,off:0:37000,off:0:38000,off:0:40000,off:0:42000,maxt:0:0,maxt:0:38000,maxt:0:42000 > $O/b.json 2> $O/b.err || exit 1
python3 -c "import json; d=json.load(open('$O/b.json')); print({k:v['ms_median'] for k,v in d.items()})"

#!/bin/bash
# LDS budget (band height) re-check after this round's kernel changes: the in-tree kernels with
# the host geometry knobs compiled in (build/libfdf_geo.so), one process per budget, 2 rounds.
set -o pipefail
O=gpurun_out/s9; mkdir -p $O
L=build/libfdf_geo.so
run() { echo "$1 $2 $(FDF_LIB_PATH=$L FDF_LDS_BUDGET=$2 timeout -k 10 200 python3 tools/ablate.py --rounds 5 --iters 10 --variants $1 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print({k:v['ms_median'] for k,v in d.items()})")"; }
for r in 1 2; do
  for b in 30000 35000 40000; do run off:0 $b || exit 1; done
  for b in 34000 37000 40000; do run maxt:0,sad:0 $b || exit 1; done
done > $O/budget.txt
cat $O/budget.txt
echo s9-done

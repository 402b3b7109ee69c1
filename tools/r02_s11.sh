#!/bin/bash
# Candidate build/libfdf_rounds.so (small grids: band height by rounds x steps): gpu tests, then
# bench lines at 64 / 128 / 256 / 512 frames for max-t and off, in-tree vs candidate.
set -o pipefail
O=gpurun_out/s11; mkdir -p $O
NEW=build/libfdf_rounds.so
FDF_LIB_PATH=$NEW timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_rounds.log 2>&1 || { tail -30 $O/pytest_rounds.log; exit 1; }
tail -2 $O/pytest_rounds.log
for f in 64 128 256 512; do for m in maxt off; do for L in feature_detector_fast_amd/libfdf.so $NEW; do
  r=$(FDF_LIB_PATH=$L timeout -k 10 200 python3 bench.py --frames $f --nms $m --cpu-seconds 0 --no-extras --steps 30 --warmup 5 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel_ms_avg'], d.get('parity',{}).get('bit_exact'))") || exit 1
  echo "$f $m $L $r"
done; done; done > $O/frames.txt
cat $O/frames.txt
echo s11-done

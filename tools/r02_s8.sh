#!/bin/bash
# Candidate build/libfdf_nmsreg.so: gpu parity tests, interleaved A/B against the in-tree build,
# single-frame latency.
set -o pipefail
O=gpurun_out/s8; mkdir -p $O
NEW=build/libfdf_nmsreg.so
FDF_LIB_PATH=$NEW timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_nmsreg.log 2>&1 || { tail -30 $O/pytest_nmsreg.log; exit 1; }
tail -2 $O/pytest_nmsreg.log
for r in 1 2; do
  bash tools/ab_libs.sh $O/ab_$r.txt maxt:0,sad:0,off:0 feature_detector_fast_amd/libfdf.so $NEW || exit 1
  cat $O/ab_$r.txt
done
for r in 1 2; do for L in feature_detector_fast_amd/libfdf.so $NEW; do
  echo "== $L"; FDF_LIB_PATH=$L timeout -k 10 200 python3 tools/ablate.py --width 3840 --height 2160 --frames 128 --threshold 8 --count 12 --rounds 5 --iters 10 --variants sad:0 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print({k:v['ms_median'] for k,v in d.items()})" || exit 1
done; done > $O/ab4k.txt
cat $O/ab4k.txt
for m in off maxt; do
  FDF_LIB_PATH=$NEW timeout -k 10 120 python3 tools/single_frame.py --nms $m || exit 1
done > $O/single.txt
cat $O/single.txt
echo s8-done

set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_e6
mkdir -p $O
# one device-resident 1080p frame: the 8-slot ring (4 waves per SIMD) against a 16-slot ring
# (12 rows in flight per wave, 2 waves per SIMD), interleaved
for r in 1 2 3; do
  for L in abbase ring16; do
    for nm in maxt off; do
      FDF_LIB_PATH=build/libfdf_$L.so timeout -k 10 60 python3 tools/single_frame.py --nms $nm --iters 300 > $O/sf_${L}_${nm}_r$r.json
    done
  done
done
FDF_LIB_PATH=build/libfdf_ring16.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -q -k "golden or random_sizes" --timeout 200 --timeout-method thread > $O/parity_ring16.txt 2>&1 || true
echo done

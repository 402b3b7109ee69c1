set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_e1
mkdir -p $O
# the deep-ring in-place kernel (product build) through the host tests
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_host_inplace.py tests/test_gpu_stride.py -q --timeout 120 --timeout-method thread > $O/host_tests.txt 2>&1
# the age variants are parity-green: whole-batch config 4 / 5 checks and the compare.rs configurations
for v in age6 age3; do
  FDF_LIB_PATH=build/libfdf_$v.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_stress.py::test_config4_exact_batch tests/test_gpu_geometry.py::test_config5_batch_repeated -q --timeout 200 --timeout-method thread > $O/parity_$v.txt 2>&1
done
# host call: the deep-ring in-place kernel against the device kernel on the same frames (debug build switch)
for r in 1 2 3; do
  for hr in 0 1; do
    FDF_LIB_PATH=build/libfdf_debug.so FDF_HOST_RING=$hr timeout -k 10 120 python3 tools/host_latency.py --iters 200 --mem pinned --chunks 0 > $O/host_ring${hr}_r$r.json
  done
done
# candidate-path variants: interleaved A/B, 1080p (max-t, off, SAD) and 4K t=8 n=12 SAD
timeout -k 10 600 bash tools/ab_interleave.sh $O/ab_age_1080.txt 3 "maxt:0,off:0,sad:0" "" build/libfdf_abbase.so build/libfdf_age6.so build/libfdf_age3.so
timeout -k 10 600 bash tools/ab_interleave.sh $O/ab_age_4k.txt 3 "sad:0" "--width 3840 --height 2160 --frames 128 --threshold 8 --count 12" build/libfdf_abbase.so build/libfdf_age6.so build/libfdf_age3.so
timeout -k 10 600 bash tools/pmc_variants.sh $O/pmc_1080 "" "maxt:0" build/libfdf_abbase.so build/libfdf_age6.so build/libfdf_age3.so
timeout -k 10 600 bash tools/pmc_variants.sh $O/pmc_4k "--width 3840 --height 2160 --frames 128 --threshold 8 --count 12" "sad:0" build/libfdf_abbase.so build/libfdf_age6.so build/libfdf_age3.so
echo done

set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_e2
mkdir -p $O
# the LDS-window variants are parity-green: whole-batch config 4 / 5 checks (n = 9, 12 builds)
for v in lds8 lds16; do
  FDF_LIB_PATH=build/libfdf_$v.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_stress.py::test_config4_exact_batch tests/test_gpu_geometry.py::test_config5_batch_repeated -q --timeout 200 --timeout-method thread > $O/parity_$v.txt 2>&1
done
timeout -k 10 600 bash tools/ab_interleave.sh $O/ab_lds_1080.txt 3 "maxt:0,off:0,sad:0" "" build/libfdf_abbase.so build/libfdf_lds8.so build/libfdf_lds16.so
timeout -k 10 600 bash tools/ab_interleave.sh $O/ab_lds_4k.txt 3 "sad:0" "--width 3840 --height 2160 --frames 128 --threshold 8 --count 12" build/libfdf_abbase.so build/libfdf_lds8.so build/libfdf_lds16.so
timeout -k 10 600 bash tools/pmc_variants.sh $O/pmc_1080 "" "maxt:0" build/libfdf_abbase.so build/libfdf_lds8.so build/libfdf_lds16.so
timeout -k 10 600 bash tools/pmc_variants.sh $O/pmc_4k "--width 3840 --height 2160 --frames 128 --threshold 8 --count 12" "sad:0" build/libfdf_abbase.so build/libfdf_lds8.so build/libfdf_lds16.so
echo done

set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_e11
mkdir -p $O
FDF_LIB_PATH=build/libfdf_rpdpp.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_stress.py::test_config4_exact_batch tests/test_gpu_geometry.py::test_config5_batch_repeated tests/test_gpu_stress.py::test_nms_overflow_tiers -q --timeout 200 --timeout-method thread > $O/parity_rpdpp.txt 2>&1
timeout -k 10 600 bash tools/ab_interleave.sh $O/ab_rp_1080.txt 5 "maxt:0,sad:0,off:0" "" build/libfdf_abhead.so build/libfdf_rpdpp.so
timeout -k 10 600 bash tools/ab_interleave.sh $O/ab_rp_4k.txt 5 "sad:0" "--width 3840 --height 2160 --frames 128 --threshold 8 --count 12" build/libfdf_abhead.so build/libfdf_rpdpp.so
echo done

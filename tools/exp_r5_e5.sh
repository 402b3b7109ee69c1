set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_e5
mkdir -p $O
# the LDS window's occupancy alone: the base kernel with the same 40 KB per workgroup reserved (2 per CU)
timeout -k 10 600 bash tools/ab_interleave.sh $O/ab_pad_1080.txt 3 "maxt:0,off:0,sad:0" "" build/libfdf_abbase.so build/libfdf_pad.so build/libfdf_lds8.so
timeout -k 10 600 bash tools/ab_interleave.sh $O/ab_pad_4k.txt 3 "sad:0" "--width 3840 --height 2160 --frames 128 --threshold 8 --count 12" build/libfdf_abbase.so build/libfdf_pad.so build/libfdf_lds8.so
echo done

cd "$GRAFT_REPO_ROOT"
# ablation switches live in the debug build only (make debug)
export FDF_LIB_PATH=${FDF_LIB_PATH:-$(cd "$(dirname "$0")/.." && pwd)/build/libfdf_debug.so}
for t in 1 2 3 6 12 24; do
  echo "tpg $t 4k $(FDF_COMPACT_TPG=$t timeout -k 10 120 python3 bench.py --width 3840 --height 2160 --frames 128 --threshold 8 --count 12 --nms sad --steps 10 --warmup 3 --cpu-seconds 0 --no-extras 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['roofline']['compaction_kernel_ms_avg'])") 1080off $(FDF_COMPACT_TPG=$t timeout -k 10 120 python3 bench.py --nms off --steps 10 --warmup 3 --cpu-seconds 0 --no-extras 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['roofline']['compaction_kernel_ms_avg'])")"
done > gpurun_out/tpg.txt

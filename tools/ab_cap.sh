cd "$GRAFT_REPO_ROOT"
# ablation switches live in the debug build only (make debug)
export FDF_LIB_PATH=${FDF_LIB_PATH:-$(cd "$(dirname "$0")/.." && pwd)/build/libfdf_debug.so}
V="maxt:0,sad:0"
run() { echo "== $1 $2"; FDF_LIB_PATH=$1 FDF_LDS_BUDGET=$2 timeout -k 10 200 python3 tools/ablate.py --rounds 5 --iters 10 --variants "$V" 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print({k:v['ms_median'] for k,v in d.items()})" || exit 1; }
{ run build/libfdf_base.so 40000 && run build/libfdf_c1536.so 40960 && run build/libfdf_c1280.so 40000 && run build/libfdf_base.so 40000 && run build/libfdf_c1280.so 40000; } > gpurun_out/ab_cap.txt 2>&1

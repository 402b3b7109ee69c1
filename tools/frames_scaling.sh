cd "$GRAFT_REPO_ROOT"
for f in 256 384 448 512 576 640 1024; do
  echo "frames $f $(timeout -k 10 120 python3 tools/ablate.py --frames $f --rounds 3 --iters 10 --variants maxt:0,off:0 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print({k:v['ms_median'] for k,v in d.items()})")"
done > gpurun_out/scale.txt

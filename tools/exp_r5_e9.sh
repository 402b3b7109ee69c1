set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_e9
mkdir -p $O
for r in 1 2; do
  for nm in maxt off; do
    timeout -k 10 60 python3 tools/single_frame.py --nms $nm --iters 300 > $O/sf_${nm}_auto_r$r.json
    timeout -k 10 60 python3 tools/single_frame.py --nms $nm --iters 300 --rows 14 > $O/sf_${nm}_rows14_r$r.json
  done
done

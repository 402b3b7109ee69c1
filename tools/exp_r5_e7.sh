set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_e7
mkdir -p $O
# one device-resident 1080p frame: band height (fdf_ctx_set_band_rows) against the model's pick
for r in 1 2; do
  for nm in maxt off; do
    for rows in 0 4 6 8 10 14 20 28; do
      timeout -k 10 60 python3 tools/single_frame.py --nms $nm --iters 300 --rows $rows > $O/sf_${nm}_rows${rows}_r$r.json
    done
  done
done
echo done

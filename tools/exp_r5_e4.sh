set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_e4
mkdir -p $O
# headline protocol A/B: one shared input copy (rounds 1-4) against one copy per lane, interleaved
for r in 1 2 3; do
  for c in 1 0; do
    timeout -k 10 200 python3 bench.py --no-extras --cpu-seconds 0 --copies $c > $O/copies${c}_r$r.json
  done
done
echo done

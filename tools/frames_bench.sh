cd "$GRAFT_REPO_ROOT"
for f in 64 128 256 512 1024; do
  for m in maxt off; do
    timeout -k 10 200 python3 bench.py --frames $f --nms $m --cpu-seconds 0 --no-extras 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print($f, '$m', d['ms_per_step'], r['kernel_ms_avg'], r['compaction_kernel_ms_avg'])"
  done
done > gpurun_out/frames_bench.txt

cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof4k
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof4k/stats -o p -- python3 bench.py --width 3840 --height 2160 --frames 128 --threshold 8 --count 12 --nms sad --steps 10 --warmup 3 --cpu-seconds 0 --no-extras > gpurun_out/prof4k/bench.json 2> gpurun_out/prof4k/err.log
find gpurun_out/prof4k/stats -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof4k/kernel_stats.csv \;
rm -rf gpurun_out/prof4k/stats

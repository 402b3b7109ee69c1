#!/bin/bash
# Round profile on the GPU box: kernel-trace stats of a bench run plus the two PMC traffic
# passes.  Usage: tools/profile_round.sh TAG [bench args...]   (outputs under gpurun_out/)
# Each rocprofv3 run is its own step with its own time limit; --pmc is never combined with
# tracing.  The program under the profiler is python3 itself.
set -e
TAG=$1; shift
O=gpurun_out/prof_$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ARGS="--cpu-seconds 0 --no-extras $*"   # the bench defaults (50 timed steps after 10 warm-up)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/stats" -o p -- \
    python3 bench.py $ARGS > "$O/bench_under_trace.json" 2> "$O/stats.log"
python3 tools/trace_span.py "$O/stats" --last 50 > "$O/trace_span.json"
# counters per dispatch: one lane, so no other launch runs beside the counted one
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/fetch" -o p -- \
    python3 bench.py --steps 3 --warmup 1 --settle-seconds 0 --cpu-seconds 0 --no-extras --lanes 1 $* > "$O/fetch.json" 2> "$O/fetch.log"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/write" -o p -- \
    python3 bench.py --steps 3 --warmup 1 --settle-seconds 0 --cpu-seconds 0 --no-extras --lanes 1 $* > "$O/write.json" 2> "$O/write.log"
KEY=$(python3 -c "import json,sys; c=json.load(open('$O/fetch.json'))['config']; print(f\"{c['width']}x{c['height']}_b{c['frames_per_gpu']}_t{c['threshold']}_n{c['count']}_{c['nms']}\")")
python3 tools/traffic_json.py "$O/fetch" "$O/write" "$KEY" "$O/pmc_traffic.json"
find "$O/stats" -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats.csv" \;
echo "profile done: $O"

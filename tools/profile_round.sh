#!/bin/bash
# Round profile on the GPU box: kernel-trace stats of a bench run plus the PMC traffic passes.
# Usage: tools/profile_round.sh TAG [bench args...]   (outputs under gpurun_out/prof_TAG)
# Each rocprofv3 run is its own step with its own time limit; --pmc is never combined with
# tracing.  The program under the profiler is python3 itself.  Counter passes run the bench
# protocol twice: on one lane (one input copy) and on the bench's default lanes, each lane
# reading its own copy (rocprofv3 serialises the dispatches it counts: the per-dispatch bytes
# of the headline's own input rotation).
set -e
TAG=$1; shift
O=gpurun_out/prof_$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ARGS="--cpu-seconds 0 --no-extras --no-parity $*"   # the bench defaults (50 timed steps after 10 warm-up)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/stats" -o p -- \
    python3 bench.py $ARGS > "$O/bench_under_trace.json" 2> "$O/stats.log"
python3 tools/trace_span.py "$O/stats" --last 50 > "$O/trace_span.json"
SHORT="--steps 6 --warmup 1 --settle-seconds 0 --cpu-seconds 0 --no-extras --no-parity"
for L in 1 3; do
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/fetch_l$L" -o p -- \
      python3 bench.py $SHORT --lanes $L $* > "$O/fetch_l$L.json" 2> "$O/fetch_l$L.log"
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/write_l$L" -o p -- \
      python3 bench.py $SHORT --lanes $L $* > "$O/write_l$L.json" 2> "$O/write_l$L.log"
done
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$O/tcc_l3" -o p -- \
    python3 bench.py $SHORT --lanes 3 $* > "$O/tcc_l3.json" 2> "$O/tcc_l3.log"
python3 tools/pmc_summary.py "$O/tcc_l3" > "$O/tcc_l3_summary.json"
KEY=$(python3 -c "import json,sys; c=json.load(open('$O/fetch_l1.json'))['config']; print(f\"{c['width']}x{c['height']}_b{c['frames_per_gpu']}_t{c['threshold']}_n{c['count']}_{c['nms']}\")")
python3 tools/traffic_json.py "$O/fetch_l1" "$O/write_l1" "$KEY" "$O/pmc_traffic.json"
python3 tools/traffic_json.py "$O/fetch_l3" "$O/write_l3" "${KEY}_lanes3" "$O/pmc_traffic.json"
find "$O/stats" -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats.csv" \;
# the raw traces and counter rows stay on the box (gpurun copies back <= 64 MiB)
rm -rf "$O/stats" "$O"/fetch_l? "$O"/write_l? "$O/tcc_l3"
echo "profile done: $O"

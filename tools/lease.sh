#!/bin/bash
# One GPU lease, many steps: tools/lease.sh OUT STEP [STEP ...]   (outputs under gpurun_out/OUT)
# Every step runs under its own time limit; the first failing step ends the lease (no retries).
# A STEP is "kind|arg|arg...":
#   tests[|EXPR]                       pytest -m gpu (all GPU tests, or those matching -k EXPR)
#   testslib|LIB|EXPR                  the same on another build of the library (FDF_LIB_PATH)
#   smoke                              __graft_entry__.smoke()
#   bench|NAME|ARGS                    python bench.py ARGS            -> NAME.json
#   ab|NAME|ROUNDS|VARIANTS|ARGS|LIBS  interleaved A/B of library builds (LIBS comma-separated,
#                                      tools/ablate.py variants)       -> NAME.txt
#   ablate|NAME|ARGS                   tools/ablate.py ARGS on the debug build -> NAME.json
#   pmc|NAME|VARIANT|ARGS              SQ / TCC counter passes of one variant (debug build)
#   pmcv|NAME|VARIANTS|ARGS            one instruction-count pass per variant (debug build)
#   pmct|NAME|VARIANTS|ARGS            L2 hit/miss + FETCH_SIZE (+ VALU/VMEM) per variant (debug build)
#   pmcx|NAME|VARIANTS|ARGS|COUNTERS   one pass of the given counters per variant (debug build)
#   stamps|NAME|ARGS                   tools/stamps.py ARGS (debug build) -> NAME.json
#   profile|TAG|ARGS                   tools/profile_round.sh TAG ARGS (kernel stats + traffic)
#   single|NAME                        single-frame latency + kernel traces (off, max-t)
#   py|NAME|SCRIPT ARGS                python3 SCRIPT ARGS             -> NAME.json
#   trace|NAME|SCRIPT ARGS[|LAST]      rocprofv3 kernel trace of a script -> NAME.json (overlap, gaps)
#   htrace|NAME|SCRIPT ARGS            kernel + memory-copy trace of a host-API script -> NAME.json
set -o pipefail
O=gpurun_out/${1:?out}; shift
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
DEBUG_LIB=build/libfdf_debug.so
fail() { echo "step failed: $1"; tail -25 "$2"; exit 1; }
i=0
for STEP in "$@"; do
  i=$((i+1))
  IFS='|' read -r KIND A1 A2 A3 A4 A5 <<< "$STEP"
  L="$O/$(printf %02d $i)_$KIND.log"
  echo "== [$i] $STEP"
  case "$KIND" in
    tests)
      K=()
      [ -n "$A1" ] && K=(-k "$A1")
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${K[@]}" > "$L" 2>&1 || fail "$STEP" "$L"
      tail -2 "$L" ;;
    testslib)
      FDF_LIB_PATH=$A1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$A2" > "$L" 2>&1 || fail "$STEP" "$L"
      tail -2 "$L" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$L" 2>&1 || fail "$STEP" "$L"
      tail -1 "$L" ;;
    bench)
      timeout -k 10 600 python bench.py $A2 > "$O/$A1.json" 2> "$L" || fail "$STEP" "$L"
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel_ms_avg'], r['frac'], d.get('parity'))" "$O/$A1.json" ;;
    ab)
      IFS=',' read -r -a LIBS <<< "$A5"
      timeout -k 10 1000 bash tools/ab_interleave.sh "$O/$A1.txt" "$A2" "$A3" "$A4" "${LIBS[@]}" > "$L" 2>&1 || fail "$STEP" "$L"
      cat "$L" | tail -"${#LIBS[@]}" ;;
    ablate)
      FDF_LIB_PATH=$DEBUG_LIB timeout -k 10 400 python3 tools/ablate.py $A2 > "$O/$A1.json" 2> "$L" || fail "$STEP" "$L"
      python3 -c "import json,sys; print({k: v['ms_median'] for k, v in json.load(open(sys.argv[1])).items()})" "$O/$A1.json" ;;
    pmc)
      D="$O/$A1"; mkdir -p "$D"; j=0
      for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_INSTS_SMEM" \
                 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
                 "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_VMEM SQ_THREAD_CYCLES_VALU" \
                 "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
        j=$((j+1))
        FDF_LIB_PATH=$DEBUG_LIB timeout -s KILL 120 rocprofv3 --pmc $set -d "$D/p$j" -o p --output-format csv -- \
            python3 tools/ablate.py --rounds 1 --iters 2 $A3 --variants "$A2" > "$D/p$j.log" 2>&1 || fail "$STEP pass $j" "$D/p$j.log"
      done
      python3 tools/pmc_summary.py "$D"/p* > "$O/$A1.txt" 2>&1 || fail "$STEP summary" "$O/$A1.txt"
      cat "$O/$A1.txt"
      rm -rf "$D" ;;
    pmcv)
      # one instruction-count pass per variant (comma-separated): where the issue cycles go
      D="$O/$A1"; mkdir -p "$D"; : > "$O/$A1.txt"
      IFS=',' read -r -a VS <<< "$A2"
      for v in "${VS[@]}"; do
        t=$(echo "$v" | tr ':.' '__')
        FDF_LIB_PATH=$DEBUG_LIB timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d "$D/$t" -o p --output-format csv -- \
            python3 tools/ablate.py --rounds 1 --iters 2 $A3 --variants "$v" > "$D/$t.log" 2>&1 || fail "$STEP $v" "$D/$t.log"
        echo "$v $(python3 tools/pmc_summary.py "$D/$t" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(json.dumps({k: round(v) for k, v in d.items() if not k.startswith("_")}))')" >> "$O/$A1.txt"
      done
      cat "$O/$A1.txt"
      rm -rf "$D" ;;
    pmct)
      # memory-side traffic per variant (comma-separated): L2 hits / misses and FETCH_SIZE,
      # each counter set in its own rocprofv3 run
      D="$O/$A1"; mkdir -p "$D"; : > "$O/$A1.txt"
      IFS=',' read -r -a VS <<< "$A2"
      for v in "${VS[@]}"; do
        t=$(echo "$v" | tr ':.' '__')
        k=0
        for set in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE"; do
          k=$((k+1))
          FDF_LIB_PATH=$DEBUG_LIB timeout -s KILL 120 rocprofv3 --pmc $set -d "$D/${t}_$k" -o p --output-format csv -- \
              python3 tools/ablate.py --rounds 1 --iters 2 $A3 --variants "$v" > "$D/${t}_$k.log" 2>&1 || fail "$STEP $v $k" "$D/${t}_$k.log"
        done
        echo "$v $(python3 tools/pmc_summary.py "$D/${t}_1" "$D/${t}_2" "$D/${t}_3" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(json.dumps({k: round(v) for k, v in d.items() if not k.startswith("_")}))')" >> "$O/$A1.txt"
      done
      cat "$O/$A1.txt"
      rm -rf "$D" ;;
    pmcx)
      # one pass of the given counters (A4, space-separated, one block's limits) per variant
      D="$O/$A1"; mkdir -p "$D"; : > "$O/$A1.txt"
      IFS=',' read -r -a VS <<< "$A2"
      for v in "${VS[@]}"; do
        t=$(echo "$v" | tr ':.' '__')
        FDF_LIB_PATH=$DEBUG_LIB timeout -s KILL 120 rocprofv3 --pmc $A4 -d "$D/$t" -o p --output-format csv -- \
            python3 tools/ablate.py --rounds 1 --iters 2 $A3 --variants "$v" > "$D/$t.log" 2>&1 || fail "$STEP $v" "$D/$t.log"
        echo "$v $(python3 tools/pmc_summary.py "$D/$t" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(json.dumps({k: round(v) for k, v in d.items() if not k.startswith("_")}))')" >> "$O/$A1.txt"
      done
      cat "$O/$A1.txt"
      rm -rf "$D" ;;
    stamps)
      FDF_LIB_PATH=$DEBUG_LIB timeout -k 10 400 python3 tools/stamps.py $A2 > "$O/$A1.json" 2> "$L" || fail "$STEP" "$L"
      python3 -c "import json,sys; d=json.load(open(sys.argv[1]))['by_frames']; [print(f, {k: v[k] for k in ('span_us','ramp_us','tail_us_p90_to_last','wg_us_p5_p50_p95','busy_fraction','clock_mhz_p50','event_ms_p50','workgroups','phases_cycles_p50')}) for f, v in d.items()]" "$O/$A1.json" ;;
    profile)
      timeout -k 10 900 bash tools/profile_round.sh "$A1" $A2 > "$L" 2>&1 || fail "$STEP" "$L"
      tail -1 "$L" ;;
    single)
      for m in off maxt; do
        timeout -k 10 120 python3 tools/single_frame.py --nms $m > "$O/${A1}_$m.json" 2> "$L" || fail "$STEP" "$L"
        cat "$O/${A1}_$m.json"
        timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$O/${A1}_trace_$m" -o p -- python3 tools/single_frame.py --nms $m --iters 50 > /dev/null 2>> "$L" || fail "$STEP trace" "$L"
      done ;;
    py)
      timeout -k 10 600 python3 $A2 > "$O/$A1.json" 2> "$L" || fail "$STEP" "$L"
      tail -c 2000 "$O/$A1.json"; echo ;;
    trace)
      # kernel trace of a python script, then the kernels' overlap / gaps (tools/trace_overlap.py)
      timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/$A1" -o p -- python3 $A2 > "$O/$A1.out" 2> "$L" || fail "$STEP" "$L"
      python3 tools/trace_overlap.py "$O/$A1" --last ${A3:-200} > "$O/$A1.json" || fail "$STEP overlap" "$O/$A1.json"
      cat "$O/$A1.json"; rm -rf "$O/$A1" ;;
    htrace)
      # kernel + memory-copy trace of a host-API script, cut into calls (tools/host_timeline.py)
      timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$O/$A1" -o p -- python3 $A2 > "$O/$A1.out" 2> "$L" || fail "$STEP" "$L"
      python3 tools/host_timeline.py "$O/$A1" > "$O/$A1.json" || fail "$STEP timeline" "$O/$A1.json"
      cat "$O/$A1.out" "$O/$A1.json"; rm -rf "$O/$A1" ;;
    *)
      echo "unknown step kind: $KIND"; exit 2 ;;
  esac
done
echo "lease done: $O"

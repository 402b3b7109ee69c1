#!/bin/bash
# Round-5 experiments, one function each (they were 17 one-off scripts): run on the GPU box as
#   bash tools/exp_r5.sh <id>      e.g. bash tools/exp_r5.sh e19
# Each writes under gpurun_out/r5_<id>/; the committed results are in profiles/r05/<id>_*/.
# The variant builds some of them compare (build/libfdf_*.so) come from tools/build_variant.sh
# on the commits the functions name; the variants themselves live on branches.
set -e
cd "$GRAFT_REPO_ROOT"

exp_e1() {
  O=gpurun_out/r5_e1
  mkdir -p $O
  # the deep-ring in-place kernel (product build) through the host tests
  timeout -k 10 300 python3 -u -m pytest tests/test_gpu_host_inplace.py tests/test_gpu_stride.py -q --timeout 120 --timeout-method thread > $O/host_tests.txt 2>&1
  # the age variants are parity-green: whole-batch config 4 / 5 checks and the compare.rs configurations
  for v in age6 age3; do
    FDF_LIB_PATH=build/libfdf_$v.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_stress.py::test_config4_exact_batch tests/test_gpu_geometry.py::test_config5_batch_repeated -q --timeout 200 --timeout-method thread > $O/parity_$v.txt 2>&1
  done
  # host call: the deep-ring in-place kernel against the device kernel on the same frames (debug build switch)
  for r in 1 2 3; do
    for hr in 0 1; do
      FDF_LIB_PATH=build/libfdf_debug.so FDF_HOST_RING=$hr timeout -k 10 120 python3 tools/host_latency.py --iters 200 --mem pinned --chunks 0 > $O/host_ring${hr}_r$r.json
    done
  done
  # candidate-path variants: interleaved A/B, 1080p (max-t, off, SAD) and 4K t=8 n=12 SAD
  timeout -k 10 600 bash tools/ab_interleave.sh $O/ab_age_1080.txt 3 "maxt:0,off:0,sad:0" "" build/libfdf_abbase.so build/libfdf_age6.so build/libfdf_age3.so
  timeout -k 10 600 bash tools/ab_interleave.sh $O/ab_age_4k.txt 3 "sad:0" "--width 3840 --height 2160 --frames 128 --threshold 8 --count 12" build/libfdf_abbase.so build/libfdf_age6.so build/libfdf_age3.so
  timeout -k 10 600 bash tools/pmc_variants.sh $O/pmc_1080 "" "maxt:0" build/libfdf_abbase.so build/libfdf_age6.so build/libfdf_age3.so
  timeout -k 10 600 bash tools/pmc_variants.sh $O/pmc_4k "--width 3840 --height 2160 --frames 128 --threshold 8 --count 12" "sad:0" build/libfdf_abbase.so build/libfdf_age6.so build/libfdf_age3.so
  echo done
}

exp_e2() {
  O=gpurun_out/r5_e2
  mkdir -p $O
  # the LDS-window variants are parity-green: whole-batch config 4 / 5 checks (n = 9, 12 builds)
  for v in lds8 lds16; do
    FDF_LIB_PATH=build/libfdf_$v.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_stress.py::test_config4_exact_batch tests/test_gpu_geometry.py::test_config5_batch_repeated -q --timeout 200 --timeout-method thread > $O/parity_$v.txt 2>&1
  done
  timeout -k 10 600 bash tools/ab_interleave.sh $O/ab_lds_1080.txt 3 "maxt:0,off:0,sad:0" "" build/libfdf_abbase.so build/libfdf_lds8.so build/libfdf_lds16.so
  timeout -k 10 600 bash tools/ab_interleave.sh $O/ab_lds_4k.txt 3 "sad:0" "--width 3840 --height 2160 --frames 128 --threshold 8 --count 12" build/libfdf_abbase.so build/libfdf_lds8.so build/libfdf_lds16.so
  timeout -k 10 600 bash tools/pmc_variants.sh $O/pmc_1080 "" "maxt:0" build/libfdf_abbase.so build/libfdf_lds8.so build/libfdf_lds16.so
  timeout -k 10 600 bash tools/pmc_variants.sh $O/pmc_4k "--width 3840 --height 2160 --frames 128 --threshold 8 --count 12" "sad:0" build/libfdf_abbase.so build/libfdf_lds8.so build/libfdf_lds16.so
  echo done
}

exp_e3() {
  O=gpurun_out/r5_e3
  mkdir -p $O
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  # the in-place host kernel: bytes it fetches per call (FETCH_SIZE x2, gfx950), default geometry
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_inplace -o p --output-format csv -- \
      python3 tools/host_latency.py --iters 20 --mem pinned --chunks 0 --modes maxt > $O/fetch_inplace.log 2>&1
  python3 tools/pmc_summary.py $O/fetch_inplace > $O/fetch_inplace.json
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_copy -o p --output-format csv -- \
      python3 tools/host_latency.py --iters 20 --mem pinned --chunks 1 --modes maxt > $O/fetch_copy.log 2>&1
  python3 tools/pmc_summary.py $O/fetch_copy > $O/fetch_copy.json
  # band height and sub-bands per band of the in-place read (debug build: FDF_NSUB)
  # (this debug build predates the removal of the deep-ring in-place kernel: FDF_HOST_RING=0 keeps
  # the product kernel)
  FDF_LIB_PATH=build/libfdf_debug.so FDF_HOST_RING=0 timeout -k 10 300 python3 tools/host_latency.py --iters 100 --mem pinned --chunks 0 --rows 0,8,14,24,32,46 > $O/rows_nsub_default.json
  FDF_LIB_PATH=build/libfdf_debug.so FDF_HOST_RING=0 FDF_NSUB=1 timeout -k 10 300 python3 tools/host_latency.py --iters 100 --mem pinned --chunks 0 --rows 0,8,14,24,32,46 > $O/rows_nsub1.json
  for m in pinned copy; do
    for nm in maxt off; do
      FDF_HOST_RING=0 timeout -k 10 120 python3 tools/stamps.py --host $m --nms $nm --iters 20 > $O/stamps_host_${m}_$nm.json
    done
  done
  FDF_HOST_RING=1 timeout -k 10 120 python3 tools/stamps.py --host pinned --nms maxt --iters 20 > $O/stamps_host_pinned_maxt_ring16.json
  echo done
}

exp_e4() {
  O=gpurun_out/r5_e4
  mkdir -p $O
  # headline protocol A/B: one shared input copy (rounds 1-4) against one copy per lane, interleaved
  for r in 1 2 3; do
    for c in 1 0; do
      timeout -k 10 200 python3 bench.py --no-extras --cpu-seconds 0 --copies $c > $O/copies${c}_r$r.json
    done
  done
  echo done
}

exp_e5() {
  O=gpurun_out/r5_e5
  mkdir -p $O
  # the LDS window's occupancy alone: the base kernel with the same 40 KB per workgroup reserved (2 per CU)
  timeout -k 10 600 bash tools/ab_interleave.sh $O/ab_pad_1080.txt 3 "maxt:0,off:0,sad:0" "" build/libfdf_abbase.so build/libfdf_pad.so build/libfdf_lds8.so
  timeout -k 10 600 bash tools/ab_interleave.sh $O/ab_pad_4k.txt 3 "sad:0" "--width 3840 --height 2160 --frames 128 --threshold 8 --count 12" build/libfdf_abbase.so build/libfdf_pad.so build/libfdf_lds8.so
  echo done
}

exp_e6() {
  O=gpurun_out/r5_e6
  mkdir -p $O
  # one device-resident 1080p frame: the 8-slot ring (4 waves per SIMD) against a 16-slot ring
  # (12 rows in flight per wave, 2 waves per SIMD), interleaved
  for r in 1 2 3; do
    for L in abbase ring16; do
      for nm in maxt off; do
        FDF_LIB_PATH=build/libfdf_$L.so timeout -k 10 60 python3 tools/single_frame.py --nms $nm --iters 300 > $O/sf_${L}_${nm}_r$r.json
      done
    done
  done
  FDF_LIB_PATH=build/libfdf_ring16.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -q -k "golden or random_sizes" --timeout 200 --timeout-method thread > $O/parity_ring16.txt 2>&1 || true
  echo done
}

exp_e7() {
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
}

exp_e9() {
  O=gpurun_out/r5_e9
  mkdir -p $O
  for r in 1 2; do
    for nm in maxt off; do
      timeout -k 10 60 python3 tools/single_frame.py --nms $nm --iters 300 > $O/sf_${nm}_auto_r$r.json
      timeout -k 10 60 python3 tools/single_frame.py --nms $nm --iters 300 --rows 14 > $O/sf_${nm}_rows14_r$r.json
    done
  done
}

exp_e10() {
  O=gpurun_out/r5_e10
  mkdir -p $O
  # workgroup phase stamps of the final kernels (debug build): 512 x 1080p max-t / off / SAD and 4K SAD
  for nm in maxt off sad; do
    timeout -k 10 200 python3 tools/stamps.py --frames 512 --nms $nm --iters 10 > $O/stamps_512_$nm.json
  done
  timeout -k 10 200 python3 tools/stamps.py --frames 128 --width 3840 --height 2160 --threshold 8 --count 12 --nms sad --iters 6 > $O/stamps_4k_sad.json
  # ablation of the final kernels (debug build flags): stream only, + issue, + evaluation, full, no-sweep
  timeout -k 10 300 python3 tools/ablate.py --rounds 3 --iters 10 --variants "maxt:0,maxt:1,maxt:64,maxt:16,maxt:4,off:0,off:4" > $O/ablate_1080.json
  echo done
}

exp_e11() {
  O=gpurun_out/r5_e11
  mkdir -p $O
  FDF_LIB_PATH=build/libfdf_rpdpp.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_stress.py::test_config4_exact_batch tests/test_gpu_geometry.py::test_config5_batch_repeated tests/test_gpu_stress.py::test_nms_overflow_tiers -q --timeout 200 --timeout-method thread > $O/parity_rpdpp.txt 2>&1
  timeout -k 10 600 bash tools/ab_interleave.sh $O/ab_rp_1080.txt 5 "maxt:0,sad:0,off:0" "" build/libfdf_abhead.so build/libfdf_rpdpp.so
  timeout -k 10 600 bash tools/ab_interleave.sh $O/ab_rp_4k.txt 5 "sad:0" "--width 3840 --height 2160 --frames 128 --threshold 8 --count 12" build/libfdf_abhead.so build/libfdf_rpdpp.so
  echo done
}

exp_e13() {
  # Round 5 e13: host round trip of a tiny launch (blocking vs polled), and the link's read rate
  # for a 1080p frame of pinned host memory read by a kernel, each byte once, by grid size.
  OUT=gpurun_out/r5_e13
  mkdir -p $OUT
  timeout -k 10 120 ./build/sync_latency > $OUT/sync_latency2.txt
}

exp_e14() {
  # Round 5 e14: the in-launch upload (copier workgroups move the pinned frame into HBM, each
  # byte once over the link, the bands wait per chunk): host-path parity, then the end-to-end
  # fdf_detect A/B against reading in place (FDF_UP_COPIERS=0) and 16 / 64 copiers, interleaved.
  # The copier code is on branch exp-inlaunch-upload (not kept: DESIGN.md §7.5); build the
  # variants there with tools/build_variant.sh upN "-DFDF_UP_COPIERS=N".
  OUT=gpurun_out/r5_e14
  mkdir -p $OUT
  timeout -k 10 300 python3 -u -m pytest -q --timeout 120 --timeout-method thread \
    tests/test_gpu_host_inplace.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
  tail -3 $OUT/tests.log
  for r in 1 2 3; do
    for lib in build/libfdf_up0.so feature_detector_fast_amd/libfdf.so build/libfdf_up16.so build/libfdf_up64.so; do
      echo -n "$lib " >> $OUT/host_ab.txt
      FDF_LIB_PATH=$lib timeout -k 10 120 python3 tools/host_latency.py --iters 300 \
        --modes off,maxt --mem pinned --chunks 0 >> $OUT/host_ab.txt
    done
  done
  cat $OUT/host_ab.txt
}

exp_e15() {
  # Round 5 e15: the sweep stops at a unit's last row instead of finishing its 8-step block
  # (FDF_EARLY_EXIT), and a direct launch's ticket round trip runs under the band's LDS setup
  # (FDF_TICKET_OVERLAP): single device frames and the batch configurations, interleaved
  # against the base build of the same tree.
  O=gpurun_out/r5_e15
  mkdir -p $O
  LIBS="${LIBS:-feature_detector_fast_amd/libfdf.so build/libfdf_ee.so build/libfdf_to.so build/libfdf_eeto.so}"; O=${OUT:-$O}; mkdir -p $O
  for r in 1 2 3; do
    for L in $LIBS; do
      for nm in maxt off; do
        echo -n "$(basename $L) " >> $O/single.txt
        FDF_LIB_PATH=$L timeout -k 10 60 python3 tools/single_frame.py --nms $nm --iters 300 >> $O/single.txt
      done
    done
  done
  timeout -k 10 600 bash tools/ab_interleave.sh $O/ab_1080.txt 3 "maxt:0,off:0,sad:0" "--frames 512" $LIBS > $O/ab_1080.log 2>&1
  tail -4 $O/ab_1080.log
  timeout -k 10 600 bash tools/ab_interleave.sh $O/ab_4k.txt 3 "sad:0" "--frames 128 --width 3840 --height 2160 --threshold 8 --count 12" $LIBS > $O/ab_4k.log 2>&1
  tail -4 $O/ab_4k.log
}

exp_e16() {
  # (The latency instances measured here are in commit 3307c16, taken out again: DESIGN.md §7.5.)
  # Round 5 e16: latency instances (fdf_sweep_latency.hip: units leave their last 8-step block
  # at their last row) for grids whose units end inside a block.  The GPU suite on the new
  # library, then single device frames and the batch configurations against the previous build
  # (build/libfdf_base.so), interleaved.
  O=gpurun_out/r5_e16
  mkdir -p $O
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
  LIBS="build/libfdf_base.so feature_detector_fast_amd/libfdf.so"
  for r in 1 2 3; do
    for L in $LIBS; do
      for nm in maxt off; do
        echo -n "$(basename $L) " >> $O/single.txt
        FDF_LIB_PATH=$L timeout -k 10 60 python3 tools/single_frame.py --nms $nm --iters 300 >> $O/single.txt
      done
      echo -n "$(basename $L) " >> $O/host.txt
      FDF_LIB_PATH=$L timeout -k 10 120 python3 tools/host_latency.py --iters 300 --modes off,maxt --mem pinned --chunks 0 >> $O/host.txt
    done
  done
  timeout -k 10 600 bash tools/ab_interleave.sh $O/ab_1080.txt 3 "maxt:0,off:0,sad:0" "--frames 512" $LIBS > $O/ab_1080.log 2>&1
  tail -2 $O/ab_1080.log
  timeout -k 10 600 bash tools/ab_interleave.sh $O/ab_64.txt 3 "maxt:0,off:0" "--frames 64" $LIBS > $O/ab_64.log 2>&1
  tail -2 $O/ab_64.log
}

exp_e17() {
  # Round 5 e17 (variant macro not kept in the source; add "#define FDF_SWEEP_TU_WAVES FDF_LAT_WAVES" to fdf_sweep_latency.hip to rebuild): the latency instances occupancy target (FDF_LAT_WAVES: 4 default, 2, 1 waves
  # per SIMD, i.e. 128 / 256 / 512 VGPRs): single device-resident 1080p frames, interleaved.
  O=gpurun_out/r5_e17
  mkdir -p $O
  for r in 1 2 3; do
    for L in feature_detector_fast_amd/libfdf.so build/libfdf_lat2.so build/libfdf_lat1.so; do
      for nm in maxt off; do
        echo -n "$(basename $L) " >> $O/single.txt
        FDF_LIB_PATH=$L timeout -k 10 60 python3 tools/single_frame.py --nms $nm --iters 300 >> $O/single.txt
      done
    done
  done
}

exp_e18() {
  # Round 5 e18 (variant macro not kept; add "#ifdef FDF_LAT_AGE / #define FDF_MAX_AGE FDF_LAT_AGE" to fdf_sweep_latency.hip
  # to rebuild): the latency instances issue partial batches once a candidate is 1 or 2 rows old.
  O=gpurun_out/r5_e18
  mkdir -p $O
  for r in 1 2 3; do
    for L in feature_detector_fast_amd/libfdf.so build/libfdf_age1.so build/libfdf_age2.so; do
      for nm in maxt off; do
        echo -n "$(basename $L) " >> $O/single.txt
        FDF_LIB_PATH=$L timeout -k 10 60 python3 tools/single_frame.py --nms $nm --iters 300 >> $O/single.txt
      done
    done
  done
}

exp_e19() {
  # (The pinned-output change measured here is in commit 6fd9651, taken out again: DESIGN.md §7.5.)
  # Round 5 e19: points written by the kernels straight into a caller's pinned output buffer
  # (no memcpy from the context's staging after the call): host-path tests, then fdf_detect end
  # to end (pinned frame, pinned output: tools/host_latency.py) against the previous build.
  O=gpurun_out/r5_e19
  mkdir -p $O
  timeout -k 10 400 python3 -u -m pytest -q --timeout 120 --timeout-method thread \
    tests/test_gpu_host_inplace.py tests/test_gpu_api.py tests/test_gpu_parity.py tests/test_gpu_stride.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
  for r in 1 2 3; do
    for L in build/libfdf_base.so feature_detector_fast_amd/libfdf.so; do
      echo -n "$(basename $L) " >> $O/host.txt
      FDF_LIB_PATH=$L timeout -k 10 120 python3 tools/host_latency.py --iters 300 --modes off,maxt --mem pinned,pageable --chunks 0 >> $O/host.txt
    done
  done
}

exp_t25_pmcv() {
  # Round 5 t25: instruction counts per detector launch of the final kernels (VERDICT r04 item 3's
  # measure): SQ_INSTS_VALU / SALU / LDS / VMEM and waves, one lane (serialised dispatches), at
  # 512 x 1080p max-t / off / SAD and 128 x 4K t=8 n=12 SAD.  One --pmc pass per configuration.
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  O=gpurun_out/t25_pmcv
  mkdir -p $O
  SHORT="--steps 6 --warmup 1 --settle-seconds 0 --cpu-seconds 0 --no-extras --no-parity --lanes 1"
  run() {
    local tag=$1; shift
    timeout -k 10 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES \
        --output-format csv -d "$O/$tag" -o p -- python3 bench.py $SHORT "$@" > "$O/$tag.json" 2> "$O/$tag.log"
    python3 tools/pmc_summary.py "$O/$tag" > "$O/${tag}_summary.json"
    rm -rf "$O/$tag"
  }
  run maxt --nms maxt
  run off --nms off
  run sad --nms sad
  run 4k --width 3840 --height 2160 --frames 128 --threshold 8 --count 12 --nms sad
  cat $O/*_summary.json
}

case "${1:-}" in
  e1|e2|e3|e4|e5|e6|e7|e9|e10|e11|e13|e14|e15|e16|e17|e18|e19|t25_pmcv) "exp_$1" ;;
  *) echo "usage: $0 {e1|e2|e3|e4|e5|e6|e7|e9|e10|e11|e13|e14|e15|e16|e17|e18|e19|t25_pmcv}" >&2; exit 2 ;;
esac

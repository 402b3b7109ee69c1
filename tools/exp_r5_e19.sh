#!/bin/bash
# (The pinned-output change measured here is in commit 6fd9651, taken out again: DESIGN.md §7.5.)
# Round 5 e19: points written by the kernels straight into a caller's pinned output buffer
# (no memcpy from the context's staging after the call): host-path tests, then fdf_detect end
# to end (pinned frame, pinned output: tools/host_latency.py) against the previous build.
set -e
cd "$GRAFT_REPO_ROOT"
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

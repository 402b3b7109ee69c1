#!/bin/bash
# A/B: band emit as a wave sweep over 64-word rounds (default) vs per-thread word ranges
# (FDF_EMIT_PER_THREAD) + parity of the default build.
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_emit.log 2>&1 || { echo "pytest failed"; exit 1; }
bash tools/ab_libs.sh gpurun_out/ab_emit.txt "off:0,maxt:0,sad:0" build/libfdf_temit.so build/libfdf_wemit.so build/libfdf_temit.so build/libfdf_wemit.so

#!/bin/bash
# A/B: pre-filter of look-ahead/padding rows masked (default) vs branched around (FDF_LIVE_BRANCH) + parity.
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_live.log 2>&1 || { echo "pytest failed"; exit 1; }
bash tools/ab_libs.sh gpurun_out/ab_live.txt "off:0,maxt:0,sad:0" build/libfdf_live.so build/libfdf_nolive.so build/libfdf_live.so build/libfdf_nolive.so

#!/bin/bash
# A/B of the batch expansion loop (uniform count vs per-iteration ballot) + parity.
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_uni.log 2>&1 || { echo "pytest failed"; exit 1; }
bash tools/ab_libs.sh gpurun_out/ab_expand.txt "off:0,maxt:0,sad:0" build/libfdf_ballot.so build/libfdf_uni.so build/libfdf_ballot.so build/libfdf_uni.so

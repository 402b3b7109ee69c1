set -e
cd "$GRAFT_REPO_ROOT"
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

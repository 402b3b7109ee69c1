set -e
cd "$GRAFT_REPO_ROOT"
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

#!/bin/bash
# Round-2 starting point on the GPU box: short bench lines (max-t, off), the 4K config-5
# kernel stats, a 4K ablation (where the time goes at t=8 n=12) and 4K PMC passes.
set -o pipefail
mkdir -p gpurun_out/r02b
O=gpurun_out/r02b
timeout -k 10 200 python bench.py --nms maxt --cpu-seconds 0 --no-extras > $O/maxt.json 2> $O/maxt.err || exit 1
timeout -k 10 200 python bench.py --nms off --cpu-seconds 0 --no-extras > $O/off.json 2> $O/off.err || exit 1
timeout -k 10 200 python tools/ablate.py --width 3840 --height 2160 --frames 128 --threshold 8 --count 12 \
   --variants sad:0,sad:1,sad:64,sad:16,sad:2,off:0,off:1,off:64,off:8,off:4 > $O/ablate4k.json 2> $O/ablate4k.err || exit 1
bash tools/profile_4k.sh > $O/prof4k.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A="--width 3840 --height 2160 --frames 128 --threshold 8 --count 12 --nms sad --steps 3 --warmup 1 --cpu-seconds 0 --no-extras"
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d $O/pmc4k_sq -o p -- python3 bench.py $A > $O/pmc4k_sq.json 2> $O/pmc4k_sq.log || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc4k_fetch -o p -- python3 bench.py $A > $O/pmc4k_fetch.json 2> $O/pmc4k_fetch.log || exit 1
echo done

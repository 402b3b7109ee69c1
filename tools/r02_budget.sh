#!/bin/bash
# LDS-budget (band height) sweep with the debug build: 4K config 5 and 1080p max-t / off.
set -o pipefail
O=gpurun_out/${1:-budget}
mkdir -p $O
export FDF_LIB_PATH=build/libfdf_debug.so
timeout -k 10 300 python3 tools/ablate.py --rounds 3 --iters 10 --width 3840 --height 2160 --frames 128 --threshold 8 --count 12 \
  --variants sad:0:0,sad:0:30000,sad:0:34000,sad:0:37000,sad:0:44000,sad:0:48000,sad:0:54000 > $O/budget4k.json 2> $O/budget4k.err || exit 1
python3 -c "import json; d=json.load(open('$O/budget4k.json')); print({k:v['ms_median'] for k,v in d.items()})"
timeout -k 10 300 python3 tools/ablate.py --rounds 3 --iters 10 \
  --variants maxt:0:0,maxt:0:36000,maxt:0:44000,maxt:0:48000,off:0:0,off:0:30000,off:0:40000,off:0:44000 > $O/budget1080.json 2> $O/budget1080.err || exit 1
python3 -c "import json; d=json.load(open('$O/budget1080.json')); print({k:v['ms_median'] for k,v in d.items()})"

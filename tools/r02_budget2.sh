#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-budget2}
mkdir -p $O
export FDF_LIB_PATH=build/libfdf_debug.so
timeout -k 10 300 python3 tools/ablate.py --rounds 3 --iters 10 --width 3840 --height 2160 --frames 128 --threshold 8 --count 12 \
  --variants sad:0:0,sad:0:20000,sad:0:24000,sad:0:27000,sad:0:30000,sad:0:40000:2,sad:0:30000:2,off:0:0,off:0:25000,off:0:30000 > $O/b4k.json 2> $O/b4k.err || exit 1
python3 -c "import json; d=json.load(open('$O/b4k.json')); print({k:v['ms_median'] for k,v in d.items()})"
timeout -k 10 300 python3 tools/ablate.py --rounds 3 --iters 10 --width 3840 --height 2160 --frames 128 \
  --variants maxt:0:0,maxt:0:30000,maxt:0:25000,off:0:0,off:0:25000,off:0:30000 > $O/b4k16.json 2> $O/b4k16.err || exit 1
python3 -c "import json; d=json.load(open('$O/b4k16.json')); print({k:v['ms_median'] for k,v in d.items()})"

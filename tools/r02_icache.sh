set -o pipefail
mkdir -p gpurun_out/ic
bash tools/pmc_icache.sh gpurun_out/ic maxt:0 off:0 > gpurun_out/ic/1080p.log 2>&1 || exit 1
ABL_ARGS="--width 3840 --height 2160 --frames 128 --threshold 8 --count 12" bash tools/pmc_icache.sh gpurun_out/ic sad:0 sad:16 > gpurun_out/ic/4k.log 2>&1 || exit 1
echo ok

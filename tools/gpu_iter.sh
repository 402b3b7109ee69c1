set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 ; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
timeout -k 10 200 python3 tools/ablate.py --rounds 5 --iters 10 --variants ${VARIANTS:-maxt:0,maxt:16,maxt:1,off:0,off:1,sad:0} > gpurun_out/abl2.json 2> gpurun_out/abl2.err

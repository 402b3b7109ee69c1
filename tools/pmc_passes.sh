#!/bin/bash
# Counter passes for one ablation variant (one --pmc set per rocprofv3 run; never combined
# with tracing).  Usage: tools/pmc_passes.sh VARIANT OUTDIR   e.g. off:0 gpurun_out/pmc_off
set -e
V=${1:-off:0}
O=${2:-gpurun_out/pmc}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_INSTS_SMEM" \
           "SQ_INST_LEVEL_VMEM SQ_IFETCH SQ_LDS_UNALIGNED_STALL SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_INT SQ_CYCLES" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $set -d "$O/p$i" -o p --output-format csv -- \
      python3 tools/ablate.py --rounds 1 --iters 1 --variants "$V" > "$O/p$i.log" 2>&1
done
python3 tools/pmc_summary.py "$O"/p*

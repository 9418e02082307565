#!/bin/bash
# SQ counter passes for the K3 kernels on the C3 bench (one group per pass).
# Usage: tools/pmc_sq.sh [kernel-regex]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
re=${1:-k_cover|k_insert_work}
i=0
for c in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU_INT64" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
         "SQ_INSTS_VALU_INT32 SQ_LEVEL_WAVES SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_BRANCH SQ_CYCLES SQ_INSTS_SMEM SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $c --kernel-include-regex "$re" -d gpurun_out/sq_$i -o pmc --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/sq_$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done

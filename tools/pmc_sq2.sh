#!/bin/bash
# Two SQ counter passes over the C3 bench for kernels matching a regex.
# Usage: tools/pmc_sq2.sh <regex> <tag>   Output: gpurun_out/sq2_<tag>_<i>/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
re=${1:-k_cover}
tag=${2:-k}
i=0
for c in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" \
         "SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $c --kernel-include-regex "$re" -d gpurun_out/sq2_${tag}_$i -o pmc --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-window > gpurun_out/sq2_${tag}_$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done

#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over the C3 bench for the
# kernels matching a regex.  Usage: tools/pmc_kernels.sh <regex> [tag]
# Output: gpurun_out/pmc_<tag>_<i>/ (csv).  Development tool.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
re=${1:-k_build_range|k_split}
tag=${2:-k}
only=${3:-all}                     # "traffic": the FETCH_SIZE and WRITE_SIZE passes only
i=0
for c in "FETCH_SIZE" "WRITE_SIZE" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  if [ "$only" = traffic ] && [ $i -gt 2 ]; then break; fi
  timeout -s KILL 180 rocprofv3 --pmc $c --kernel-include-regex "$re" -d gpurun_out/pmc_${tag}_$i -o pmc --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-window --no-cli --no-exchange --no-concurrent --no-c5 > gpurun_out/pmc_${tag}_$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done

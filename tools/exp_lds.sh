#!/bin/bash
# Development: LDS counters of k_cover for experiment libraries (tools/exp_build.sh)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for n in "$@"; do
  lib=libpangenome_hip_e$n.so; [ "$n" = 0 ] && lib=libpangenome_hip.so
  PG_LIB_NAME=$lib timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY --kernel-include-regex "${LDS_RE:-k_cover}" -d gpurun_out/lds_$n -o pmc --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-window > gpurun_out/lds_$n.log 2>&1
  rc=$?; echo "exp $n rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done

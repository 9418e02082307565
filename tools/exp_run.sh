#!/bin/bash
# Development: kernel stats of the C3 bench for each experiment library
# (tools/exp_build.sh).  Usage: tools/exp_run.sh <n>...  (0 = product build)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for n in "$@"; do
  lib=libpangenome_hip_e$n.so; [ "$n" = 0 ] && lib=libpangenome_hip.so
  PG_LIB_NAME=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/exp_$n -o run --output-format csv -- python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-c5 --no-host-window > gpurun_out/exp_$n.log 2>&1
  rc=$?; echo "exp $n rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done

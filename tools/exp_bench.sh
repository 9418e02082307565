#!/bin/bash
# Development: bench spans for experiment libraries (tools/exp_build.sh); the
# variants break parity on purpose, so a parity failure (rc 1) is expected.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for n in "$@"; do
  lib=libpangenome_hip_e$n.so; [ "$n" = 0 ] && lib=libpangenome_hip.so
  PG_LIB_NAME=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-window > gpurun_out/expb_$n.log 2>&1
  rc=$?; echo "exp $n rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done

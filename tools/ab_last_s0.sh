#!/bin/bash
# A/B of the last K3 work pass on the coverage stream (PG_K3_LAST_S0) on the C3 bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in 1 0 1 0 1 0; do
  PG_K3_LAST_S0=$v timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/lasts0_$v.log 2>&1
  rc=$?; echo "last_s0=$v rc=$rc $(grep -o '"value": [0-9.]*\|"ms_insert": [0-9.]*' gpurun_out/lasts0_$v.log | tr '\n' ' ')"
  if [ $rc -ne 0 ]; then exit $rc; fi
done

#!/bin/bash
# Sweep the last K3 work pass's blocks per CU (PG_K3_WLAST) on the C3 bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for w in ${WLAST:-0 3 4 6 8}; do
  PG_K3_WLAST=$w timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/wlast_$w.log 2>&1
  rc=$?; echo "wlast=$w rc=$rc $(grep -o '"value": [0-9.]*\|"ms_insert": [0-9.]*' gpurun_out/wlast_$w.log | tr '\n' ' ')"
  if [ $rc -ne 0 ]; then exit $rc; fi
done

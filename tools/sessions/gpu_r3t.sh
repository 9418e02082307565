#!/bin/bash
# round 3: A/B of the working tree's library against the last commit's
# (libpangenome_hip_prev.so), alternating, then the parity suite
set -o pipefail
mkdir -p gpurun_out
for v in _prev "" _prev ""; do
  PG_LIB_NAME=libpangenome_hip$v.so timeout -k 10 200 python -u tools/ab_k3.py --steps 12 --tune base > gpurun_out/abt$v.log 2>&1 || exit $?
  echo "lib$v: $(grep step gpurun_out/abt$v.log)"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q --timeout 120 --timeout-method thread > gpurun_out/parityt.log 2>&1; rc=$?; tail -3 gpurun_out/parityt.log; exit $rc

#!/bin/bash
# round 3: k_cover_q hint-first check and 8 waves/SIMD (product) vs without
# either (e4194304: no launch bound, e8388608: no hint check, e12582912:
# neither), then the parity suite of the product
set -o pipefail
mkdir -p gpurun_out
for v in "" _e4194304 _e8388608 _e12582912 ""; do
  PG_LIB_NAME=libpangenome_hip$v.so timeout -k 10 200 python -u tools/ab_k3.py --steps 12 --tune base > gpurun_out/ab9$v.log 2>&1 || exit $?
  echo "lib$v: $(grep step gpurun_out/ab9$v.log)"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q --timeout 120 --timeout-method thread > gpurun_out/parity9.log 2>&1; rc=$?; tail -3 gpurun_out/parity9.log; exit $rc

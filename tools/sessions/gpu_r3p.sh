#!/bin/bash
# round 3: coverage groups of 8 members (product) vs 4 (e65536), parity of the product
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_k3.py --steps 12 --tune base --tune K3_COVER=1 > gpurun_out/ab7_qm8.log 2>&1 || exit $?
PG_LIB_NAME=libpangenome_hip_e65536.so timeout -k 10 300 python -u tools/ab_k3.py --steps 12 --tune base > gpurun_out/ab7_qm4.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_k3.py --steps 12 --tune base > gpurun_out/ab7_qm8b.log 2>&1 || exit $?
grep step gpurun_out/ab7_*.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q --timeout 120 --timeout-method thread > gpurun_out/parity7.log 2>&1; rc=$?; tail -3 gpurun_out/parity7.log; exit $rc

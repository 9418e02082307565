#!/bin/bash
# round 3: work pass in two halves (default) vs at once, and parity
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_k3.py --steps 12 --tune base --tune K3_EMIT=1 --tune K3_WBLK=6 --tune K3_WBLK=8 > gpurun_out/ab8.log 2>&1 || exit $?
grep step gpurun_out/ab8.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q --timeout 120 --timeout-method thread > gpurun_out/parity8.log 2>&1; rc=$?; tail -3 gpurun_out/parity8.log; exit $rc

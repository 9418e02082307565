#!/bin/bash
# round 3: C5 form on one GPU (tests/test_gpu_c5.py), then the 3.75 Gbp shard
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_c5.py -m gpu -x -v -s --timeout 900 --timeout-method thread > gpurun_out/l_c5s.log 2>&1 || { tail -40 gpurun_out/l_c5s.log; exit 1; }
tail -5 gpurun_out/l_c5s.log
if [ "${1:-}" = full ]; then
  PG_RUN_C5_FULL=1 timeout -k 10 1100 python -u -m pytest tests/test_gpu_c5.py -m gpu -x -v -s -k full_size --timeout 1100 --timeout-method thread > gpurun_out/l_c5full.log 2>&1 || { tail -40 gpurun_out/l_c5full.log; exit 1; }
  grep -E "c5 shard|passed|failed" gpurun_out/l_c5full.log
fi

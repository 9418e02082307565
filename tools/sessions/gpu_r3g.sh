#!/bin/bash
# round 3: copy-stream / tail-split variants of the host window (experiment builds)
set -o pipefail
mkdir -p gpurun_out
for v in "" _e1048576 _e2097152 _e3145728 ""; do
  echo "variant [$v]"
  PG_LIB_NAME=libpangenome_hip$v.so timeout -k 10 200 python -u tools/stage_sweep.py 32,4,8,1 32,4,8,1 2>&1 | grep "^{"
done

#!/bin/bash
# round 3: stage C over 2048-bucket partitions at 3 blocks per CU with an
# 8-bit split (e33554432) vs 4096 at 2 (product), alternating
set -o pipefail
mkdir -p gpurun_out
for v in "" _e33554432 "" _e33554432; do
  PG_LIB_NAME=libpangenome_hip$v.so timeout -k 10 200 python -u tools/ab_k3.py --steps 16 --tune base > gpurun_out/abw$v.log 2>&1 || exit $?
  echo "lib$v: $(grep step gpurun_out/abw$v.log)"
done

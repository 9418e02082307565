#!/bin/bash
# round 3: k_cover_p phase stamps (experiment build e65536)
set -o pipefail
mkdir -p gpurun_out
PG_LIB_NAME=libpangenome_hip_e65536.so timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-host-window > gpurun_out/j_bench.log 2>&1 || { tail -20 gpurun_out/j_bench.log; exit 1; }
grep cov_stamp gpurun_out/j_bench.log | tail -4

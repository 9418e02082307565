#!/bin/bash
# round 3: where k_cover's time goes (experiment builds: 32 = no drift search,
# 64 = no segment compare, 96 = neither); kernel stats per variant
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "" _e32 _e64 _e96; do
  PG_LIB_NAME=libpangenome_hip$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/kc$v" -o kc --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-window > gpurun_out/kc$v.log 2>&1 || { tail -5 gpurun_out/kc$v.log; exit 1; }
  echo "variant [$v]"
  grep -h "k_cover\|k_emit_work" gpurun_out/kc$v/*kernel_stats.csv | cut -c1-160
done

#!/bin/bash
# round 3: stage A decomposition - kernel stats of tools/ab_k3.py for the
# product and the timing-experiment builds (e131072: no record stores,
# e262144: no emission, e524288: no work pass, e1048576: no drift search)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "" _e131072 _e262144 _e524288 _e1048576; do
  PG_LIB_NAME=libpangenome_hip$v.so timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/dec$v -o run --output-format csv -- python tools/ab_k3.py --steps 4 --tune base > gpurun_out/dec$v.log 2>&1 || exit $?
  grep step gpurun_out/dec$v.log
done

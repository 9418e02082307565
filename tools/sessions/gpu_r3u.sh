#!/bin/bash
# round 3: work-pass forms beside the new coverage pass (A/B), then the
# 3.75 Gbp C5 shard property run (tools/c5_full.py)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab_k3.py --steps 12 --tune base --tune K3_EMIT=1 --tune K3_EMIT=1,K3_WBLK=3 --tune K3_WBLK=3 --tune base > gpurun_out/abu.log 2>&1 || exit $?
grep step gpurun_out/abu.log
timeout -k 10 1000 python -u tools/c5_full.py > gpurun_out/c5_full.log 2>&1; rc=$?; tail -8 gpurun_out/c5_full.log; exit $rc

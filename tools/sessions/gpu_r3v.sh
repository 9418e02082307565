#!/bin/bash
# round 3: last-chunk size and work-pass grid beside the current coverage pass (A/B)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_k3.py --steps 20 --tune base --tune K3_WBLK=84 --tune K3_TAIL=8 --tune K3_TAIL=12 --tune K3_WBLK=84,K3_TAIL=8 --tune K3_WBLK=3 > gpurun_out/abx.log 2>&1; rc=$?; grep step gpurun_out/abx.log; exit $rc

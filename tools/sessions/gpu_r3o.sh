#!/bin/bash
# round 3: K3 chunk count x work-pass grid A/B (tools/ab_k3.py)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/ab_k3.py --steps 12 --tune base --tune K3_WBLK=68 --tune K3_WBLK=68,K3_CHUNKS=4 --tune K3_WBLK=68,K3_CHUNKS=5 --tune K3_WBLK=66,K3_CHUNKS=4 --tune K3_WBLK=4 --tune K3_WBLK=4,K3_CHUNKS=4 > gpurun_out/ab6.log 2>&1; rc=$?; grep step gpurun_out/ab6.log; exit $rc

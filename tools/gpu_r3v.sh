#!/bin/bash
# round 3: size of the last stage A chunk (A/B)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_k3.py --steps 24 --tune base --tune K3_TAIL=10 --tune K3_TAIL=12 --tune K3_TAIL=8 --tune K3_TAIL=14 > gpurun_out/abv.log 2>&1; rc=$?; grep step gpurun_out/abv.log; exit $rc

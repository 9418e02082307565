#!/bin/bash
# round 3: RCCL all_to_all sizes at world 1
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/rccl_a2a_check.py 2>&1 | tee gpurun_out/n_rccl.log | grep -E "rows|Error|error"

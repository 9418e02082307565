#!/bin/bash
# SQ instruction counters of k_cover under PG_K3_DBG knob variants (one
# k3_probe run; the dispatches appear in variant order after the real build).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
v=${1:-tile:128,tile:1152,tile:1664,tile:16512,tile:17536,tile:18048}
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM --kernel-include-regex k_cover -d gpurun_out/k3pmc -o pmc --output-format csv -- python tools/k3_probe.py --reps 1 --variants $v > gpurun_out/k3pmc.log 2>&1
echo "rc=$?"

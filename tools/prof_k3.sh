#!/bin/bash
# Development: kernel trace + SQ counter passes of tools/ab_k3.py (variants as
# its --tune arguments) for the kernels matching a regex.
# Usage: tools/prof_k3.sh <tag> <regex> [ab_k3 args...]   Output: gpurun_out/pk3_<tag>_*/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; re=$2; shift 2
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/pk3_${tag}_trace -o run --output-format csv -- python tools/ab_k3.py --steps 4 "$@" > gpurun_out/pk3_${tag}_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
i=0
for c in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" \
         "SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $c --kernel-include-regex "$re" -d gpurun_out/pk3_${tag}_$i -o pmc --output-format csv -- python tools/ab_k3.py --steps 2 "$@" > gpurun_out/pk3_${tag}_$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done

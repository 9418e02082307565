#!/bin/bash
# Development: L2 / EA counters of the K3 probe variants (one rocprofv3 pass per counter set).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=${1:-tile:0,tile:2,tile:24}
for ctr in "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "TCC_EA0_ATOMIC_sum TCC_EA0_WRREQ_64B_sum"; do
  tag=$(echo $ctr | tr ' ' '_')
  timeout -k 10 600 rocprofv3 --pmc $ctr --kernel-include-regex "k_insert" -d gpurun_out/pmck3_$tag -o pmc \
    --output-format csv -- python3 tools/k3_probe.py --reps 1 --variants "$V" > gpurun_out/pmck3_$tag.log 2>&1
  rc=$?
  echo "== $tag rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done

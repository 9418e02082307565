#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration passes over tools/bin/fetch_calib (one counter group per pass).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 60 ./tools/bin/fetch_calib > gpurun_out/calib_plain.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" TCC_EA0_ATOMIC_sum "TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_64B_sum"; do
  t=$(echo $c | tr ' ' '_')
  timeout -s KILL 60 rocprofv3 --pmc $c -d gpurun_out/calib_$t -o pmc --output-format csv -- ./tools/bin/fetch_calib > gpurun_out/calib_$t.log 2>&1
  rc=$?; echo "$c rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done

#!/bin/bash
# PMC passes for the dominant kernel (K3 k_insert) on the C3 bench, one counter
# group per pass (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE cannot share a pass).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" TCC_EA0_ATOMIC_sum "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVES" "TA_BUSY_avr TA_TA_BUSY_sum" GRBM_GUI_ACTIVE; do
  t=$(echo $c | tr ' ' '_')
  timeout -k 10 400 rocprofv3 --pmc $c --kernel-include-regex "k_cover|k_insert|k_zero16|k_reduce|k_emit|k_span_sum" -d gpurun_out/pmc3_$t -o pmc --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc3_$t.log 2>&1
  rc=$?; echo "$c rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done

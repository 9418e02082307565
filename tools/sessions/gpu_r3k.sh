#!/bin/bash
# round 3: A/B of coverage-pass variants (HBM-resident step; PG_K3_COVER=1: k_cover, 0: k_cover_p)
set -o pipefail
mkdir -p gpurun_out
run() {  # tag lib form
  PG_LIB_NAME=$2 PG_K3_COVER=$3 timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host-window > gpurun_out/k_$1.log 2>&1 || { tail -20 gpurun_out/k_$1.log; exit 1; }
  python3 - $1 <<'PY'
import json,sys
d=[json.loads(l) for l in open("gpurun_out/k_%s.log"%sys.argv[1]) if l.startswith("{")][0]
k=d["kernels"]; p=d["path"]
print("%-10s dev_ms %s k3a %s recA %s parity %s"%(sys.argv[1],p.get("device_resident_ms",d["ms_per_step"]),k["k3a_cover_emit"]["ms"],p["n_records_a"],d["parity"]["ok"]))
PY
  grep cov_stamp gpurun_out/k_$1.log | tail -1 || true
}
for rep in 1 2; do
  run old_uncond libpangenome_hip.so 1 || exit 1
  run old_cond libpangenome_hip_e131072.so 1 || exit 1
  run pers_stamp libpangenome_hip_e65536.so 0 || exit 1
done

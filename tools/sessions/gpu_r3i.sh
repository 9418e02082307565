#!/bin/bash
# round 3: persistent coverage pass (k_cover_p) parity + A/B against k_cover
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -x -q --timeout 300 --timeout-method thread -k "k3 or c3_default or alternating or full_size or device_resident" > gpurun_out/i_tests.log 2>&1 || { tail -30 gpurun_out/i_tests.log; exit 1; }
tail -3 gpurun_out/i_tests.log
for form in 0 1 0 1; do
  PG_K3_COVER=$form timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/i_bench$form.log 2>&1 || { tail -20 gpurun_out/i_bench$form.log; exit 1; }
  python3 - $form <<'PY'
import json,sys
d=[json.loads(l) for l in open("gpurun_out/i_bench%s.log"%sys.argv[1]) if l.startswith("{")][0]
k=d["kernels"]; p=d["path"]
print("form",sys.argv[1],"value",d["value"],"dev_ms",p["device_resident_ms"],"k1",k["k1_parse"]["ms"],"k3a",k["k3a_cover_emit"]["ms"],"k3b",k["k3b_split"]["ms"],"k3c",k["k3c_range"]["ms"],"recA",p["n_records_a"],"parity",d["parity"]["ok"])
PY
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/i_prof" -o kc --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-window > gpurun_out/i_prof.log 2>&1 || { tail -5 gpurun_out/i_prof.log; exit 1; }
echo done

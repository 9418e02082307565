#!/bin/bash
# Development: the packed coverage pass's anchor count / search window
# variants (tools/exp_lib.sh builds), one bench line each, parity checked.
set -o pipefail
o=gpurun_out/nap2; mkdir -p $o
for L in "$@"; do
  PG_LIB_NAME=libpangenome_hip$L.so timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-concurrent > $o/bench$L.json 2> $o/bench$L.err || exit 3
  python - "$o/bench$L.json" "$L" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels"]
print(sys.argv[2] or "default", d["ms_per_step"], d["path"]["n_records_a"], " ".join("%s=%.4f" % (n, v["ms"]) for n, v in k.items()), d["parity"]["ok"])
PY
done

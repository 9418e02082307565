#!/bin/bash
# Development: kernel stats of tools/ab_k3.py per experiment library
# (tools/exp_lib.sh), e.g. the packed coverage pass's anchor variants.
# Usage: tools/nap_prof.sh <suffix>...   ("" = the product library)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/napp; mkdir -p $o
for L in "$@"; do
  n=${L:-_default}
  PG_LIB_NAME=libpangenome_hip$L.so timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $o/t$n -o run --output-format csv -- python tools/ab_k3.py --steps 8 > $o/ab$n.log 2>&1 || exit 3
  s=$(ls $o/t$n/run_kernel_stats.csv $o/t$n/*/run_kernel_stats.csv 2>/dev/null | head -1)
  echo "== $n"; grep -E "^(variant|base)|records|step" $o/ab$n.log | tail -3
  python - "$s" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if any(x in r["Name"] for x in ("k_cover_p", "k_emit_work", "k_short_emit", "k_split", "k_build_range")):
        print("  %-40s calls %6s avg_us %8.1f total_ms %8.2f" % (r["Name"][:40], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6))
PY
done

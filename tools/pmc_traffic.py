#!/usr/bin/env python3
"""profiles/traffic_<config>.json from the FETCH_SIZE / WRITE_SIZE passes of
tools/pmc_kernels.sh (gpurun_out/pmc_<tag>_1, _2): HBM bytes per build and
per bench.py span.  Development tool; bench.py only reads the JSON.

FETCH_SIZE and WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE counts a
coalesced 16/8/4-byte-per-lane stream at half its bytes (128-B requests
tallied at 64 B, MI355X_MICROARCH.md §HBM; profiles/fetch_calib.json), so it
is doubled for every kernel except k_emit_work, whose reads are per-lane
16-B loads of scattered segments (a random 16-B load is one 64-B request,
counted exactly).  WRITE_SIZE reads streaming stores exactly.  Per kernel the
mean over its dispatches of the last three builds (the HBM-resident ones:
the cold first build runs the chunked host window) times its dispatches per
build (3 chunks for the coverage / emission passes)."""
import collections
import csv
import glob
import json
import re
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "tr"
config = sys.argv[2] if len(sys.argv) > 2 else "c3"
SPANS = {
    "k1_parse": r"k_span_sum|k_span_whole|k_span_fix|lookback_scan|scan_impl|k_emit\b|k_emit\(|k_emit<|k_headers|"
                r"k_records|k_pack_records|k_pack_fix",
    "k3a_cover_emit": r"k_cover|k_emit_work|k_short_emit",
    "k3b_split": r"k_split",
    "k3c_range": r"k_build_range",
}
PER_BUILD = {"k_cover": 3, "k_emit_work": 3}


def load(i):
    vals = collections.defaultdict(list)
    for f in glob.glob("gpurun_out/pmc_%s_%d/**/*counter_collection.csv" % (tag, i), recursive=True):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            per[(int(r["Dispatch_Id"]), r["Kernel_Name"])] += float(r["Counter_Value"])
        for (d, k), v in sorted(per.items()):
            vals[k].append(v * 1024.0)
    return vals


def last_builds(v, per_build, builds=3):
    """The kernel's dispatches of the last `builds` builds: the bench's
    HBM-resident builds (its cold first build goes through the chunked host
    window, whose K1 / stage A dispatches are smaller)."""
    return v[-builds * per_build:] or v


fetch, write = load(1), load(2)
per_kernel = {}
for k in set(fetch) | set(write):
    short = re.sub(r"\(.*", "", k).replace("void ", "")
    mult = next((m for n, m in PER_BUILD.items() if n in short), 1)

    def mean(v):
        v = last_builds(v, mult)
        return sum(v) / len(v) if v else 0.0
    f = mean(fetch.get(k, [])) * (1 if "k_emit_work" in short else 2)
    w = mean(write.get(k, []))
    e = per_kernel.setdefault(short, {"fetch_bytes": 0.0, "write_bytes": 0.0, "dispatches_per_build": mult})
    e["fetch_bytes"] += f * mult
    e["write_bytes"] += w * mult
spans = {}
for name, rx in SPANS.items():
    spans[name] = int(sum(v["fetch_bytes"] + v["write_bytes"] for k, v in per_kernel.items() if re.search(rx, k)))
out = {"source": "tools/pmc_kernels.sh (rocprofv3 --pmc FETCH_SIZE, then WRITE_SIZE, separate passes) on "
                 "python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-window; folded by tools/pmc_traffic.py",
       "hbm_bytes_per_build": spans,
       "per_kernel": {k: {kk: (int(vv) if kk != "dispatches_per_build" else vv) for kk, vv in v.items()}
                      for k, v in sorted(per_kernel.items())}}
json.dump(out, open("gpurun_out/traffic_%s.json" % config, "w"), indent=1)      # (copied into profiles/ by hand)
print(json.dumps(spans, indent=1))

#!/usr/bin/env python3
"""Development: per-kernel sums of the SQ passes of tools/prof_k3.sh
(gpurun_out/pk3_<tag>_<i>/) and the stage A/B/C timeline of its trace."""
import collections
import csv
import glob
import sys

tag = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in sorted(glob.glob("gpurun_out/pk3_%s_[0-9]/pmc_counter_collection.csv" % tag)):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("pg::", "")
        agg[n][r["Counter_Name"]] += float(r["Counter_Value"])
for n, d in agg.items():
    w = d["SQ_WAVES"]
    print(n, "waves", w)
    for c in sorted(d):
        print("   %-24s %14.0f  per wave %10.1f" % (c, d[c], d[c] / w if w else 0))


def short(n):
    n = n.replace("pg::", "")
    return n.split("(")[0].replace("void ", "")


rows = list(csv.DictReader(open("gpurun_out/pk3_%s_trace/run_kernel_trace.csv" % tag)))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r["Queue_Id"]) for r in rows)
idx = [i for i, e in enumerate(ev) if e[2] == "k_span_sum"]
for a, b in zip(idx[-3:-1], idx[-2:]):
    t0 = ev[a][0]
    print("----")
    for s, e, n, q in ev[a:b]:
        if n.startswith(("k_cover", "k_emit_work", "k_split", "k_build_range", "k_short")):
            print("%9.1f %9.1f %8.1f q%s %s" % ((s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3, q, n))

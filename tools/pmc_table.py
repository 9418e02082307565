#!/usr/bin/env python3
"""Per-kernel averages of the PMC passes of tools/pmc_kernels.sh
(gpurun_out/pmc_<tag>_*/): one line per kernel and counter, the mean over
its dispatches after the first bench step's.  Development tool."""
import collections
import csv
import glob
import re
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "k"
acc = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/pmc_%s_*/**/*counter_collection.csv" % tag, recursive=True)):
    rows = list(csv.DictReader(open(f)))
    per = collections.defaultdict(float)
    for r in rows:
        per[(r["Dispatch_Id"], re.sub(r"\(.*", "", r["Kernel_Name"]), r["Counter_Name"])] += float(r["Counter_Value"])
    for (d, k, c), v in per.items():
        acc[(k, c)].append((int(d), v))
for (k, c), vs in sorted(acc.items()):
    vs.sort()
    tail = vs[len(vs) // 3:] or vs
    print("%-28s %-24s n=%3d  mean %.4g" % (k[-28:], c, len(vs), sum(v for _, v in tail) / len(tail)))

#!/usr/bin/env python3
"""Print rocprofv3 kernel stats and the last bench step's dispatch timeline
(gpurun_out/prof/).  Development tool."""
import csv
import re
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
for r in csv.DictReader(open(d + "/run_kernel_stats.csv")):
    n = re.sub(r"\(.*", "", r["Name"])[-50:]
    print("%-50s %4s avg %9.1f us  min %9.1f" % (n, r["Calls"], float(r["AverageNs"]) / 1e3, float(r["MinNs"]) / 1e3))
t = list(csv.DictReader(open(d + "/run_kernel_trace.csv")))
starts = [i for i, r in enumerate(t) if "k_span_sum" in r["Kernel_Name"]]
t0 = int(t[starts[-1]]["Start_Timestamp"])
for r in t[starts[-1]:]:
    n = re.sub(r"\(.*", "", r["Kernel_Name"])[-40:]
    s = int(r["Start_Timestamp"])
    print("%-42s %8.1f at %8.1f" % (n, (int(r["End_Timestamp"]) - s) / 1e3, (s - t0) / 1e3))

#!/usr/bin/env python3
"""The last pg_build_host window of a rocprofv3 --kernel-trace
--memory-copy-trace run (gpurun_out/<dir>/): every copy and kernel from the
window's first H2D chunk on, relative to it, and the tail - what runs after
the last H2D chunk has landed.  Development tool.

    rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/tw -o run \\
        --output-format csv -- python tools/ab_k3.py --host --steps 3
    python tools/trace_window.py gpurun_out/tw"""
import csv
import glob
import re
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/tw"
kt = list(csv.DictReader(open(glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0])))
mf = glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True)
mt = list(csv.DictReader(open(mf[0]))) if mf else []
ev = []
for r in kt:
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K", re.sub(r"\(.*", "", r["Kernel_Name"])[-44:],
               r.get("Queue_Id", "")))
for r in mt:
    kind = (r.get("Direction") or r.get("Operation") or "COPY").replace("MEMORY_COPY_", "")
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C", kind, ""))
ev.sort()
# the chunk uploads: H2D copies of more than 200 us (no byte counts in the
# trace; a 64 MiB chunk takes ~1.2 ms, record tables and flags a few us)
h2d = [e for e in ev if e[2] == "C" and "HOST_TO_DEVICE" in e[3] and e[1] - e[0] > 200_000]
if not h2d:
    sys.exit("no H2D chunk copies in the trace (run with --memory-copy-trace)")
# windows start where consecutive big copies are separated by > 1 ms
starts = [h2d[0][0]] + [b[0] for a, b in zip(h2d, h2d[1:]) if b[0] - a[1] > 1_000_000]
t0 = starts[-1]
win = [e for e in ev if e[0] >= t0]
last_copy_end = max(e[1] for e in h2d if e[0] >= t0)
end = max(e[1] for e in win if e[2] == "K" and e[0] < last_copy_end + 5_000_000)
print("window: first chunk at 0, last chunk landed at %.1f us, last kernel ends at %.1f us (tail %.1f us)"
      % ((last_copy_end - t0) / 1e3, (end - t0) / 1e3, (end - last_copy_end) / 1e3))
for s, e, kind, name, q in win:
    if s > end:
        break
    mark = " *" if s >= last_copy_end else ""
    print("%9.1f %9.1f %8.1f %s q%-3s %s%s" % ((s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3, kind, q, name, mark))

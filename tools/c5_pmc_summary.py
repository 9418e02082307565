#!/usr/bin/env python3
"""profiles/r06_c5_pmc.json from the C5 PMC passes (tools/gpu_session.sh
c5pmc: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / two SQ groups, each its own
run of tools/c5_probe.py stream routed) and the kernel trace of
tools/gpu_session.sh c5probeprof.  Per kernel: dispatches, total time, HBM
bytes (FETCH_SIZE x2 for coalesced streams as MI355X_MICROARCH.md's HBM
section prescribes - k_emit_work's scattered 16-B loads are counted at 1x -
plus WRITE_SIZE, both KiB), their rate over the kernel's time, and the SQ
ratios (LDS bank-conflict cycles / LDS cycles, waiting / wave cycles).
Development tool."""
import collections
import csv
import json
import re
import sys

OUT = sys.argv[1] if len(sys.argv) > 1 else "profiles/r06_c5_pmc.json"


def short(name):
    return re.sub(r"\(.*", "", name).replace("void ", "")


def counters(i):
    d = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open("gpurun_out/c5pmc_%d/pmc_counter_collection.csv" % i)):
        d[short(r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
    return d


def main():
    c = [None] + [counters(i) for i in (1, 2, 3, 4)]
    ks = collections.defaultdict(lambda: [0, 0.0])
    for r in csv.DictReader(open("gpurun_out/prof_c5r/run_kernel_trace.csv")):
        k = short(r["Kernel_Name"])
        ks[k][0] += 1
        ks[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    out = {}
    for k in sorted(c[1]):
        fetch = c[1][k]["FETCH_SIZE"] * 1024 * (1 if "k_emit_work" in k else 2)
        write = c[2][k]["WRITE_SIZE"] * 1024
        ms = ks[k][1]
        sq3, sq4 = c[3][k], c[4][k]
        out[k] = {
            "dispatches": ks[k][0], "ms": round(ms, 3), "hbm_bytes": int(fetch + write),
            "fetch_bytes": int(fetch), "write_bytes": int(write),
            "hbm_tb_per_s": round((fetch + write) / (ms * 1e-3) / 1e12, 3) if ms else None,
            "lds_bank_conflict_frac": round(sq4["SQ_LDS_BANK_CONFLICT"] / sq4["SQ_LDS_IDX_ACTIVE"], 3)
            if sq4.get("SQ_LDS_IDX_ACTIVE") else None,
            "wait_frac": round(sq4["SQ_WAIT_ANY"] / sq3["SQ_WAVE_CYCLES"], 3) if sq3.get("SQ_WAVE_CYCLES") else None,
            "valu_insts": int(sq3.get("SQ_INSTS_VALU", 0)), "salu_insts": int(sq3.get("SQ_INSTS_SALU", 0)),
            "lds_insts": int(sq3.get("SQ_INSTS_LDS", 0)),
        }
    doc = {"source": "tools/gpu_session.sh c5pmc (4 separate rocprofv3 --pmc runs) + c5probeprof (kernel trace) of "
                     "tools/c5_probe.py stream routed: one routed streamed build of the 3.75 Gbp C5 rank-0 shard "
                     "(2^30-base chunks: 4 rounds of stage A + route scatter, then 4 sub-log merges of ~0.94e9 "
                     "records each: re-binning k_route_emit, 2 k_split passes, k_build_range); the session's first "
                     "build, so k_emit_work's time includes its first touch of fresh stage A buffers",
           "kernels": out}
    json.dump(doc, open(OUT, "w"), indent=1)
    for k, v in out.items():
        print("%-28s %3d  %8.2f ms  %7.1f GB  %6s TB/s  lds-conflict %s  wait %s" %
              (k[:28], v["dispatches"], v["ms"], v["hbm_bytes"] / 1e9, v["hbm_tb_per_s"], v["lds_bank_conflict_frac"],
               v["wait_frac"]))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Fold the rocprofv3 PMC passes of tools/pmc_insert.sh (gpurun_out/pmc3_*/)
and the calibration passes of tools/calib.sh (gpurun_out/calib_*/) into
profiles/traffic_<config>.json, the file bench.py reads `roofline.traffic`
from.  Development tool; not part of the product.

Per kernel and counter, values are summed over the dispatches of one bench
step (K3 runs in chunks) and averaged over the steps after the first (the
warm-up build runs on a larger first-guess table).

HBM bytes per K3 launch (coverage pass + work pass), from the calibration
(tools/fetch_calib.hip, profiles/fetch_calib.json):
  * FETCH_SIZE counts 64 B per memory read request.  A random 16-B or 8-B
    load is one 64-B request (counted exactly); a coalesced 16 B/lane stream
    issues 128-B requests, counted at half (MI355X_MICROARCH.md).  The
    coverage passes (k_cover) stream the class codes and their reference
    spans and never touch the table, so their FETCH_SIZE is doubled; the work
    passes are dominated by random bucket loads, so their FETCH_SIZE is taken
    as is (their segment reads are then under-counted by half - a lower
    bound).  The table clear (k_zero16) is streaming 16-byte stores, counted
    exactly; pg_parse queues it on the side stream, so it runs before K3's
    event span and is reported apart from K3 (table_clear_hbm_bytes_per_build).
  * WRITE_SIZE counts a returning 64-bit atomic (CAS) as 64 B, a
    non-returning atomicOr as 32 B and streaming stores exactly.
"""
from __future__ import annotations

import collections
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")


def short(name: str) -> str:
    n = re.sub(r"\(.*", "", name)
    return n.replace("void ", "").strip()


def collect(pattern: str, drop_first: bool):
    """Per kernel and counter: the value per BUILD (one bench step), i.e. the
    sum over the kernel's dispatches of a step (K3 runs in chunks: several
    k_cover / k_insert_work dispatches per step), averaged over the steps;
    the first step (the warm-up build on the larger first-guess table) is
    dropped.  A step is delimited by the k_reduce dispatches (one per step)."""
    vals = collections.defaultdict(list)
    per_file_reduce = {}
    for f in sorted(glob.glob(os.path.join(OUT, pattern, "pmc_counter_collection.csv"))):
        rows = list(csv.DictReader(open(f)))
        for r in rows:
            vals[(short(r["Kernel_Name"]), r["Counter_Name"], f)].append((int(r["Dispatch_Id"]),
                                                                           float(r["Counter_Value"])))
        per_file_reduce[f] = sorted({int(r["Dispatch_Id"]) for r in rows if "k_reduce" in r["Kernel_Name"]})
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for (k, c, f), v in vals.items():
        bounds = per_file_reduce.get(f) or []
        if not bounds:                                 # no step structure (calibration runs)
            acc[k][c].append(sum(x for _, x in v) / len(v))
            continue
        steps = collections.defaultdict(float)
        for d, x in v:
            steps[sum(1 for b in bounds if b < d)] += x   # step index = k_reduce dispatches before d
        keys = sorted(steps)
        if drop_first and len(keys) > 1:
            keys = keys[1:]
        acc[k][c].append(sum(steps[s] for s in keys) / len(keys))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def main(config: str = "c3"):
    pmc = collect("pmc3_*", True)
    cov = next(k for k in pmc if k.startswith("pg::k_cover") or k.startswith("pg::k_insert<"))
    work = next((k for k in pmc if k.startswith("pg::k_insert_work")), None)
    kb = 1024.0
    t_cov = 2 * pmc[cov]["FETCH_SIZE"] * kb + pmc[cov]["WRITE_SIZE"] * kb
    t_work = (pmc[work]["FETCH_SIZE"] + pmc[work]["WRITE_SIZE"]) * kb if work else 0.0
    zk = next((k for k in pmc if k.startswith("pg::k_zero16")), None)
    t_zero = (2 * pmc[zk]["FETCH_SIZE"] + pmc[zk]["WRITE_SIZE"]) * kb if zk else 0.0
    hit = {k: v["TCC_HIT_sum"] / (v["TCC_HIT_sum"] + v["TCC_MISS_sum"]) for k, v in pmc.items()
           if "TCC_HIT_sum" in v and v["TCC_HIT_sum"] + v["TCC_MISS_sum"] > 0}
    res = {
        "kernel": "K3 = %s (coverage passes) + %s (work passes), all chunks of one build; the table "
                  "clear (k_zero16) is queued by pg_parse on the side stream and runs before K3's event "
                  "span, so it is reported separately" % (cov, work),
        "config": "%s (bench.py default), 1 x MI355X" % config,
        "k_insert_hbm_bytes_per_launch": int(t_cov + t_work),
        "per_pass_bytes": {cov: int(t_cov), work: int(t_work)},
        "table_clear_hbm_bytes_per_build": int(t_zero),
        "method": __doc__.split("HBM bytes per K3 launch", 1)[1].strip(),
        "raw_per_launch": {k: dict(sorted(v.items())) for k, v in sorted(pmc.items())},
        "l2_hit_rate": hit,
    }
    calib = collect("calib_*", False)
    if calib:
        cj = {k: dict(sorted(v.items())) for k, v in sorted(calib.items()) if k.startswith("c_")}
        json.dump({"tool": "tools/fetch_calib.hip via tools/calib.sh; 2 GiB buffer, 64 M accesses per random "
                           "kernel (16 384 blocks x 256 lanes x 16), 1 GiB for stream16/store16",
                   "per_kernel": cj,
                   "bytes_requested": {"c_stream16": 2 ** 30, "c_rand16": 64 * 2 ** 20 * 16,
                                       "c_rand8": 64 * 2 ** 20 * 8, "c_cas8": 64 * 2 ** 20 * 8,
                                       "c_or8": 64 * 2 ** 20 * 8, "c_store16": 2 ** 30}},
                  open(os.path.join(ROOT, "profiles", "fetch_calib.json"), "w"), indent=1)
    json.dump(res, open(os.path.join(ROOT, "profiles", "traffic_%s.json" % config), "w"), indent=1)
    print(json.dumps({"traffic": res["k_insert_hbm_bytes_per_launch"], "per_pass": res["per_pass_bytes"]}))


if __name__ == "__main__":
    main(*sys.argv[1:])

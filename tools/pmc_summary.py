#!/usr/bin/env python3
"""Fold the rocprofv3 PMC passes of tools/pmc_insert.sh (gpurun_out/pmc3_*/)
and the calibration passes of tools/calib.sh (gpurun_out/calib_*/) into
profiles/traffic_<config>.json, the file bench.py reads `roofline.traffic`
from.  Development tool; not part of the product.

Per kernel and counter, the first dispatch of the process is dropped (the
warm-up build runs on a larger first-guess table) and the rest averaged.

HBM bytes per K3 launch (coverage pass + work pass), from the calibration
(tools/fetch_calib.hip, profiles/fetch_calib.json):
  * FETCH_SIZE counts 64 B per memory read request.  A random 16-B or 8-B
    load is one 64-B request (counted exactly); a coalesced 16 B/lane stream
    issues 128-B requests, counted at half (MI355X_MICROARCH.md).  The
    coverage pass is a class-stream read (its random bucket probes hit L2),
    so its FETCH_SIZE is doubled; the work pass is dominated by random
    bucket loads, so its FETCH_SIZE is taken as is (its streamed class bytes,
    <= 0.5 GB, are then under-counted by half - a lower bound).
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
    vals = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(OUT, pattern, "pmc_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            vals[(short(r["Kernel_Name"]), r["Counter_Name"])].append((int(r["Dispatch_Id"]),
                                                                        float(r["Counter_Value"])))
    out = collections.defaultdict(dict)
    for (k, c), v in vals.items():
        v.sort()
        xs = [x for _, x in (v[1:] if drop_first and len(v) > 1 else v)]
        out[k][c] = sum(xs) / len(xs)
    return out


def main(config: str = "c3"):
    pmc = collect("pmc3_*", True)
    cov = next(k for k in pmc if k.startswith("pg::k_cover") or k.startswith("pg::k_insert<"))
    work = next((k for k in pmc if k.startswith("pg::k_insert_work")), None)
    kb = 1024.0
    t_cov = 2 * pmc[cov]["FETCH_SIZE"] * kb + pmc[cov]["WRITE_SIZE"] * kb
    t_work = (pmc[work]["FETCH_SIZE"] + pmc[work]["WRITE_SIZE"]) * kb if work else 0.0
    hit = {k: v["TCC_HIT_sum"] / (v["TCC_HIT_sum"] + v["TCC_MISS_sum"]) for k, v in pmc.items()
           if "TCC_HIT_sum" in v and v["TCC_HIT_sum"] + v["TCC_MISS_sum"] > 0}
    res = {
        "kernel": "K3 = %s (coverage pass) + %s (work pass)" % (cov, work),
        "config": "%s (bench.py default), 1 x MI355X" % config,
        "k_insert_hbm_bytes_per_launch": int(t_cov + t_work),
        "per_pass_bytes": {cov: int(t_cov), work: int(t_work)},
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

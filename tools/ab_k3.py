#!/usr/bin/env python3
"""Development A/B of K3 variants on the C3 batch c3a, HBM-resident input
(pg_build_device; --host: pg_build_host from the mmap), alternating the variants step by step in one process.

    python tools/ab_k3.py [--steps 12] [--tune WHAT=V,WHAT=V ...] ...

Each --tune argument is one variant (a comma-separated list of pg_tune
settings by PG_TUNE_* name, or "base" for none).  Prints per variant the
median step, stage A / split / range spans (HIP events), stage A records, and
whether every step's counts match the oracle digest of c3a."""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--genomes", type=int, default=100)
    ap.add_argument("--tune", action="append", default=[])
    ap.add_argument("--host", action="store_true", help="pg_build_host from the page-cache-warm mmap instead")
    args = ap.parse_args()
    import torch
    from pangenome_amd import _lib, kmer, synth
    variants = args.tune or ["base"]
    tmp = tempfile.mkdtemp(prefix="ab_k3_")
    p = os.path.join(tmp, "c3a.fa")
    t0 = time.time()
    synth.write_pangenome(p, args.genomes, 5_000_000, first_index=0, workers=16)
    print("generated %.1f s" % (time.time() - t0), flush=True)
    mm = kmer.seq2bytes(p)
    d = torch.from_numpy(np.array(mm)).to("cuda:0")
    if not args.host:
        os.unlink(p)
    dig = json.load(open(os.path.join(ROOT, "tests", "golden", "scale", "c3a.json"))) if args.genomes == 100 else None
    ctxs = []
    for v in variants:
        ctx = _lib.Context(27, 0)
        if v != "base":
            for kv in v.split(","):
                what, val = kv.split("=")
                ctx.tune(getattr(_lib, "PG_TUNE_" + what), int(val))
        ctxs.append(ctx)
    res = {v: [] for v in variants}
    for step in range(args.steps + 2):
        for v, ctx in zip(variants, ctxs):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            if args.host:
                st = ctx.build_host(mm, True)
            else:
                st = ctx.build_device(d.data_ptr(), d.numel(), True, keepalive=d)
            ms = 1e3 * (time.perf_counter() - t1)
            ok = dig is None or (st.n_dbg, st.n_rdbg) == (dig["n_dbg"], dig["n_rdbg"])
            if step >= 2:
                res[v].append((ms, st.ms_parse, st.ms_insert, st.ms_split, st.ms_range, st.n_records_a, ok))
    for v in variants:
        a = np.array([r[:6] for r in res[v]])
        med = np.median(a, axis=0)
        print("%-40s step %.3f  parse %.3f  stageA %.3f  split %.3f  range %.3f  recA %d  ok %s" %
              (v, med[0], med[1], med[2], med[3], med[4], int(med[5]), all(r[6] for r in res[v])), flush=True)


if __name__ == "__main__":
    main()

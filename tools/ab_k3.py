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
    ap.add_argument("--alt", action="store_true", help="alternate two batches (genomes 0-99, 100-199), as bench.py does")
    ap.add_argument("--env", action="append", default=[], help="per-variant environment NAME=V (index-aligned with --tune)")
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
    mms = [mm]
    if args.alt:
        p2 = os.path.join(tmp, "c3b.fa")
        synth.write_pangenome(p2, args.genomes, 5_000_000, first_index=args.genomes, workers=16)
        mms.append(kmer.seq2bytes(p2))
    ds = [torch.from_numpy(np.array(m)).to("cuda:0") for m in mms]   # (--alt: both batches in HBM)
    if not args.host:
        os.unlink(p)
    digs = [json.load(open(os.path.join(ROOT, "tests", "golden", "scale", n + ".json"))) for n in ("c3a", "c3b")] \
        if args.genomes == 100 else [None, None]
    ctxs = []
    for v in variants:
        ctx = _lib.Context(27, 0)
        if v != "base":
            for kv in v.split(","):
                what, val = kv.split("=")
                ctx.tune(getattr(_lib, "PG_TUNE_" + what), int(val))
        ctxs.append(ctx)
    res = [[] for _ in variants]
    envs = dict(e.split("=", 1) for e in args.env)
    for step in range(args.steps + 2):
        for vi, (v, ctx) in enumerate(zip(variants, ctxs)):
            for e in envs:
                os.environ.pop(e, None)
            if vi < len(args.env):
                name, val = args.env[vi].split("=", 1)
                if val:
                    os.environ[name] = val
            b = step % len(mms)
            dig = digs[b]
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            if args.host:
                st = ctx.build_host(mms[b], True)
            else:
                d = ds[b]
                st = ctx.build_device(d.data_ptr(), d.numel(), True, keepalive=d)
            ms = 1e3 * (time.perf_counter() - t1)
            ok = dig is None or (st.n_dbg, st.n_rdbg) == (dig["n_dbg"], dig["n_rdbg"])
            if step >= 2:
                res[vi].append((ms, st.ms_parse, st.ms_insert, st.ms_split, st.ms_range, st.n_records_a, ok))
    for vi, v in enumerate(variants):
        a = np.array([r[:6] for r in res[vi]])
        med = np.median(a, axis=0)
        print("%-40s step %.3f (max %.3f)  parse %.3f  stageA %.3f  split %.3f  range %.3f  recA %d  ok %s" %
              (v + (" " + args.env[vi] if vi < len(args.env) else ""), med[0], a[:, 0].max(), med[1], med[2],
               med[3], med[4], int(med[5]), all(r[6] for r in res[vi])), flush=True)


if __name__ == "__main__":
    main()

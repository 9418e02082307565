#!/usr/bin/env python3
"""Development sweep (not part of the product): pg_build_host from a
page-cache-warm mmap of C3 batch A against the staging ring's piece size,
slot count and thread count; and the bare staged upload (pg_set_fasta)."""
import itertools
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    from scale_util import make_input
    from pangenome_amd import kmer
    from pangenome_amd._lib import Context, PG_TUNE_HOST_REGISTER, PG_TUNE_HOST_THREADS, PG_TUNE_STAGE_PIECE, PG_TUNE_STAGE_SLOTS
    fa = make_input("c3a")
    d = tempfile.mkdtemp()
    q = os.path.join(d, "c3.fa")
    open(q, "wb").write(fa)
    del fa
    mm = kmer.seq2bytes(q)
    ctx = Context(27)
    res = []
    combos = [c + (0,) for c in itertools.product((8, 16, 32, 64), (4, 6, 8), (4, 8, 12))]
    if len(sys.argv) > 1:
        combos = [tuple(int(x) for x in a.split(",")) for a in sys.argv[1:]]
    for piece, slots, thr, reg in combos:
        ctx.tune(PG_TUNE_STAGE_PIECE, piece << 20)
        ctx.tune(PG_TUNE_STAGE_SLOTS, min(slots, 8))
        ctx.tune(PG_TUNE_HOST_THREADS, thr)
        ctx.tune(PG_TUNE_HOST_REGISTER, reg)
        t = time.perf_counter()
        ctx.build_host(mm, True)
        first = time.perf_counter() - t
        for _ in range(2):
            ctx.build_host(mm, True)
        ts = []
        for _ in range(8):
            t = time.perf_counter()
            ctx.build_host(mm, True)
            ts.append(time.perf_counter() - t)
        us = []
        for _ in range(4):
            t = time.perf_counter()
            ctx.set_fasta(mm)
            us.append(time.perf_counter() - t)
        r = {"piece_mib": piece, "slots": slots, "threads": thr, "register": reg, "first_ms": round(1e3 * first, 3), "window_ms_mean": round(1e3 * sum(ts) / len(ts), 3),
             "window_ms_min": round(1e3 * min(ts), 3), "upload_ms_min": round(1e3 * min(us), 3)}
        res.append(r)
        print(json.dumps(r), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(res, open("gpurun_out/stage_sweep.json", "w"), indent=1)


if __name__ == "__main__":
    main()

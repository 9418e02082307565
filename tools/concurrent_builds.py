#!/usr/bin/env python3
"""Development measurement (not part of the product): C3 builds from HBM
(pg_build_device) back to back in one context, against the same number of
builds spread over `--ctx` contexts, one host thread each (ctypes releases
the GIL during the call), on one GPU: does a second build in flight fill
what one build leaves idle?  Alternating batches as bench.py; every build's
counts are checked against the oracle digests.

    python tools/concurrent_builds.py [--builds 24] [--ctx 2]
"""
import argparse
import json
import os
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--builds", type=int, default=24)
    ap.add_argument("--ctx", type=int, default=2)
    args = ap.parse_args()
    import numpy as np
    import torch
    from pangenome_amd import _lib, kmer, synth
    tmp = tempfile.mkdtemp(prefix="conc_")
    ds, digs = [], []
    for name, first in (("c3a", 0), ("c3b", 100)):
        p = os.path.join(tmp, name + ".fa")
        synth.write_pangenome(p, 100, 5_000_000, first_index=first, workers=16)
        ds.append(torch.from_numpy(np.array(kmer.seq2bytes(p))).to("cuda:0"))
        os.unlink(p)
        digs.append(json.load(open(os.path.join(ROOT, "tests", "golden", "scale", name + ".json"))))
    ctxs = [_lib.Context(27, 0) for _ in range(args.ctx)]
    bases = [0, 0]
    ok = [True]

    def build(ctx, i):
        d = ds[i % 2]
        st = ctx.build_device(d.data_ptr(), d.numel(), True, keepalive=d)
        if (st.n_dbg, st.n_rdbg) != (digs[i % 2]["n_dbg"], digs[i % 2]["n_rdbg"]):
            ok[0] = False
        return st.n_bases

    for c in ctxs:                                   # warm every context on both batches
        build(c, 0)
        build(c, 1)
    torch.cuda.synchronize()
    res = {}
    # one context, sequential
    t0 = time.perf_counter()
    nb = sum(build(ctxs[0], i) for i in range(args.builds))
    torch.cuda.synchronize()
    t1 = time.perf_counter() - t0
    res["one_ctx"] = {"ms_per_build": round(1e3 * t1 / args.builds, 3), "gbps": round(nb / t1 / 1e9, 2)}

    # `ctx` contexts, one thread each, builds dealt round-robin
    def worker(k, out):
        out[k] = sum(build(ctxs[k], i) for i in range(k, args.builds, args.ctx))
    out = [0] * args.ctx
    th = [threading.Thread(target=worker, args=(k, out)) for k in range(args.ctx)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    torch.cuda.synchronize()
    t2 = time.perf_counter() - t0
    res["%d_ctx" % args.ctx] = {"ms_per_build": round(1e3 * t2 / args.builds, 3), "gbps": round(sum(out) / t2 / 1e9, 2)}
    res["ok"] = ok[0]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

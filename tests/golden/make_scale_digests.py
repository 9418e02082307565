#!/usr/bin/env python3
"""Benchmark-scale parity digests: the pinned C oracle run on the exact inputs
bench.py measures (TEST INFRASTRUCTURE; run in the build container).

The oracle (oracle/pg_oracle.c, a faithful restatement of kmer_numba.py's
oakht / build_dbg / build_rdbg_jit_) is pinned bit-for-bit against the
reference's own fixtures by tests/test_oracle_golden.py.  Running it on the
full C3 and C2 inputs takes a few minutes of one core each, too slow for a GPU
test, so this script stores compact digests of its results instead:

* n_dbg, n_rdbg and the sentinel flag;
* SHA-256 of the dBG sorted by key: the little-endian uint64 keys followed by
  the little-endian uint16 12-bit masks (dump()'s content, :243-261);
* SHA-256 of the sorted rdBG keys (dbg2rdbg, :1313-1321);
* for C2 (one record, cheap to walk): SHA-256 of the `.xyz` text and of the
  region rows with an empty `.mcl` (seq2graph, :1853-1951).

Inputs are regenerated from pangenome_amd/synth.py (deterministic splitmix64),
so only the digests are committed (tests/golden/scale/*.json).

Inputs with a `ranges` count (C5 at full chunk size: billions of keys, more
than one in-memory oakht holds) are digested key range by key range with the
oracle's sorted form (pgo_dbg_range, pinned to the reference's fixtures like
the oakht form by tests/test_oracle_golden.py): the ranges are consecutive,
so their sorted outputs concatenate into the same SHA-256 streams.  `--ranged`
digests any input that way (c5s's agreement with its oakht digest checks the
two forms against each other at scale).

    python tests/golden/make_scale_digests.py [--ranged] [--workers W] [c3a c3b c2 ...]
"""
from __future__ import annotations

import json
import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.dirname(HERE))

from scale_util import INPUTS, make_input, dbg_digest, rdbg_digest, text_digest  # noqa: E402

OUT = os.path.join(HERE, "scale")


def one(name: str):
    from oracle import oracle
    spec = INPUTS[name]
    fasta = make_input(name)
    t0 = time.time()
    r = oracle.OracleRun(fasta, spec["k"], spec["c"])
    dk, dm = r.dbg()
    rk = r.rdbg()
    res = {"name": name, "desc": spec["desc"], "k": spec["k"], "c": spec["c"],
           "fasta_bytes": len(fasta), "n_bases": int(r.n_bases()),
           "n_dbg": int(dk.shape[0]), "n_rdbg": int(rk.shape[0]),
           "sentinel": bool(dk.shape[0] and dk[-1] == 2 ** 64 - 1),
           "dbg_sha256": dbg_digest(dk, dm), "rdbg_sha256": rdbg_digest(rk)}
    if spec.get("walk"):
        xyz = r.xyz()
        rows = r.rows(oracle.label_table(xyz, ""))
        res["n_edges"] = xyz.count("\n")
        res["n_rows"] = len(rows)
        res["xyz_sha256"] = text_digest(xyz)
        res["rows_sha256"] = text_digest("".join(x + "\n" for x in rows))
    res["oracle_seconds"] = round(time.time() - t0, 1)
    return res


def _range_job(args):
    """one key range of a ranged digest: its sorted dBG keys, masks and rdBG
    keys saved under `tmp` (the parent hashes them in range order)"""
    import numpy as np
    from oracle import oracle
    path, k, c, lo, hi, idx, tmp = args
    buf = np.memmap(path, dtype=np.uint8, mode="r")
    keys, masks = oracle.dbg_range(buf, k, c, lo, hi)
    np.save(os.path.join(tmp, "k%04d.npy" % idx), keys)
    np.save(os.path.join(tmp, "m%04d.npy" % idx), masks)
    np.save(os.path.join(tmp, "r%04d.npy" % idx), keys[oracle.rdbg_member(masks)])
    return idx, int(keys.shape[0])


def _fasta_bases(buf) -> int:
    """seqio_jit_'s base count (:160-167) of a FASTA whose every line ends
    in '\n': the bytes of the sequence lines, each without its last byte."""
    import numpy as np
    nl = np.flatnonzero(np.asarray(buf) == 10)
    starts = np.concatenate([[0], nl[:-1] + 1])
    hdr = np.asarray(buf)[starts] == 62
    lens = nl - starts                                   # without the '\n'
    return int(lens[~hdr].sum())


def one_ranged(name: str, workers: int, parts=None):
    import hashlib
    import tempfile
    import numpy as np
    from oracle import oracle
    from pangenome_amd import synth
    spec = INPUTS[name]
    parts = parts or spec.get("ranges", 16)
    t0 = time.time()
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as tmp:
        path = os.path.join(tmp, name + ".fa")
        if spec["kind"] == "c5pairs":
            nbytes = synth.write_c5(path, pairs=spec["pairs"], workers=min(workers, 8))
        else:
            data = make_input(name)
            open(path, "wb").write(data)
            nbytes = len(data)
        t_gen = time.time() - t0
        jobs = [(path, spec["k"], spec["c"], lo, hi, i, tmp) for i, (lo, hi) in enumerate(oracle.key_ranges(spec["k"], parts))]
        hk, hr = hashlib.sha256(), hashlib.sha256()
        n_dbg = n_rdbg = 0
        last = -1
        sentinel = False
        done = {}
        with ProcessPoolExecutor(max_workers=workers) as ex:
            for idx, _ in ex.map(_range_job, jobs):
                done[idx] = True
                while last + 1 in done:              # hash the ranges in order as they complete
                    last += 1
                    kf = os.path.join(tmp, "k%04d.npy" % last)
                    keys = np.load(kf)
                    hk.update(np.ascontiguousarray(keys, dtype="<u8").tobytes())
                    n_dbg += keys.shape[0]
                    sentinel |= bool(keys.shape[0] and keys[-1] == 2 ** 64 - 1)
                    os.unlink(kf)
                    rf = os.path.join(tmp, "r%04d.npy" % last)
                    rk = np.load(rf)
                    hr.update(np.ascontiguousarray(rk, dtype="<u8").tobytes())
                    n_rdbg += rk.shape[0]
                    os.unlink(rf)
                    print("  %s: range %d/%d, %d keys so far, %.0f s" % (name, last + 1, parts, n_dbg,
                                                                         time.time() - t0), flush=True)
        for i in range(parts):                       # dbg_digest: all keys, then all masks
            hk.update(np.ascontiguousarray(np.load(os.path.join(tmp, "m%04d.npy" % i)), dtype="<u2").tobytes())
        n_bases = _fasta_bases(np.memmap(path, dtype=np.uint8, mode="r"))
    res = {"name": name, "desc": spec["desc"], "k": spec["k"], "c": spec["c"], "fasta_bytes": nbytes,
           "n_bases": n_bases, "n_dbg": n_dbg, "n_rdbg": n_rdbg, "sentinel": sentinel,
           "dbg_sha256": hk.hexdigest(), "rdbg_sha256": hr.hexdigest(),
           "oracle": "pgo_dbg_range over %d key ranges" % parts, "generate_seconds": round(t_gen, 1),
           "oracle_seconds": round(time.time() - t0 - t_gen, 1)}
    return res


def main(argv):
    os.makedirs(OUT, exist_ok=True)
    from oracle import oracle
    oracle.build()
    ranged = "--ranged" in argv
    workers = 4
    if "--workers" in argv:
        workers = int(argv[argv.index("--workers") + 1])
        argv = argv[:argv.index("--workers")] + argv[argv.index("--workers") + 2:]
    names = [a for a in argv if not a.startswith("--")] or sorted(INPUTS)
    big = [n for n in names if ranged or INPUTS[n].get("ranges")]
    small = [n for n in names if n not in big]
    results = []
    if small:
        with ProcessPoolExecutor(max_workers=min(4, len(small))) as ex:
            results += list(ex.map(one, small))
    for n in big:
        results.append(one_ranged(n, workers))
    for res in results:
        with open(os.path.join(OUT, res["name"] + (".ranged" if ranged and not INPUTS[res["name"]].get("ranges")
                                                   else "") + ".json"), "w") as f:
            json.dump(res, f, indent=1, sort_keys=True)
            f.write("\n")
        print(res["name"], res["n_dbg"], res["n_rdbg"], res["oracle_seconds"], "s", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])

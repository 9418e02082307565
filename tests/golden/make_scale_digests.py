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

    python tests/golden/make_scale_digests.py [c3a c3b c2 ...]
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


def main(names):
    os.makedirs(OUT, exist_ok=True)
    from oracle import oracle
    oracle.build()
    with ProcessPoolExecutor(max_workers=min(4, len(names))) as ex:
        for res in ex.map(one, names):
            with open(os.path.join(OUT, res["name"] + ".json"), "w") as f:
                json.dump(res, f, indent=1, sort_keys=True)
                f.write("\n")
            print(res["name"], res["n_dbg"], res["n_rdbg"], res["oracle_seconds"], "s", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:] or sorted(INPUTS))

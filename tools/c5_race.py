#!/usr/bin/env python3
"""Development check (not part of the product): the c5m input (tests/golden/
scale/c5m.json) through the streamed exchange at 2^30 bases per chunk, the
rank's own run sent through RCCL, with and without dist._fence
(PG_DEBUG_NO_FENCE=1 restores round 4's unfenced exchange), N times each.
With the integrity checks on, an unfenced run that races prints the
ExchangeIntegrityError naming where the records changed.

    python tools/c5_race.py [nofence_runs] [fenced_runs]
"""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _rank(rank, world, port, q, path, nofence):
    os.environ["PG_EXCHANGE_SELF_RCCL"] = "1"
    if nofence:
        os.environ["PG_DEBUG_NO_FENCE"] = "1"
    import test_gpu_c5
    from pangenome_amd import dist as pdist
    try:
        test_gpu_c5._c5_rank(rank, world, port, q, path, "nccl", 1 << 30, None, False, None, "rccl")
    except pdist.ExchangeIntegrityError as e:
        q.put((rank, {"error": str(e)}))
        raise SystemExit(0)


def main():
    from pangenome_amd import synth
    from dist_util import spawn_ranks
    from scale_util import INPUTS, load_digest
    n_nofence = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    n_fenced = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    dg = load_digest("c5m")
    want = [dg["n_dbg"], dg["n_rdbg"], dg["rdbg_sha256"]]
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as d:
        p = os.path.join(d, "c5m.fa")
        t0 = time.time()
        synth.write_c5(p, pairs=INPUTS["c5m"]["pairs"], workers=10)
        print("generated in %.0f s" % (time.time() - t0), flush=True)
        for nofence in [True] * n_nofence + [False] * n_fenced:
            r = spawn_ranks(1, _rank, (p, nofence), timeout=800)[0]
            ok = "stream" in r and [r["stream"][0], r["stream"][1], r["stream"][3]] == want
            print(json.dumps({"fence": not nofence, "ok_vs_oracle": ok, "result": r}), flush=True)


if __name__ == "__main__":
    main()

"""Development: C3 batch A through pg_build_device with the packed coverage
pass (form 0) and the quad form (form 2, matches the oracle digest); the dBG
entries the packed build lost or changed, saved for offline analysis.

    python tools/dbg_missing.py out.npz
"""
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from pangenome_amd import _lib, kmer, synth
    tmp = tempfile.mkdtemp(prefix="dbg_miss_")
    p = os.path.join(tmp, "c3a.fa")
    synth.write_pangenome(p, 100, 5_000_000, first_index=0, workers=16)
    mm = kmer.seq2bytes(p)
    d = torch.from_numpy(np.array(mm)).to("cuda:0")
    dig = json.load(open(os.path.join(ROOT, "tests", "golden", "scale", "c3a.json")))
    ref = _lib.Context(27, 0)
    ref.tune(_lib.PG_TUNE_K3_COVER, 2)
    st = ref.build_device(d.data_ptr(), d.numel(), True, keepalive=d)
    assert (st.n_dbg, st.n_rdbg) == (dig["n_dbg"], dig["n_rdbg"])
    rk, rm = ref.dbg()
    ref.close()
    ctx = _lib.Context(27, 0)
    out = {}
    for i in range(6):
        st = ctx.build_device(d.data_ptr(), d.numel(), True, keepalive=d)
        ok = (st.n_dbg, st.n_rdbg) == (dig["n_dbg"], dig["n_rdbg"])
        print("packed build %d: n_dbg %d n_rdbg %d ok %s" % (i, st.n_dbg, st.n_rdbg, ok), flush=True)
        if not ok:
            k, m = ctx.dbg()
            lost = np.setdiff1d(rk, k)
            extra = np.setdiff1d(k, rk)
            both, ia, ib = np.intersect1d(rk, k, return_indices=True)
            changed = both[rm[ia] != m[ib]]
            print("lost %d extra %d changed-mask %d" % (lost.shape[0], extra.shape[0], changed.shape[0]), flush=True)
            sel = np.isin(rk, np.concatenate([lost, changed]))
            out = dict(keys=rk[sel], masks_ref=rm[sel], lost=lost, extra=extra, changed=changed,
                       masks_got=np.array([m[np.searchsorted(k, x)] if np.searchsorted(k, x) < k.shape[0] and
                                           k[np.searchsorted(k, x)] == x else 0 for x in rk[sel]], np.uint16))
            break
    ctx.close()
    np.savez(sys.argv[1], **out)
    os.unlink(p)


if __name__ == "__main__":
    main()

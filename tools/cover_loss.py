"""Stage A record count vs the ideal coverage rule (diagnostic).

A window of a follower is covered when its k+2 context (the k-mer and both
neighbour bases) occurs in a reference at any offset: the reference's record
then carries the same key and masks.  This counts, on a synthetic pangenome,
the records an ideal pass with the lead alone, lead + ref2 (the shipped rule)
and lead + ref2 + ref3 would leave, beside the distinct canonical keys; with
--gpu it adds the library's own stage A record count (PgStats.n_records_a) for
the same input, so the gap between the shipped kernel and its ideal is
measured, not guessed.

  python tools/cover_loss.py --genomes 20 --length 1000000 [--gpu]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from pangenome_amd import synth  # noqa: E402


def ctx_codes(d: np.ndarray, w: int) -> np.ndarray:
    """2-bit packed codes of every w-base substring of digits d (w <= 32)."""
    n = d.shape[0] - w + 1
    if n <= 0:
        return np.zeros(0, np.uint64)
    c = np.zeros(n, np.uint64)
    for j in range(w):
        c = (c << np.uint64(2)) | d[j:j + n].astype(np.uint64)
    return c


def canon_keys(d: np.ndarray, k: int) -> np.ndarray:
    f = ctx_codes(d, k)
    r = ctx_codes((3 - d[::-1]).astype(np.uint8), k)[::-1]
    return np.minimum(f, r)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--genomes", type=int, default=20)
    ap.add_argument("--length", type=int, default=1_000_000)
    ap.add_argument("--snp", type=float, default=1e-3)
    ap.add_argument("--indel", type=float, default=1e-4)
    ap.add_argument("--k", type=int, default=27)
    ap.add_argument("--seed", type=int, default=synth.DEFAULT_SEED)
    ap.add_argument("--gpu", action="store_true")
    ap.add_argument("--no-ideal", action="store_true", help="the GPU count only")
    a = ap.parse_args()
    k, w = a.k, a.k + 2
    base = synth.base_genome(a.length, a.seed)
    gens = [synth.variant(base, gi, a.snp, a.indel, a.seed) for gi in range(a.genomes)]
    # the library's reference choice: longest two (stable), make_tiles
    order = sorted(range(a.genomes), key=lambda g: -gens[g].shape[0])
    refs = [np.unique(ctx_codes(gens[g], w)) for g in order[:3]]
    out = {"windows": int(sum(g.shape[0] - k + 1 for g in gens))}
    for nref in (() if a.no_ideal else (1, 2, 3)):
        tot = gens[order[0]].shape[0] - k + 1
        for i, g in enumerate(order[1:], 1):
            c = ctx_codes(gens[g], w)
            cov = np.zeros(c.shape[0], bool)
            for r in refs[:min(nref, i)]:
                cov |= np.isin(c, r)
            tot += int((~cov).sum()) + 2          # the two end windows have no full context
        out["ideal_refs%d" % nref] = tot
    if not a.no_ideal:
        out["distinct_keys"] = int(np.unique(np.concatenate([canon_keys(g, k) for g in gens])).shape[0])
    if a.gpu:
        from pangenome_amd._lib import Context
        fasta = b"".join(synth.to_fasta_lines(b"g%d" % gi, g) for gi, g in enumerate(gens))
        ctx = Context(k)
        ctx.set_fasta(fasta)
        ctx.parse()
        st = ctx.build(None, 0, True)
        out["gpu_records_a"] = int(st.n_records_a)
        out["gpu_work_items"] = int(st.n_work_items)
        ctx.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()

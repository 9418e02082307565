"""Synthetic pangenome FASTA generator (splitmix64, numpy-vectorised).

The reference ships no benchmark inputs; the
configurations named in BASELINE.json are rebuilt here from the model stated in
SURVEY.md §8(d): a random base genome plus per-genome SNPs and short indels,
uppercase ACGT, 60-column lines, ``\\n`` line ends and a trailing newline.

Everything is deterministic in (seed, genome index), so every rank of a
multi-GPU run can build its own shard without communication.
"""
from __future__ import annotations

import numpy as np

GAMMA = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)
DEFAULT_SEED = 0x5EED2026
ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)


def splitmix64(seed: int, stream: int, n: int) -> np.ndarray:
    """n outputs of splitmix64 started at state ``seed ^ mix(stream)``."""
    with np.errstate(over="ignore"):
        base = np.uint64((seed ^ (stream * 0xD1B54A32D192ED03)) & 0xFFFFFFFFFFFFFFFF)
        z = base + (np.arange(1, n + 1, dtype=np.uint64) * GAMMA)
        z = (z ^ (z >> np.uint64(30))) * M1
        z = (z ^ (z >> np.uint64(27))) * M2
        return z ^ (z >> np.uint64(31))


def uniform(seed: int, stream: int, n: int) -> np.ndarray:
    return (splitmix64(seed, stream, n) >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))


def base_genome(length: int, seed: int = DEFAULT_SEED) -> np.ndarray:
    """Random ACGT digits (0..3) of a base genome."""
    return (splitmix64(seed, 1, length) >> np.uint64(62)).astype(np.uint8)


def variant(base: np.ndarray, index: int, snp: float, indel: float,
            seed: int = DEFAULT_SEED) -> np.ndarray:
    """One mutated copy of ``base`` (digits 0..3): SNPs then 1-10 bp indels."""
    n = base.shape[0]
    s = seed + 7919 * (index + 1)
    g = base.copy()
    if snp > 0:
        u = uniform(s, 2, n)
        pos = np.nonzero(u < snp)[0]
        shift = (splitmix64(s, 3, pos.shape[0]) % np.uint64(3)).astype(np.uint8) + 1
        g[pos] = (g[pos] + shift) & 3
    if indel > 0:
        u = uniform(s, 4, n)
        pos = np.nonzero(u < indel)[0]
        r = splitmix64(s, 5, pos.shape[0])
        lens = (r % np.uint64(10)).astype(np.int64) + 1
        ins = ((r >> np.uint64(8)) & np.uint64(1)).astype(bool)
        # deletions: drop [p, p+len)
        dpos, dlen = pos[~ins], lens[~ins]
        keep = np.ones(n, dtype=bool)
        if dpos.shape[0]:
            idx = np.concatenate([np.arange(p, min(p + l, n)) for p, l in zip(dpos, dlen)])
            keep[idx] = False
        # insertions before position p (in original coordinates)
        ipos, ilen = pos[ins], lens[ins]
        if ipos.shape[0]:
            total = int(ilen.sum())
            ib = (splitmix64(s, 6, total) >> np.uint64(62)).astype(np.uint8)
            offs = np.repeat(ipos, ilen)
            out_idx = np.concatenate([np.nonzero(keep)[0], offs])
            out_val = np.concatenate([g[keep], ib])
            order = np.argsort(out_idx, kind="stable")
            return out_val[order]
        return g[keep]
    return g


def to_fasta_lines(name: bytes, digits: np.ndarray, width: int = 60) -> bytes:
    """Format one record: ``>name\\n`` then ``width``-column lines with ``\\n``."""
    seq = ACGT[digits]
    n = seq.shape[0]
    full = n // width
    rem = n - full * width
    body = np.empty(full * (width + 1) + (rem + 1 if rem else 0), dtype=np.uint8)
    if full:
        v = body[: full * (width + 1)].reshape(full, width + 1)
        v[:, :width] = seq[: full * width].reshape(full, width)
        v[:, width] = 10
    if rem:
        body[full * (width + 1): full * (width + 1) + rem] = seq[full * width:]
        body[-1] = 10
    return b">" + name + b"\n" + body.tobytes()


def pangenome(n_genomes: int, genome_len: int, snp: float = 1e-3, indel: float = 1e-4,
              seed: int = DEFAULT_SEED, first_index: int = 0,
              records_per_genome: int = 1, width: int = 60) -> bytes:
    """FASTA bytes of ``n_genomes`` variants of one base genome.

    ``first_index`` lets ranks of a weak-scaling run draw disjoint genomes of the
    same population (rank r uses indices r*n .. r*n+n-1).
    """
    base = base_genome(genome_len, seed)
    parts = []
    for gi in range(first_index, first_index + n_genomes):
        v = variant(base, gi, snp, indel, seed)
        if records_per_genome == 1:
            parts.append(to_fasta_lines(b"g%d" % gi, v, width))
        else:
            cuts = np.linspace(0, v.shape[0], records_per_genome + 1).astype(np.int64)
            for j in range(records_per_genome):
                parts.append(to_fasta_lines(b"g%d_c%d" % (gi, j), v[cuts[j]:cuts[j + 1]], width))
    return b"".join(parts)


_BASE = {}


def _genome_fasta(args) -> bytes:
    """One genome of pangenome() as FASTA bytes (a pool worker; the base
    genome is made once per worker)."""
    gi, genome_len, snp, indel, seed, width = args
    key = (genome_len, seed)
    if key not in _BASE:
        _BASE.clear()
        _BASE[key] = base_genome(genome_len, seed)
    return to_fasta_lines(b"g%d" % gi, variant(_BASE[key], gi, snp, indel, seed), width)


def write_pangenome(path: str, n_genomes: int, genome_len: int, snp: float = 1e-3, indel: float = 1e-4,
                    seed: int = DEFAULT_SEED, first_index: int = 0, width: int = 60, workers: int = 8,
                    progress=None) -> int:
    """pangenome(...) (one record per genome) streamed to `path` by a pool of
    `workers` spawned processes, genome by genome in order, so inputs of
    several GB (C4: 5.08 GB) are never held whole.  Byte-identical to
    pangenome(...).  Returns the bytes written."""
    import multiprocessing
    jobs = [(gi, genome_len, snp, indel, seed, width) for gi in range(first_index, first_index + n_genomes)]
    n = 0
    with open(path, "wb") as f:
        if workers <= 1:
            it = map(_genome_fasta, jobs)
            pool = None
        else:
            # spawn: the caller may already hold a GPU context, which a forked child must not inherit
            pool = multiprocessing.get_context("spawn").Pool(workers)
            it = pool.imap(_genome_fasta, jobs, chunksize=2)
        try:
            for i, b in enumerate(it):
                f.write(b)
                n += len(b)
                if progress and (i + 1) % 100 == 0:
                    progress(i + 1, n)
        finally:
            if pool is not None:
                pool.close()
                pool.join()
    return n


# Named workloads of BASELINE.json "configs" (SURVEY.md §8(d) table).
CONFIGS = {
    # C2: synthetic stand-in for E. coli K-12 MG1655 (4,641,652 bp) with 7 inserted
    # 5 kb repeat copies (rRNA-operon-like).
    "c2": dict(kind="ecoli", genome_len=4_641_652),
    # C3: 100 x 5 Mbp variants, 0.1% SNP, 0.01% indels -> 0.5 Gbp.
    "c3": dict(kind="pan", n_genomes=100, genome_len=5_000_000, snp=1e-3, indel=1e-4),
    # C4: 1000 x 5 Mbp (5 Gbp), sharded 125 genomes per GPU at 8 GPUs.
    "c4": dict(kind="pan", n_genomes=1000, genome_len=5_000_000, snp=1e-3, indel=1e-4),
    # C5: 10 x 3 Gbp variants, 1% SNP, 0.1% indels, each genome split into 24
    # records of 125 Mbp (30 Gbp, 240 records): generated record by record
    # (c5_record / write_c5), never held whole.
    "c5": dict(kind="pan_records", n_genomes=10, records=24, record_len=125_000_000, snp=1e-2, indel=1e-3),
}


def c5_record(genome: int, record: int, record_len: int = 125_000_000, snp: float = 1e-2,
              indel: float = 1e-3, seed: int = DEFAULT_SEED) -> bytes:
    """Record `record` of genome `genome` of C5: a variant of base segment
    `record` (each 125 Mbp segment of the 3 Gbp base genome has its own
    splitmix64 stream, so any record is generated alone in ~1 GB of memory)."""
    base = base_genome(record_len, seed ^ (0xC5 << 40) ^ (record * 0x100000001B3))
    v = variant(base, genome, snp, indel, seed ^ (0xC5C5 << 32) ^ record)
    return to_fasta_lines(b"g%d_c%d" % (genome, record), v)


def _c5_job(args) -> bytes:
    g, r, record_len = args
    return c5_record(g, r, record_len)


def write_c5(path: str, n_genomes: int = 10, records: int = 24, record_len: int = 125_000_000,
             genomes=None, pairs=None, workers: int = 1) -> int:
    """Stream C5 (or the genomes listed, or the (genome, record) pairs listed,
    in that order) to `path` through `workers` spawned processes (~5 GB of
    memory each at 125 Mbp); returns the bytes written."""
    if pairs is None:
        pairs = [(g, r) for g in (range(n_genomes) if genomes is None else genomes) for r in range(records)]
    jobs = [(g, r, record_len) for g, r in pairs]
    n = 0
    with open(path, "wb") as f:
        if workers <= 1:
            it, pool = map(_c5_job, jobs), None
        else:
            import multiprocessing
            pool = multiprocessing.get_context("spawn").Pool(workers)
            it = pool.imap(_c5_job, jobs)
        try:
            for b in it:
                f.write(b)
                n += len(b)
        finally:
            if pool is not None:
                pool.close()
                pool.join()
    return n


def ecoli_like(length: int = 4_641_652, seed: int = DEFAULT_SEED, repeats: int = 7,
               repeat_len: int = 5000) -> bytes:
    g = base_genome(length - repeats * repeat_len, seed ^ 0xEC011)
    rep = base_genome(repeat_len, seed ^ 0x5EE7)
    cut = np.linspace(0, g.shape[0], repeats + 2).astype(np.int64)[1:-1]
    parts, prev = [], 0
    for c in cut:
        parts += [g[prev:c], rep]
        prev = c
    parts.append(g[prev:])
    return to_fasta_lines(b"NC_000913.3 synthetic E. coli K-12 MG1655 stand-in", np.concatenate(parts))


if __name__ == "__main__":
    # python -m pangenome_amd.synth c3|c4|popN OUT [workers]: write a workload's FASTA
    import sys
    import time
    name, out = sys.argv[1], sys.argv[2]
    workers = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    n = {"c3": 100, "c4": 1000}.get(name) or int(name[3:]) * 100
    t0 = time.time()
    size = write_pangenome(out, n, 5_000_000, workers=workers,
                           progress=lambda i, b: print("%s: %d genomes, %.2f GB, %.0f s" % (name, i, b / 1e9,
                                                                                            time.time() - t0),
                                                       flush=True))
    print("%s: wrote %d bytes to %s in %.0f s" % (name, size, out, time.time() - t0), flush=True)

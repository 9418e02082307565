"""Benchmark-scale inputs and the digests their parity is checked through
(tests/golden/make_scale_digests.py writes tests/golden/scale/*.json from the
oracle; tests/test_gpu_scale.py and bench.py compare the GPU against them)."""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np

GOLDEN_SCALE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "scale")

# name -> how bench.py / the tests build it (pangenome_amd/synth.py, deterministic)
INPUTS = {
    # C3, batch A: bench.workload("c3", rank 0) — 100 x 5 Mbp, 0.1 % SNP, 0.01 % indel
    "c3a": dict(kind="pan", n=100, length=5_000_000, snp=1e-3, indel=1e-4, first=0, k=27, c=2,
                desc="C3 batch A: genomes 0..99 of the 5 Mbp population"),
    # C3, batch B: the next 100 genomes of the same population (bench alternates A/B)
    "c3b": dict(kind="pan", n=100, length=5_000_000, snp=1e-3, indel=1e-4, first=100, k=27, c=2,
                desc="C3 batch B: genomes 100..199 of the 5 Mbp population"),
    # C2: the synthetic E. coli K-12 stand-in, one 4,641,652 bp record; walked too
    "c2": dict(kind="ecoli", k=27, c=2, walk=True, desc="C2: synthetic E. coli stand-in, 1 record"),
    # C3 batch A through the whole CLI (seq2graph :1853-1951, empty .mcl):
    # -c 2 (edges/labels forward only) and -c 3 (both strands walked)
    "c3a_c2": dict(kind="pan", n=100, length=5_000_000, snp=1e-3, indel=1e-4, first=0, k=27, c=2, walk=True,
                   desc="C3 batch A, whole CLI at -c 2: dBG, rdBG, .xyz, region rows"),
    "c3a_c3": dict(kind="pan", n=100, length=5_000_000, snp=1e-3, indel=1e-4, first=0, k=27, c=3, walk=True,
                   desc="C3 batch A, whole CLI at -c 3: dBG, rdBG, .xyz, region rows"),
    # C4: 1000 x 5 Mbp (5.08 GB of FASTA: past 2^32 bytes), on one GPU
    "c4": dict(kind="pan", n=1000, length=5_000_000, snp=1e-3, indel=1e-4, first=0, k=27, c=2,
               desc="C4: genomes 0..999 of the 5 Mbp population (5 Gbp)"),
    # the global populations of the N-GPU weak-scaling bench (100 genomes per
    # rank; bench.py rotates which rank holds which 100, so one digest per N)
    "pop2": dict(kind="pan", n=200, length=5_000_000, snp=1e-3, indel=1e-4, first=0, k=27, c=2,
                 desc="bench --gpus 2 population: genomes 0..199"),
    "pop4": dict(kind="pan", n=400, length=5_000_000, snp=1e-3, indel=1e-4, first=0, k=27, c=2,
                 desc="bench --gpus 4 population: genomes 0..399"),
    "pop8": dict(kind="pan", n=800, length=5_000_000, snp=1e-3, indel=1e-4, first=0, k=27, c=2,
                 desc="bench --gpus 8 population: genomes 0..799"),
    # C5's form at a size the oracle finishes (125 Mbp records
    # of 3 Gbp genomes, 1 % SNP, 0.1 % indel): records 0-1 of genomes 0-1 in
    # the file's genome-major order (0.5 Gbp; two segments, each twice)
    "c5s": dict(kind="c5", genomes=[0, 1], records=[0, 1], k=27, c=2,
                desc="C5 form: synth.c5_record(g, r) for g in 0-1, r in 0-1 (4 x 125 Mbp, 1 % SNP, 0.1 % indel)"),
    # C5 at the streamed exchange's production chunk (2^30 forward bases): the
    # first 8 records of genome 0 fill one chunk (1.0 Gbp), genome 1's first
    # two (their 1 %-SNP variants) the next; 1.25 Gbp, ~2.3 G dBG keys, too
    # many for one in-memory oakht, so digested by key range (pgo_dbg_range)
    "c5m": dict(kind="c5pairs", pairs=[(0, r) for r in range(8)] + [(1, 0), (1, 1)], k=27, c=2, ranges=32,
                desc="C5 at 2^30-base chunks: synth.c5_record(0, 0..7), then (1, 0..1) (10 x 125 Mbp)"),
    # the C5 shard one rank holds at N = 8 (tests/test_gpu_c5.py): genome 0's
    # 24 records and genome 1's first 6 (3.75 Gbp), digested by key range
    "c5shard": dict(kind="c5pairs", pairs=[(0, r) for r in range(24)] + [(1, r) for r in range(6)], k=27, c=2,
                    ranges=96, desc="C5 shard of rank 0 at N = 8: synth.c5_record(0, 0..23), then (1, 0..5)"),
}


def make_input(name: str) -> bytes:
    from pangenome_amd import synth
    s = INPUTS[name]
    if s["kind"] == "ecoli":
        return synth.ecoli_like()
    if s["kind"] == "c5":
        return b"".join(synth.c5_record(g, r) for g in s["genomes"] for r in s["records"])
    if s["kind"] == "c5pairs":
        return b"".join(synth.c5_record(g, r) for g, r in s["pairs"])
    return synth.pangenome(s["n"], s["length"], snp=s["snp"], indel=s["indel"], first_index=s["first"])


def load_digest(name: str):
    p = os.path.join(GOLDEN_SCALE, name + ".json")
    return json.load(open(p)) if os.path.isfile(p) else None


def dbg_digest(keys_sorted: np.ndarray, masks: np.ndarray) -> str:
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(keys_sorted, dtype="<u8").tobytes())
    h.update(np.ascontiguousarray(masks, dtype="<u2").tobytes())
    return h.hexdigest()


def rdbg_digest(keys_sorted: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(keys_sorted, dtype="<u8").tobytes()).hexdigest()


def text_digest(text) -> str:
    return hashlib.sha256(text.encode() if isinstance(text, str) else text).hexdigest()

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
}


def make_input(name: str) -> bytes:
    from pangenome_amd import synth
    s = INPUTS[name]
    if s["kind"] == "ecoli":
        return synth.ecoli_like()
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

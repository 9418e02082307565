"""Helpers to read the committed golden fixtures (tests/golden/*)."""
import gzip
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def fixture_names():
    return sorted(d for d in os.listdir(GOLDEN)
                  if os.path.isfile(os.path.join(GOLDEN, d, "meta.json")))


class Fixture:
    def __init__(self, name):
        self.name = name
        self.dir = os.path.join(GOLDEN, name)
        self.meta = json.load(open(os.path.join(self.dir, "meta.json")))
        self.input_path = os.path.join(GOLDEN, "inputs", self.meta["input"])
        self.fasta = open(self.input_path, "rb").read()
        g = np.load(os.path.join(GOLDEN, "graphs", self.meta["graph"]))
        self.dbg_keys, self.dbg_masks, self.rdbg_keys = g["dbg_keys"], g["dbg_masks"], g["rdbg_keys"]
        # the reference's own `<in>_db.npz` (:243-261): occurrence counts per key
        # (sorted like dbg_keys) and its parameters row
        self.dbg_counts, self.db_params = g["dbg_counts"], g["db_params"]
        self.xyz = gzip.open(os.path.join(self.dir, "rdbg_weight.xyz.gz")).read().decode()
        self.rows = gzip.open(os.path.join(self.dir, "rows.tsv.gz")).read().decode().split("\n")[:-1]
        mp = os.path.join(self.dir, "input.mcl")
        self.mcl = open(mp).read() if os.path.isfile(mp) else ""
        self.k, self.c = self.meta["k"], self.meta["c"]
        n = self.meta["n"]
        self.ns = int(float(n)) if n is not None else None
        self.edge_chunk = self.meta["chunk"] or 2 ** 33


def resume_names():
    d = os.path.join(GOLDEN, "resume")
    return sorted(x for x in os.listdir(d) if os.path.isfile(os.path.join(d, x, "meta.json"))) \
        if os.path.isdir(d) else []


class ResumeFixture:
    """A checkpoint the reference wrote (brkpt.npz) and its CLI's output when
    resuming from it with -r or -R (tests/golden/make_goldens.py)."""

    def __init__(self, name):
        self.name = name
        self.dir = os.path.join(GOLDEN, "resume", name)
        self.meta = json.load(open(os.path.join(self.dir, "meta.json")))
        self.fasta = open(os.path.join(GOLDEN, "inputs", self.meta["input"]), "rb").read()
        self.brkpt = os.path.join(self.dir, "brkpt.npz")
        self.flag, self.k, self.c = self.meta["flag"], self.meta["k"], self.meta["c"]
        self.xyz = gzip.open(os.path.join(self.dir, "rdbg_weight.xyz.gz")).read().decode()
        self.rows = gzip.open(os.path.join(self.dir, "rows.tsv.gz")).read().decode().split("\n")[:-1]
        self.graph = None
        if "graph" in self.meta:
            g = np.load(os.path.join(GOLDEN, "graphs", self.meta["graph"]))
            self.graph = {k: g[k] for k in ("dbg_keys", "dbg_masks", "dbg_counts")}

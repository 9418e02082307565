"""ctypes front end of the C oracle (pg_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package.  It restates, in a
few lines of Python, the parts of kmer_numba.py that are plain Python in the
reference too: the `.xyz` writer (:1893-1904), the label dictionary built from
the `.mcl` + `.xyz` files (:1918-1944) and the row printer (:1946-1949).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libpg_oracle.so")
NEVER = 2 ** 63
CHUNK = 2 ** 33          # entry_point :2073

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.isfile(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        i64, i32, u8p = C.c_int64, C.c_int, C.POINTER(C.c_uint8)
        L.pgo_build_graph.argtypes = [u8p, i64, i32, i32, i64, i32, i64, C.POINTER(P)]
        L.pgo_edges.argtypes = [P, u8p, i64, i32, i64, i32, i64]
        L.pgo_rows.argtypes = [P, u8p, i64, i32, i64, i32, P, P, P, i64]
        for f in ("pgo_n_dbg", "pgo_n_rdbg", "pgo_n_edges", "pgo_n_rows", "pgo_n_bases", "pgo_n_records"):
            getattr(L, f).argtypes = [P]
            getattr(L, f).restype = i64
        for f in ("pgo_seconds_dbg", "pgo_seconds_rdbg"):
            getattr(L, f).argtypes = [P]
            getattr(L, f).restype = C.c_double
        L.pgo_get_dbg.argtypes = [P, P, P]
        L.pgo_get_rdbg.argtypes = [P, P]
        L.pgo_get_dbg_counts.argtypes = [P, P]
        L.pgo_dbg_capacity.argtypes = [P]
        L.pgo_dbg_capacity.restype = i64
        L.pgo_get_edges.argtypes = [P, P, P]
        L.pgo_get_rows.argtypes = [P, P]
        L.pgo_set_rdbg.argtypes = [P, P, i64]
        L.pgo_free.argtypes = [P]
        _lib = L
    return _lib


def _ns(ns):
    if ns is None or ns >= NEVER:
        return 0, 1
    return int(ns), 0


def _buf(data: bytes):
    arr = np.frombuffer(data, dtype=np.uint8)
    return arr, arr.ctypes.data_as(C.POINTER(C.c_uint8))


class OracleRun:
    """One pass of the reference pipeline over an in-memory FASTA."""

    def __init__(self, fasta: bytes, k: int, c: int = 2, ns=None, dbg_chunk: int = CHUNK):
        self.fasta = fasta
        self.k = min(max(1, k), 27)
        self.c = c
        self.ns = ns
        self._arr, self._ptr = _buf(fasta)
        h = C.c_void_p()
        ns_v, never = _ns(ns)
        rc = lib().pgo_build_graph(self._ptr, len(fasta), k, int((c >> 1) == 1), ns_v, never,
                                   dbg_chunk, C.byref(h))
        if rc != 0:
            raise RuntimeError("pgo_build_graph failed")
        self.h = h

    def __del__(self):
        if getattr(self, "h", None):
            lib().pgo_free(self.h)
            self.h = None

    # --------------------------------------------------------------- graph
    def dbg(self):
        n = lib().pgo_n_dbg(self.h)
        keys = np.empty(n, np.uint64)
        masks = np.empty(n, np.uint16)
        lib().pgo_get_dbg(self.h, keys.ctypes.data, masks.ctypes.data)
        o = np.argsort(keys, kind="stable")
        return keys[o], masks[o]

    def dbg_counts(self):
        """(keys, masks, counts) sorted by key: the oakht's saturating occurrence
        counts (__setitem__ :556), as `<in>_db.npz` stores them."""
        n = lib().pgo_n_dbg(self.h)
        keys = np.empty(n, np.uint64)
        masks = np.empty(n, np.uint16)
        counts = np.empty(n, np.uint8)
        lib().pgo_get_dbg(self.h, keys.ctypes.data, masks.ctypes.data)
        lib().pgo_get_dbg_counts(self.h, counts.ctypes.data)
        o = np.argsort(keys, kind="stable")
        return keys[o], masks[o], counts[o]

    def dbg_capacity(self):
        return int(lib().pgo_dbg_capacity(self.h))

    def rdbg(self):
        n = lib().pgo_n_rdbg(self.h)
        keys = np.empty(n, np.uint64)
        lib().pgo_get_rdbg(self.h, keys.ctypes.data)
        return np.sort(keys)

    def set_rdbg(self, keys):
        """Replace the rdBG key set the edge and row passes query (-D)."""
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        lib().pgo_set_rdbg(self.h, keys.ctypes.data, keys.shape[0])

    def timings(self):
        return lib().pgo_seconds_dbg(self.h), lib().pgo_seconds_rdbg(self.h)

    def n_bases(self):
        return lib().pgo_n_bases(self.h)

    # --------------------------------------------------------------- edges
    def edges(self, chunk: int = CHUNK):
        ns_v, never = _ns(self.ns)
        lib().pgo_edges(self.h, self._ptr, len(self.fasta), int((self.c & 1) == 1), ns_v, never, chunk)
        n = lib().pgo_n_edges(self.h)
        t = np.empty((n, 4), np.uint64)
        cnt = np.empty(n, np.int64)
        lib().pgo_get_edges(self.h, t.ctypes.data, cnt.ctypes.data)
        return t, cnt

    def xyz(self, chunk: int = CHUNK) -> str:
        t, cnt = self.edges(chunk)
        return "".join("%d_%d\t%d_%d\t%d\n" % (a, b, c, d, e)
                       for (a, b, c, d), e in zip(t.tolist(), cnt.tolist()))

    # ---------------------------------------------------------------- rows
    def rows(self, labels):
        keys, vals, ids = labels
        ns_v, never = _ns(self.ns)
        lib().pgo_rows(self.h, self._ptr, len(self.fasta), int((self.c & 1) == 1), ns_v, never,
                       keys.ctypes.data, vals.ctypes.data, ids.ctypes.data, keys.shape[0])
        n = lib().pgo_n_rows(self.h)
        out = np.empty((n, 6), np.int64)
        lib().pgo_get_rows(self.h, out.ctypes.data)
        lines = []
        for hst, hlen, s, e, strand, lab in out.tolist():
            qid = self.fasta[hst:hst + hlen].decode()[1:]
            lines.append("%s\t%d\t%d\t%s\t%d" % (qid, s, e, "+" if strand == 1 else "-", lab))
        return lines


def label_table(xyz_text: str, mcl_text: str):
    """seq2graph :1918-1944: `.mcl` line index, then unseen `.xyz` nodes in order."""
    lab = {}
    flag = 0
    for line in mcl_text.splitlines(keepends=True):
        for tok in line[:-1].split("\t"):
            a = tok.split("_")[:2]
            lab[tuple(map(int, a))] = flag
        flag += 1
    for line in xyz_text.splitlines(keepends=True):
        j, k = line[:-1].split("\t")[:2]
        for t in (j, k):
            key = tuple(map(int, t.split("_")[:2]))
            if key not in lab:
                lab[key] = flag
                flag += 1
    items = list(lab.items())
    keys = np.array([a for (a, _), _ in items], dtype=np.int64)
    vals = np.array([b for (_, b), _ in items], dtype=np.int64)
    ids = np.array([v for _, v in items], dtype=np.int64)
    return keys, vals, ids


def run_pipeline(fasta: bytes, k: int, c: int = 2, ns=None, mcl_text: str = "",
                 edge_chunk: int = CHUNK):
    """Whole reference pipeline with an existing `.mcl` (empty by default)."""
    r = OracleRun(fasta, k, c, ns)
    xyz = r.xyz(edge_chunk)
    rows = r.rows(label_table(xyz, mcl_text))
    dk, dm = r.dbg()
    return dict(dbg_keys=dk, dbg_masks=dm, rdbg_keys=r.rdbg(), xyz=xyz, rows=rows)

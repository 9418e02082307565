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
        L.pgo_dbg_range.argtypes = [u8p, i64, i32, i32, i64, i32, i64, C.c_uint64, C.c_uint64,
                                    C.POINTER(P), C.POINTER(P)]
        L.pgo_dbg_range.restype = i64
        L.pgo_free_buf.argtypes = [P]
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


def dbg_range(fasta, k: int, c: int, lo: int, hi: int, ns=None, dbg_chunk: int = CHUNK):
    """The dBG entries with keys in [lo, hi) (hi = 2**64 - 1 includes the n<k
    sentinel), sorted by key: pgo_dbg_range, the same pass as OracleRun with
    a sort instead of the oakht (inputs too large for one in-memory table are
    digested range by range).  `fasta`: bytes or a uint8 array (np.memmap)."""
    arr = np.frombuffer(fasta, dtype=np.uint8) if not isinstance(fasta, np.ndarray) else fasta
    kp, mp = C.c_void_p(), C.c_void_p()
    ns_v, never = _ns(ns)
    n = lib().pgo_dbg_range(arr.ctypes.data_as(C.POINTER(C.c_uint8)), arr.shape[0], min(max(1, k), 27),
                            int((c >> 1) == 1), ns_v, never, dbg_chunk, lo, hi, C.byref(kp), C.byref(mp))
    if n < 0:
        raise MemoryError("pgo_dbg_range: out of host memory for the range [%d, %d)" % (lo, hi))
    try:
        keys = np.ctypeslib.as_array((C.c_uint64 * n).from_address(kp.value)).copy() if n else np.zeros(0, np.uint64)
        masks = np.ctypeslib.as_array((C.c_uint16 * n).from_address(mp.value)).copy() if n else np.zeros(0, np.uint16)
    finally:
        lib().pgo_free_buf(kp)
        lib().pgo_free_buf(mp)
    return keys, masks


def key_ranges(k: int, parts: int):
    """`parts` consecutive key ranges covering every key of k digits and the
    sentinel: [lo_i, lo_{i+1}), the last one ending at 2**64 - 1."""
    top = 5 ** min(max(1, k), 27)
    b = [top * i // parts for i in range(parts)] + [2 ** 64 - 1]
    return list(zip(b[:-1], b[1:]))


def rdbg_member(masks: np.ndarray) -> np.ndarray:
    """build_rdbg_jit_ :1300-1305: kept unless exactly one predecessor bit and
    one successor bit."""
    pc = np.array([bin(i).count("1") for i in range(64)], np.int8)
    m = masks.astype(np.int64)
    return ~((pc[(m >> 6) & 63] == 1) & (pc[m & 63] == 1))


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

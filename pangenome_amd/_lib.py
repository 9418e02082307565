"""ctypes binding of include/pangenome.h (libpangenome_hip.so).

There is no CPU fallback: if the in-tree HIP library is missing or no HIP
device is usable, every call raises.  Build it with ``python -c "import
__graft_entry__ as g; g.build()"`` (or ``make -C pangenome_amd/csrc``).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, os.environ.get("PG_LIB_NAME", "libpangenome_hip.so"))   # diag builds only

PG_OK = 0
PG_TUNE_K3_CHUNKS = 1
PG_TUNE_BUCKET_SHIFT = 2
PG_TUNE_REGION_CAP = 3
PG_TUNE_H2D_CHUNK = 4
PG_TUNE_HOST_THREADS = 5
PG_TUNE_STAGE_PIECE = 6
PG_TUNE_STAGE_SLOTS = 7
PG_TUNE_HOST_REGISTER = 8
PG_TUNE_DEVICE_CAP = 9          # process-wide: caps (and restarts the peak of) every context's buffers
PG_TUNE_K3_COVER = 10
PG_TUNE_K3_WBLK = 11
PG_TUNE_K3_EMIT = 12
PG_TUNE_K3_TAIL = 13
PG_TUNE_EARLY_SPLIT = 14
PG_TUNE_K3_HEAD = 15
PG_TUNE_H2D_TAIL = 16
PG_TUNE_POISON = 17             # process-wide debug: new device buffers filled with this byte
PG_TUNE_K1 = 18                 # K1 form bits (bit 0 whole-span pass, bit 1 deeper emission prefetch, bit 2 record table ahead of the emission)
PG_TUNE_TIMERS = 19             # bits: HIP timing events of K1 / stage A / stages B-C (default 7)
PG_TUNE_K3_ANCHORS = 20         # packed coverage pass anchors per tile and reference (3-6, 8; 0 = 4)


class PgStats(C.Structure):
    _fields_ = [
        ("n_bytes", C.c_uint64), ("n_records", C.c_uint64), ("n_bases", C.c_uint64),
        ("n_windows", C.c_uint64), ("n_dbg", C.c_uint64), ("n_rdbg", C.c_uint64),
        ("n_slots", C.c_uint64), ("table_capacity", C.c_uint64),
        ("ms_parse", C.c_double), ("ms_clear", C.c_double), ("ms_insert", C.c_double),
        ("ms_scan", C.c_double), ("sentinel", C.c_uint64),
        ("n_records_a", C.c_uint64), ("ms_split", C.c_double), ("ms_range", C.c_double),
        ("build_flags", C.c_uint64), ("n_work_items", C.c_uint64),
    ]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


# every symbol include/pangenome.h declares, with (restype, argtypes)
_P, _U8P, _U64P = C.c_void_p, C.POINTER(C.c_uint8), C.POINTER(C.c_uint64)
_I64P, _U16P = C.POINTER(C.c_int64), C.POINTER(C.c_uint16)
_SP = C.POINTER(PgStats)
SIGNATURES = {
    "pg_create": (C.c_int, [C.POINTER(C.c_void_p), C.c_int, C.c_int]),
    "pg_destroy": (None, [_P]),
    "pg_last_error": (C.c_char_p, []),
    "pg_get_k": (C.c_int, [_P]),
    "pg_stream_wait": (C.c_int, [_P, _P]),
    "pg_set_fasta": (C.c_int, [_P, _P, C.c_uint64]),
    "pg_set_fasta_device": (C.c_int, [_P, _P, C.c_uint64]),
    "pg_parse": (C.c_int, [_P, _U64P, _U64P]),
    "pg_parse_host": (C.c_int, [_P, _P, C.c_uint64, _U64P, _U64P]),
    "pg_records": (C.c_int, [_P, _P, _P, _P, _P]),
    "pg_build_dbg": (C.c_int, [_P, _P, C.c_int, C.c_int, _SP]),
    "pg_build_rdbg": (C.c_int, [_P, _U64P, _SP]),
    "pg_build": (C.c_int, [_P, _P, C.c_int, C.c_int, _U64P, _SP]),
    "pg_build_host": (C.c_int, [_P, _P, C.c_uint64, C.c_int, _U64P, _SP]),
    "pg_build_device": (C.c_int, [_P, _P, C.c_uint64, C.c_int, _U64P, _SP]),
    "pg_dbg_export": (C.c_int, [_P, _P, _P, C.c_uint64, _U64P]),
    "pg_rdbg_export": (C.c_int, [_P, _P, C.c_uint64, _U64P]),
    "pg_dbg_partition": (C.c_int, [_P, C.c_int, _P, C.c_uint64, _P]),
    "pg_dbg_merge": (C.c_int, [_P, _P, C.c_uint64, C.c_uint64, C.c_int]),
    "pg_dbg_partition_sums": (C.c_int, [_P, C.c_int, _P]),
    "pg_rows_checksum": (C.c_int, [_P, _P, _P, C.c_uint64, _P]),
    "pg_dbg_merge_check": (C.c_int, [_P, _U64P, _U64P]),
    "pg_route_stage_a": (C.c_int, [_P, _P, C.c_int, C.c_int, C.c_int, _P, C.POINTER(C.c_int)]),
    "pg_route_scatter": (C.c_int, [_P, C.c_int, _P, C.c_uint64, _P]),
    "pg_route_rows_checksum": (C.c_int, [_P, _P, _P, C.c_uint64, _P]),
    "pg_route_finish": (C.c_int, [_P, _U64P, _SP]),
    "pg_route_merge": (C.c_int, [_P, _P, C.c_uint64, C.c_int, C.c_int, _U64P, _SP]),
    "pg_route_merge_segs": (C.c_int, [_P, C.POINTER(C.c_void_p), _P, C.c_int, C.c_int, C.c_int, _U64P, _SP]),
    "pg_edges": (C.c_int, [_P, _P, C.c_int, _U64P]),
    "pg_edges_export": (C.c_int, [_P, _P, _P, _P, C.c_uint64]),
    "pg_set_labels": (C.c_int, [_P, _P, _P, _P, C.c_uint64]),
    "pg_rows": (C.c_int, [_P, _P, C.c_int, _U64P]),
    "pg_rows_export": (C.c_int, [_P, _P, C.c_uint64]),
    "pg_edges_format": (C.c_int, [_P, _P, C.c_uint64, _U64P]),
    "pg_edges_format_fd": (C.c_int, [_P, C.c_int, _U64P]),
    "pg_labels_from_edges": (C.c_int, [_P, _P, C.c_uint64, _P, _P, _P, C.c_uint64, C.c_int64, _U64P]),
    "pg_labels_export": (C.c_int, [_P, _P, _P, _P, C.c_uint64]),
    "pg_rows_format": (C.c_int, [_P, _P, _P, C.c_uint64, _P, C.c_uint64, _U64P]),
    "pg_rows_format_fd": (C.c_int, [_P, _P, _P, C.c_uint64, C.c_int, _U64P]),
    "pg_get_stats": (C.c_int, [_P, _SP]),
    "pg_tune": (C.c_int, [_P, C.c_int, C.c_int64]),
    "pg_dbg_dump": (C.c_int, [_P, _U64P, _P, _P, _P, _U64P]),
    "pg_dbg_dump_fd": (C.c_int, [_P, _U64P, C.c_int, _P, _P, _U64P]),
    "pg_dbg_load": (C.c_int, [_P, _P, _P, _P, C.c_uint64]),
    "pg_oakht_capacity": (C.c_uint64, [C.c_uint64]),
    "pg_device_bytes": (C.c_uint64, [C.c_int]),
    "pg_format_xyz": (C.c_uint64, [_P, _P, C.c_uint64, _P, C.c_uint64]),
    "pg_format_rows": (C.c_uint64, [_P, C.c_uint64, _P, _P, _P, C.c_uint64]),
}

_lib = None


class PangenomeError(RuntimeError):
    pass


def load():
    """Load the in-tree HIP library (raises if it is not built)."""
    global _lib
    if _lib is None:
        if not os.path.isfile(LIB_PATH):
            raise ImportError(
                "libpangenome_hip.so is not built (%s); run __graft_entry__.build() "
                "or `make -C pangenome_amd/csrc` — there is no CPU fallback" % LIB_PATH)
        # One HIP runtime per process: torch ships its own libamdhip64.so.7
        # (same SONAME as /opt/rocm's).  Whichever loads first serves both, and
        # torch's build refuses the system one, so let torch load it first;
        # device buffers from torch (bench, multi-GPU exchange) then share it.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        lib = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def check(rc: int, what: str):
    if rc != PG_OK:
        msg = load().pg_last_error()
        raise PangenomeError("%s failed (%d): %s" % (what, rc, msg.decode() if msg else "?"))


def ptr(a: np.ndarray | None):
    return None if a is None else C.c_void_p(a.ctypes.data)


def _names_blob(names: list):
    """Record names as pg_rows_format takes them: one byte blob and R + 1
    offsets."""
    blob = b"".join(names)
    off = np.zeros(len(names) + 1, np.int64)
    if names:
        off[1:] = np.cumsum([len(x) for x in names])
    return (np.frombuffer(blob, np.uint8) if blob else np.zeros(1, np.uint8)), off


class Context:
    """One pg_ctx: one HIP device, one stream, all device buffers."""

    def __init__(self, k: int, device: int = 0):
        self.lib = load()
        h = C.c_void_p()
        check(self.lib.pg_create(C.byref(h), device, k), "pg_create")
        self.h = h
        self.k = self.lib.pg_get_k(h)
        self.n_records = 0
        self.n_bases = 0
        self._keepalive = None

    def close(self):
        if getattr(self, "h", None):
            self.lib.pg_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -------------------------------------------------------------- input
    def set_fasta(self, data):
        """Host bytes (bytes / bytearray / np.uint8 array / mmap)."""
        arr = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data
        check(self.lib.pg_set_fasta(self.h, ptr(arr), arr.shape[0]), "pg_set_fasta")

    def set_fasta_host_ptr(self, host_ptr: int, nbytes: int):
        """Host bytes at a raw address (e.g. a pinned torch tensor's data_ptr():
        the H2D copy is then plain DMA)."""
        check(self.lib.pg_set_fasta(self.h, C.c_void_p(host_ptr), nbytes), "pg_set_fasta")

    def set_fasta_device(self, dev_ptr: int, nbytes: int, keepalive=None):
        self._keepalive = keepalive
        check(self.lib.pg_set_fasta_device(self.h, C.c_void_p(dev_ptr), nbytes), "pg_set_fasta_device")

    def parse(self):
        nr, nb = C.c_uint64(), C.c_uint64()
        check(self.lib.pg_parse(self.h, C.byref(nr), C.byref(nb)), "pg_parse")
        self.n_records, self.n_bases = nr.value, nb.value
        return self.n_records, self.n_bases

    def parse_host(self, data):
        """set_fasta + parse of host bytes in one call: chunked H2D pipelined
        with K1 (pg_parse_host)."""
        arr = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data
        return self.parse_host_ptr(arr.ctypes.data if arr.shape[0] else None, arr.shape[0])

    def parse_host_ptr(self, host_ptr, nbytes: int):
        """parse_host from a raw address (e.g. a pinned torch tensor's data_ptr())."""
        nr, nb = C.c_uint64(), C.c_uint64()
        check(self.lib.pg_parse_host(self.h, C.c_void_p(host_ptr), nbytes, C.byref(nr), C.byref(nb)),
              "pg_parse_host")
        self.n_records, self.n_bases = nr.value, nb.value
        return self.n_records, self.n_bases

    def records(self):
        R = self.n_records
        out = [np.empty(R, np.int64) for _ in range(4)]
        check(self.lib.pg_records(self.h, *[ptr(a) for a in out]), "pg_records")
        return dict(seq_len=out[0], hdr_start=out[1], hdr_len=out[2], ptr=out[3])

    # ---------------------------------------------------------------- dBG
    def build_dbg(self, rec_flags=None, extra_empty: int = 0, rc0: bool = True) -> PgStats:
        st = PgStats()
        f = None if rec_flags is None else np.ascontiguousarray(rec_flags, dtype=np.uint8)
        check(self.lib.pg_build_dbg(self.h, ptr(f), int(extra_empty), int(bool(rc0)), C.byref(st)),
              "pg_build_dbg")
        return st

    def build_rdbg(self) -> PgStats:
        st = PgStats()
        n = C.c_uint64()
        check(self.lib.pg_build_rdbg(self.h, C.byref(n), C.byref(st)), "pg_build_rdbg")
        return st

    def build(self, rec_flags=None, extra_empty: int = 0, rc0: bool = True) -> PgStats:
        """build_dbg + build_rdbg in one call (pg_build: K5 runs right behind K3)."""
        st = PgStats()
        n = C.c_uint64()
        f = None if rec_flags is None else np.ascontiguousarray(rec_flags, dtype=np.uint8)
        check(self.lib.pg_build(self.h, ptr(f), int(extra_empty), int(bool(rc0)), C.byref(n), C.byref(st)),
              "pg_build")
        return st

    def build_host(self, data, rc0: bool = True) -> PgStats:
        """parse + build of every record from host bytes with stage A streamed
        under the chunked upload (pg_build_host); the record table is
        available afterwards (records())."""
        arr = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data
        return self.build_host_ptr(arr.ctypes.data if arr.shape[0] else None, arr.shape[0], rc0)

    def build_host_ptr(self, host_ptr, nbytes: int, rc0: bool = True) -> PgStats:
        st = PgStats()
        n = C.c_uint64()
        check(self.lib.pg_build_host(self.h, C.c_void_p(host_ptr), nbytes, int(bool(rc0)), C.byref(n), C.byref(st)),
              "pg_build_host")
        self.n_records, self.n_bases = st.n_records, st.n_bases
        return st

    def build_device(self, dev_ptr: int, nbytes: int, rc0: bool = True, keepalive=None) -> PgStats:
        """set_fasta_device + parse + build of every record in one call
        (pg_build_device) for a FASTA already in HBM."""
        st = PgStats()
        n = C.c_uint64()
        self._keepalive = keepalive
        check(self.lib.pg_build_device(self.h, C.c_void_p(dev_ptr), nbytes, int(bool(rc0)), C.byref(n),
                                       C.byref(st)), "pg_build_device")
        self.n_records, self.n_bases = st.n_records, st.n_bases
        return st

    def stream_wait(self, stream_handle: int):
        """This context's streams wait (on the device) for the work queued so
        far on the HIP stream `stream_handle` (e.g. torch's current stream's
        .cuda_stream): pg_stream_wait."""
        check(self.lib.pg_stream_wait(self.h, C.c_void_p(stream_handle) if stream_handle else None),
              "pg_stream_wait")

    def tune(self, what: int, value: int):
        check(self.lib.pg_tune(self.h, int(what), int(value)), "pg_tune")

    def stats(self) -> PgStats:
        st = PgStats()
        check(self.lib.pg_get_stats(self.h, C.byref(st)), "pg_get_stats")
        return st

    def dbg(self):
        n = C.c_uint64()
        check(self.lib.pg_dbg_export(self.h, None, None, 0, C.byref(n)), "pg_dbg_export")
        keys = np.empty(n.value, np.uint64)
        masks = np.empty(n.value, np.uint16)
        check(self.lib.pg_dbg_export(self.h, ptr(keys), ptr(masks), n.value, C.byref(n)), "pg_dbg_export")
        return keys, masks                        # (sorted by key on the device)

    def rdbg(self):
        n = C.c_uint64()
        check(self.lib.pg_rdbg_export(self.h, None, 0, C.byref(n)), "pg_rdbg_export")
        keys = np.empty(n.value, np.uint64)
        check(self.lib.pg_rdbg_export(self.h, ptr(keys), n.value, C.byref(n)), "pg_rdbg_export")
        return keys                               # (sorted on the device)

    # ----------------------------------------------------- npz persistence
    def dbg_dump(self, capacity: int = 0):
        """The last build's dBG as oakht slot arrays (dump(), :243-261):
        (capacity, size, keys, values, counts)."""
        cap, size = C.c_uint64(capacity), C.c_uint64()
        check(self.lib.pg_dbg_dump(self.h, C.byref(cap), None, None, None, C.byref(size)), "pg_dbg_dump")
        keys = np.empty(cap.value, np.uint64)
        values = np.empty(cap.value, np.uint16)
        counts = np.empty(cap.value, np.uint8)
        check(self.lib.pg_dbg_dump(self.h, C.byref(cap), ptr(keys), ptr(values), ptr(counts), C.byref(size)),
              "pg_dbg_dump")
        return cap.value, size.value, keys, values, counts

    def dbg_dump_size(self, capacity: int = 0):
        """(capacity, size) of dbg_dump without placing or copying anything."""
        cap, size = C.c_uint64(capacity), C.c_uint64()
        check(self.lib.pg_dbg_dump_fd(self.h, C.byref(cap), -1, None, None, C.byref(size)), "pg_dbg_dump_fd")
        return cap.value, size.value

    def dbg_dump_fd(self, fd: int, offsets, capacity: int):
        """The slot arrays of dbg_dump(capacity) written into the open file
        `fd` at offsets[0..2] (keys, values, counts); their CRC-32s."""
        cap, size = C.c_uint64(capacity), C.c_uint64()
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        crc = np.zeros(3, np.uint32)
        check(self.lib.pg_dbg_dump_fd(self.h, C.byref(cap), int(fd), ptr(off), ptr(crc), C.byref(size)),
              "pg_dbg_dump_fd")
        return [int(x) for x in crc]

    def dbg_load(self, keys, masks=None, counts=None):
        """Stage oriented (key, mask, count) slots for the following builds."""
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        m = None if masks is None else np.ascontiguousarray(masks, dtype=np.uint16)
        c = None if counts is None else np.ascontiguousarray(counts, dtype=np.uint8)
        check(self.lib.pg_dbg_load(self.h, ptr(keys), ptr(m), ptr(c), keys.shape[0]), "pg_dbg_load")

    # ------------------------------------------------------ multi-GPU hooks
    def partition(self, nparts: int, d_out: int | None = None, out_cap: int = 0):
        counts = np.zeros(nparts, np.uint64)
        check(self.lib.pg_dbg_partition(self.h, nparts, None if d_out is None else C.c_void_p(d_out),
                                        out_cap, ptr(counts)), "pg_dbg_partition")
        return counts

    def merge(self, d_records: int, n: int, capacity_hint: int = 0, sentinel: bool = False):
        check(self.lib.pg_dbg_merge(self.h, C.c_void_p(d_records) if n else None, n, capacity_hint,
                                    int(bool(sentinel))), "pg_dbg_merge")

    def partition_sums(self, nparts: int):
        """row_check sums of the last partition scatter's runs (uint64[nparts])."""
        sums = np.zeros(nparts, np.uint64)
        check(self.lib.pg_dbg_partition_sums(self.h, nparts, ptr(sums)), "pg_dbg_partition_sums")
        return sums

    def rows_checksum(self, d_rows: int, seg_off):
        """row_check sums of segments [seg_off[s], seg_off[s+1]) of the 16-byte
        records at device address d_rows (uint64[len(seg_off) - 1])."""
        off = np.ascontiguousarray(seg_off, dtype=np.uint64)
        sums = np.zeros(max(off.shape[0] - 1, 1), np.uint64)
        check(self.lib.pg_rows_checksum(self.h, C.c_void_p(d_rows) if d_rows else None, ptr(off),
                                        max(off.shape[0] - 1, 0), ptr(sums)), "pg_rows_checksum")
        return sums[:max(off.shape[0] - 1, 0)]

    def route_rows_checksum(self, d_rows: int, seg_off):
        """rows_checksum over 12-byte routed rows (pg_route_scatter's layout)."""
        off = np.ascontiguousarray(seg_off, dtype=np.uint64)
        sums = np.zeros(max(off.shape[0] - 1, 1), np.uint64)
        check(self.lib.pg_route_rows_checksum(self.h, C.c_void_p(d_rows) if d_rows else None, ptr(off),
                                              max(off.shape[0] - 1, 0), ptr(sums)), "pg_route_rows_checksum")
        return sums[:max(off.shape[0] - 1, 0)]

    def merge_check(self):
        """(non-empty records, row_check sum) the last merge read."""
        rows, s = C.c_uint64(), C.c_uint64()
        check(self.lib.pg_dbg_merge_check(self.h, C.byref(rows), C.byref(s)), "pg_dbg_merge_check")
        return rows.value, s.value

    # ---------------------------------------------------- routed exchange
    def route_stage_a(self, rec_flags=None, extra_empty: int = 0, rc0: bool = True, nparts: int = 1):
        """Stage A of the build, held for its owners: (records per owner as
        uint64[nparts], whether the n<k sentinel was seen)."""
        counts = np.zeros(nparts, np.uint64)
        sent = C.c_int(0)
        f = None if rec_flags is None else np.ascontiguousarray(rec_flags, dtype=np.uint8)
        check(self.lib.pg_route_stage_a(self.h, ptr(f), int(extra_empty), int(bool(rc0)), int(nparts), ptr(counts),
                                        C.byref(sent)), "pg_route_stage_a")
        return counts, bool(sent.value)

    def route_scatter(self, nparts: int, d_out: int, out_cap: int):
        """The held records as 12-byte rows grouped by owner at d_out; their
        integrity sums per owner (uint64[nparts])."""
        sums = np.zeros(nparts, np.uint64)
        check(self.lib.pg_route_scatter(self.h, int(nparts), C.c_void_p(d_out) if d_out else None, int(out_cap),
                                        ptr(sums)), "pg_route_scatter")
        return sums

    def route_finish(self) -> PgStats:
        st = PgStats()
        n = C.c_uint64()
        check(self.lib.pg_route_finish(self.h, C.byref(n), C.byref(st)), "pg_route_finish")
        return st

    def route_merge(self, d_rows: int, n: int, nparts: int, sentinel: bool = False) -> PgStats:
        st = PgStats()
        nr = C.c_uint64()
        check(self.lib.pg_route_merge(self.h, C.c_void_p(d_rows) if n else None, int(n), int(nparts),
                                      int(bool(sentinel)), C.byref(nr), C.byref(st)), "pg_route_merge")
        return st

    def route_merge_segs(self, segs, nparts: int, sentinel: bool = False) -> PgStats:
        """route_merge over several runs of rows [(device pointer, rows), ...]
        merged as one owner table (pg_route_merge_segs)."""
        st = PgStats()
        nr = C.c_uint64()
        m = len(segs)
        ptrs = (C.c_void_p * max(m, 1))(*[C.c_void_p(p) if n else None for p, n in segs])
        ns = np.ascontiguousarray([int(n) for _, n in segs] or [0], dtype=np.uint64)
        check(self.lib.pg_route_merge_segs(self.h, ptrs, ptr(ns), m, int(nparts), int(bool(sentinel)), C.byref(nr),
                                           C.byref(st)), "pg_route_merge_segs")
        return st

    # -------------------------------------------------------------- walks
    def edges_count(self, rec_flags=None, rc1: bool = False) -> int:
        """pg_edges only: the edges stay on the device (edges_text /
        labels_from_edges / edges_export)."""
        n = C.c_uint64()
        f = None if rec_flags is None else np.ascontiguousarray(rec_flags, dtype=np.uint8)
        check(self.lib.pg_edges(self.h, ptr(f), int(bool(rc1)), C.byref(n)), "pg_edges")
        self.n_edges = n.value
        return n.value

    def edges_export(self):
        m = getattr(self, "n_edges", 0)
        t = np.empty((m, 4), np.uint64)
        cnt = np.empty(m, np.int64)
        walk = np.empty(m, np.int64)
        if m:
            check(self.lib.pg_edges_export(self.h, ptr(t), ptr(cnt), ptr(walk), m), "pg_edges_export")
        return t, cnt, walk

    def edges(self, rec_flags=None, rc1: bool = False):
        n = C.c_uint64()
        f = None if rec_flags is None else np.ascontiguousarray(rec_flags, dtype=np.uint8)
        check(self.lib.pg_edges(self.h, ptr(f), int(bool(rc1)), C.byref(n)), "pg_edges")
        m = n.value
        t = np.empty((m, 4), np.uint64)
        cnt = np.empty(m, np.int64)
        walk = np.empty(m, np.int64)
        if m:
            check(self.lib.pg_edges_export(self.h, ptr(t), ptr(cnt), ptr(walk), m), "pg_edges_export")
        return t, cnt, walk

    def edges_text(self) -> bytes:
        """The `.xyz` text of the last edges() pass (first-occurrence order),
        formatted on the device (pg_edges_format)."""
        n = C.c_uint64()
        check(self.lib.pg_edges_format(self.h, None, 0, C.byref(n)), "pg_edges_format")
        buf = np.empty(max(n.value, 1), np.uint8)
        check(self.lib.pg_edges_format(self.h, ptr(buf), buf.shape[0], C.byref(n)), "pg_edges_format")
        return buf[:n.value].tobytes()

    def edges_write(self, fd: int) -> int:
        """edges_text() written straight to descriptor fd at its position
        (pg_edges_format_fd: pinned pieces, parallel pwrite into a regular
        file); flush any buffered writer on fd first.  Returns the bytes."""
        n = C.c_uint64()
        check(self.lib.pg_edges_format_fd(self.h, int(fd), C.byref(n)), "pg_edges_format_fd")
        return n.value

    def labels_from_edges(self, tuples=None, mcl_keys=None, mcl_vals=None, mcl_ids=None, next_label: int = 0):
        """seq2graph's label table on the device (pg_labels_from_edges): the
        .mcl entries, then the .xyz nodes in first-appearance order.  tuples
        None: the last edges() pass."""
        n = C.c_uint64()
        t = None if tuples is None else np.ascontiguousarray(tuples, dtype=np.uint64).reshape(-1, 4)
        mk = np.ascontiguousarray(mcl_keys if mcl_keys is not None else np.zeros(0), dtype=np.int64)
        mv = np.ascontiguousarray(mcl_vals if mcl_vals is not None else np.zeros(0), dtype=np.int64)
        mi = np.ascontiguousarray(mcl_ids if mcl_ids is not None else np.zeros(0), dtype=np.int64)
        check(self.lib.pg_labels_from_edges(self.h, ptr(t), 0 if t is None else t.shape[0], ptr(mk), ptr(mv),
                                            ptr(mi), mk.shape[0], int(next_label), C.byref(n)),
              "pg_labels_from_edges")
        self.n_labels = n.value
        self.label_gen = getattr(self, "label_gen", 0) + 1
        return n.value

    def labels(self, gen=None):
        """(keys, vals, ids) of the device label table, in insertion order.
        `gen`: the label_gen a caller's view was made at; a later label pass
        (set_labels / labels_from_edges) on this context replaced that table,
        and reading it then raises instead of returning the newer labels."""
        if gen is not None and gen != getattr(self, "label_gen", 0):
            raise RuntimeError("label table: replaced by a later label pass on this context (generation %d, now %d)"
                               % (gen, getattr(self, "label_gen", 0)))
        n = getattr(self, "n_labels", 0)
        out = [np.empty(n, np.int64) for _ in range(3)]
        if n:
            check(self.lib.pg_labels_export(self.h, *[ptr(a) for a in out], n), "pg_labels_export")
        return tuple(out)

    def set_labels(self, keys, vals, ids):
        keys = np.ascontiguousarray(keys, np.int64)
        vals = np.ascontiguousarray(vals, np.int64)
        ids = np.ascontiguousarray(ids, np.int64)
        check(self.lib.pg_set_labels(self.h, ptr(keys), ptr(vals), ptr(ids), keys.shape[0]), "pg_set_labels")
        self.n_labels = keys.shape[0]
        self.label_gen = getattr(self, "label_gen", 0) + 1

    def rows_count(self, rec_flags=None, rc1: bool = False) -> int:
        """pg_rows only: the rows stay on the device (rows_text / rows())."""
        n = C.c_uint64()
        f = None if rec_flags is None else np.ascontiguousarray(rec_flags, dtype=np.uint8)
        check(self.lib.pg_rows(self.h, ptr(f), int(bool(rc1)), C.byref(n)), "pg_rows")
        return n.value

    def rows_text(self, names: list) -> bytes:
        """The region rows' text of the last pg_rows, formatted on the device
        (pg_rows_format); names[r] = record r's qid."""
        nb, off = _names_blob(names)
        n = C.c_uint64()
        check(self.lib.pg_rows_format(self.h, ptr(nb), ptr(off), len(names), None, 0, C.byref(n)), "pg_rows_format")
        buf = np.empty(max(n.value, 1), np.uint8)
        check(self.lib.pg_rows_format(self.h, ptr(nb), ptr(off), len(names), ptr(buf), buf.shape[0], C.byref(n)),
              "pg_rows_format")
        return buf[:n.value].tobytes()

    def rows_write(self, names: list, fd: int) -> int:
        """rows_text(names) written straight to descriptor fd at its position
        (pg_rows_format_fd); flush any buffered writer on fd first."""
        nb, off = _names_blob(names)
        n = C.c_uint64()
        check(self.lib.pg_rows_format_fd(self.h, ptr(nb), ptr(off), len(names), int(fd), C.byref(n)),
              "pg_rows_format_fd")
        return n.value

    def rows(self, rec_flags=None, rc1: bool = False):
        n = C.c_uint64()
        f = None if rec_flags is None else np.ascontiguousarray(rec_flags, dtype=np.uint8)
        check(self.lib.pg_rows(self.h, ptr(f), int(bool(rc1)), C.byref(n)), "pg_rows")
        out = np.empty((n.value, 5), np.int64)
        if n.value:
            check(self.lib.pg_rows_export(self.h, ptr(out), n.value), "pg_rows_export")
        return out


# ------------------------------------------------------------------ text output
def format_xyz(tuples: np.ndarray, counts: np.ndarray) -> bytes:
    """The `.xyz` side file's text (kmer_numba.py:1901), formatted natively."""
    lib = load()
    t = np.ascontiguousarray(tuples, dtype=np.uint64)
    c = np.ascontiguousarray(counts, dtype=np.int64)
    n = c.shape[0]
    cap = lib.pg_format_xyz(None, None, n, None, 0)
    buf = np.empty(max(cap, 1), np.uint8)
    m = lib.pg_format_xyz(ptr(t), ptr(c), n, ptr(buf), cap)
    if n and not m:
        raise PangenomeError("pg_format_xyz: buffer too small")
    return buf[:m].tobytes()


def format_rows(rows: np.ndarray, names: list) -> bytes:
    """The region rows (:1947-1949) for records named names[r], natively."""
    lib = load()
    r5 = np.ascontiguousarray(rows, dtype=np.int64).reshape(-1, 5)
    blob = b"".join(names)
    off = np.zeros(len(names) + 1, np.int64)
    if names:
        off[1:] = np.cumsum([len(x) for x in names])
    nb = np.frombuffer(blob, np.uint8) if blob else np.zeros(1, np.uint8)
    n = r5.shape[0]
    cap = lib.pg_format_rows(ptr(r5), n, ptr(nb), ptr(off), None, 0)
    buf = np.empty(max(cap, 1), np.uint8)
    m = lib.pg_format_rows(ptr(r5), n, ptr(nb), ptr(off), ptr(buf), cap)
    if n and not m:
        raise PangenomeError("pg_format_rows: buffer too small")
    return buf[:m].tobytes()

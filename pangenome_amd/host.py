"""Host-side logic of the drop-in: which records each pass visits, the label
dictionary, the `.xyz` text and the printed rows.

The device does every per-base step; what stays here is what is plain Python
(or loop control) in the reference too:

* the record loops of the three passes with their `-n` limit, their
  2**33-base checkpoints and what resuming from a checkpoint does
  (seq2rdbg :1251-1266 + seq2dbg_jit_ :1204-1230; seq2graph :1876-1890 +
  rdbg_edge_weight_jit_ :1809-1827; seqs2path_jit_ :1831-1849);
* the `.xyz` writer (:1893-1904), the label dictionary (:1918-1944) and the
  row printer (:1946-1949).
"""
from __future__ import annotations

import ast
import io
import operator
import os

import numpy as np

CHUNK = 2 ** 33          # entry_point :2073
NEVER = 2 ** 63


# ------------------------------------------------------------------ -n parsing
_OPS = {ast.Add: operator.add, ast.Sub: operator.sub, ast.Mult: operator.mul,
        ast.Div: operator.truediv, ast.Pow: operator.pow, ast.FloorDiv: operator.floordiv,
        ast.USub: operator.neg, ast.UAdd: operator.pos}


def eval_number(text: str) -> int:
    """``int(eval(args['-n']))`` (:1997) for the numeric expressions it is given
    ('5e8', '2**63', '10**9'), without evaluating arbitrary code."""
    def ev(node):
        if isinstance(node, ast.Expression):
            return ev(node.body)
        if isinstance(node, ast.Constant) and isinstance(node.value, (int, float)):
            return node.value
        if isinstance(node, ast.BinOp) and type(node.op) in _OPS:
            return _OPS[type(node.op)](ev(node.left), ev(node.right))
        if isinstance(node, ast.UnaryOp) and type(node.op) in _OPS:
            return _OPS[type(node.op)](ev(node.operand))
        raise ValueError("unsupported -n expression: %r" % text)
    return int(ev(ast.parse(text, mode="eval")))


def ns_hit(N: int, Ns: int) -> bool:
    # numba compares int64 N with Ns; Ns >= 2**63 arrives as uint64 and the
    # mixed comparison never succeeds
    return Ns < NEVER and N > Ns


# ----------------------------------------------------------------- pass plans
class FileShape:
    """What the pass planner needs to know about the FASTA beyond the records."""

    def __init__(self, first_byte: int, last_line_has_nl: bool, first_header_at: int,
                 record_header_is_last_unterminated: bool):
        self.first_byte = first_byte
        self.last_line_has_nl = last_line_has_nl
        self.first_header_at = first_header_at            # byte offset of record 0's header
        self.last_header_unterminated = record_header_is_last_unterminated

    @classmethod
    def from_bytes(cls, buf, hdr_start: np.ndarray, hdr_len: np.ndarray):
        n = len(buf)
        first = buf[0] if n else -1
        last_nl = n > 0 and buf[n - 1] == 10
        R = hdr_start.shape[0]
        fh = int(hdr_start[0]) if R else -1
        # the last record's header is the file's final, newline-less line
        lhu = bool(R) and int(hdr_start[-1] + hdr_len[-1]) >= n - 1 and not last_nl
        return cls(first, last_nl, fh, lhu)


def _resumed_records(pos: int, R: int, shape: FileShape):
    """Records one seqio_jit_ call yields when restarted at the `ptr` of record
    pos-1 (:1240, :1860): readline_jit_ starts its first line at byte 0, so
    that line is the file's prefix up to the end of record pos's header line.
    If the file does not start with '>', that prefix is a sequence line, qid
    is never set and record pos is lost; when record pos-1 was the last one the
    prefix runs to EOF and, starting with '>', yields one extra empty record.
    A first line without '\\n' is never yielded (`end > start > 0`)."""
    if pos < R:
        if pos == R - 1 and shape.last_header_unterminated:
            return []                                  # no '\n' after ptr: nothing at all
        lost = shape.first_byte != ord(">")
        return list(range(pos + (1 if lost else 0), R))
    if shape.last_line_has_nl and shape.first_byte == ord(">"):
        return ["extra"]
    return []


def plan_dbg(seq_len: np.ndarray, shape: FileShape, rc0: bool, Ns: int, chunk: int = CHUNK,
             resume: int | None = None, checkpoint: bool = False):
    """seq2rdbg (:1251-1266) over seq2dbg_jit_ (:1204-1230): which records the
    dBG pass inserts, and how many extra empty records it meets.  `resume`
    is the record a -r checkpoint restarts at (resume_position).  With
    `checkpoint`, also the state of the last `<in>_db_brkpt.npz` dump
    (:1255-1259; each dump overwrites the previous one): (flags, extra,
    record) of the records inserted when it was written and the record whose
    seqio ptr is its offset - or None when no pass crossed `chunk`."""
    R = seq_len.shape[0]
    flags = np.zeros(R, np.uint8)
    extra = 0
    ckpt = None
    mult = 2 if rc0 else 1
    recs = list(range(R)) if not resume else _resumed_records(resume, R, shape)
    N = 0
    while True:
        Nl = chk = 0
        done, last = 1, None
        for r in recs:
            n = 0 if r == "extra" else int(seq_len[r])
            if r == "extra":
                extra += 1
            else:
                flags[r] = 1
            Nl += n * mult
            chk += n * mult
            if chk > chunk:
                done, last = -1, r
                break
            if ns_hit(Nl, Ns):
                break
        if done != -1:
            break
        ckpt = (flags.copy(), extra, last)
        recs = _resumed_records(last + 1, R, shape)
        N += Nl
        if ns_hit(N, Ns):
            break
    return (flags, extra, ckpt) if checkpoint else (flags, extra)


def plan_edges(seq_len: np.ndarray, shape: FileShape, Ns: int, chunk: int = CHUNK, resume: int | None = None,
               checkpoint: bool = False):
    """seq2graph (:1876-1890) over rdbg_edge_weight_jit_ (:1809-1827): walked
    records and, per record, the checkpoint segment it belongs to.  `resume`
    is the record a -R checkpoint restarts at (resume_position).  With
    `checkpoint`, also the record whose seqio ptr is the offset of the last
    `<in>_rdb_brkpt.npz` dump (:1880-1887), or None (no checkpoint)."""
    R = seq_len.shape[0]
    flags = np.zeros(R, np.uint8)
    segment = np.full(R, -1, np.int64)
    ckpt = None
    recs = list(range(R)) if not resume else _resumed_records(resume, R, shape)
    N = 0
    seg = 0
    n_checkpoints = 0
    while True:
        chk = 0
        done, last = 1, None
        for r in recs:
            n = 0 if r == "extra" else int(seq_len[r])
            if r != "extra":
                flags[r] = 1
                segment[r] = seg
            N += n
            if ns_hit(N, Ns):
                break
            chk += n
            if chk > chunk:
                done, last = -1, r
                break
        if done != -1:
            break
        n_checkpoints += 1
        ckpt = last
        seg += 1
        recs = _resumed_records(last + 1, R, shape)
    return (flags, segment, n_checkpoints, ckpt) if checkpoint else (flags, segment, n_checkpoints)


def plan_rows(seq_len: np.ndarray, shape: FileShape, buf, Ns: int):
    """seqs2path_jit_ (:1831-1849).  It hands `isfasta` (True) to seqio_jit_'s
    offset slot (:1833), so line scanning starts at byte 1; that differs from
    byte 0 only when the file starts with '\\n' and record 0's header is the
    next line — that record is then lost."""
    R = seq_len.shape[0]
    flags = np.zeros(R, np.uint8)
    first = 0
    if R and len(buf) > 1 and buf[0] == 10 and shape.first_header_at == 1:
        first = 1
    N = 0
    for r in range(first, R):
        flags[r] = 1
        N += int(seq_len[r])
        if ns_hit(N, Ns):
            break
    return flags


def edge_order(walk_first: np.ndarray, segment_of_record: np.ndarray, n_checkpoints: int) -> np.ndarray:
    """Iteration order of the edge Dict: first occurrence, reversed at every
    dump/reload checkpoint (dict2array pops LIFO, :229; array2dict re-inserts,
    :264-286).  Input rows are in first-occurrence order; returns the
    permutation into the reference's order."""
    m = walk_first.shape[0]
    idx = np.arange(m, dtype=np.int64)
    if m == 0 or n_checkpoints == 0:
        return idx
    seg = segment_of_record[walk_first // 2]
    order = np.zeros(0, np.int64)
    for s in range(n_checkpoints + 1):
        order = np.concatenate([order, idx[seg == s]])
        if s < n_checkpoints:
            order = order[::-1]
    return order


# -------------------------------------------------------------------- text
def xyz_text(tuples: np.ndarray, counts: np.ndarray) -> str:
    """`"%d_%d\\t%d_%d\\t%d\\n"` per edge (:1901)."""
    return "".join("%d_%d\t%d_%d\t%d\n" % (a, b, c, d, e)
                   for (a, b, c, d), e in zip(tuples.tolist(), counts.tolist()))


def label_dict(mcl_text: str, xyz_lines) -> dict:
    """seq2graph :1918-1944: `.mcl` line index, then unseen `.xyz` nodes."""
    lab = {}
    flag = 0
    for line in mcl_text.splitlines(keepends=True):
        for tok in line[:-1].split("\t"):
            lab[tuple(map(int, tok.split("_")[:2]))] = flag
        flag += 1
    for line in xyz_lines:
        j, k = line[:-1].split("\t")[:2]
        kj = tuple(map(int, j.split("_")[:2]))
        if kj not in lab:
            lab[kj] = flag
            flag += 1
        kk = tuple(map(int, k.split("_")[:2]))
        if kk not in lab:
            lab[kk] = flag
            flag += 1
    return lab


def mcl_labels(mcl_text: str):
    """The `.mcl` part of seq2graph's label dictionary (:1918-1929): every
    token's line index, a later line winning as dict assignment does.
    Returns (keys, vals, ids) as int64 (keys carry the uint64 key's bits) and
    the number of lines (the next label)."""
    seen = {}
    flag = 0
    for line in mcl_text.splitlines(keepends=True):
        for tok in line[:-1].split("\t"):
            p = tok.split("_")[:2]
            seen[(int(p[0]), int(p[1]))] = flag
        flag += 1
    mk = np.array([k for k, _ in seen.keys()], dtype=np.uint64).view(np.int64)
    mv = np.array([v for _, v in seen.keys()], dtype=np.uint64).view(np.int64)
    mi = np.fromiter(seen.values(), dtype=np.int64, count=len(seen))
    return mk, mv, mi, flag


def label_table(mcl_text: str, tuples: np.ndarray):
    """label_dict + label_arrays without the text round trip: the `.mcl` line
    index of every token (a later line wins, as dict assignment does), then
    every `.xyz` node (n0_v0 then n1_v1 of each edge, in edge order) not seen
    yet, numbered in first-appearance order.  Returns (keys, vals, ids) as
    int64 (keys carry the uint64 key's bits)."""
    seen = {}
    flag = 0
    for line in mcl_text.splitlines(keepends=True):
        for tok in line[:-1].split("\t"):
            p = tok.split("_")[:2]
            seen[(int(p[0]), int(p[1]))] = flag
        flag += 1
    t = np.ascontiguousarray(tuples, dtype=np.uint64).reshape(-1, 4)
    nodes = np.empty((2 * t.shape[0], 2), np.uint64)
    nodes[0::2] = t[:, 0:2]
    nodes[1::2] = t[:, 2:4]
    if nodes.shape[0]:
        vv = np.ascontiguousarray(nodes).view(np.dtype((np.void, 16))).ravel()
        _, first = np.unique(vv, return_index=True)
        uniq = nodes[np.sort(first)]
    else:
        uniq = nodes
    if seen:
        keep = np.fromiter(((int(a), int(b)) not in seen for a, b in uniq.tolist()), dtype=bool, count=uniq.shape[0])
        uniq = uniq[keep]
    mk = np.array([k for k, _ in seen.keys()], dtype=np.uint64)
    mv = np.array([v for _, v in seen.keys()], dtype=np.uint64)
    mi = np.fromiter(seen.values(), dtype=np.int64, count=len(seen))
    keys = np.concatenate([mk, uniq[:, 0]]).view(np.int64)
    vals = np.concatenate([mv, uniq[:, 1]]).view(np.int64)
    ids = np.concatenate([mi, flag + np.arange(uniq.shape[0], dtype=np.int64)])
    return keys, vals, ids


def label_arrays(lab: dict):
    n = len(lab)
    keys = np.fromiter((a for a, _ in lab.keys()), dtype=np.int64, count=n)
    vals = np.fromiter((b for _, b in lab.keys()), dtype=np.int64, count=n)
    ids = np.fromiter(lab.values(), dtype=np.int64, count=n)
    return keys, vals, ids


def format_rows(rows: np.ndarray, buf, hdr_start: np.ndarray, hdr_len: np.ndarray):
    """`print('%s\\t%d\\t%d\\t%s\\t%d')` (:1947-1949); qid = header line minus '>'."""
    names = {}
    out = []
    for r, s, e, strand, lab in rows.tolist():
        q = names.get(r)
        if q is None:
            hs, hl = int(hdr_start[r]), int(hdr_len[r])
            q = names[r] = bytes(buf[hs:hs + hl]).decode()[1:]
        out.append("%s\t%d\t%d\t%s\t%d" % (q, s, e, "+" if strand == 1 else "-", lab))
    return out


# ------------------------------------------------------------ npz side files
DB_LOAD = 750000000            # int(0.75 * 1e9): oakht's load factor as dump() stores it (:252)
NPZ_PIECE = 32 << 20           # bytes per CRC / write task of savez_stored


def _crc32_combine():
    """zlib's crc32_combine (libz, not exposed by Python's zlib module)."""
    import ctypes
    f = getattr(_crc32_combine, "f", None)
    if f is None:
        z = ctypes.CDLL("libz.so.1")
        f = z.crc32_combine
        f.restype = ctypes.c_ulong
        f.argtypes = [ctypes.c_ulong, ctypes.c_ulong, ctypes.c_long]
        _crc32_combine.f = f
    return f


class Deferred:
    """A savez_stored member whose data a native writer puts into the file:
    `n` elements of `dtype` (a 1-D array)."""

    def __init__(self, dtype, n: int):
        self.dtype = np.dtype(dtype)
        self.n = int(n)


def savez_stored(fn: str, fill=None, **arrays) -> None:
    """np.savez(fn, **arrays) (a zip of stored .npy members, what np.load and
    the reference's load_on_disk read, :289-335), written in parallel: every
    member's bytes go to the file in NPZ_PIECE pieces by a thread pool
    (os.pwrite at their final offsets) while the same threads CRC them
    (zlib.crc32, GIL released; pieces joined with crc32_combine); then the
    local headers, the central directory and the ZIP64 end records.  The
    single-threaded zipfile CRC and write of np.savez took 0.67 s for C3's
    dump (0.45 s of it CRC).  A `Deferred` member's data is written by
    `fill(fd, offsets)` (its data offsets in member order), which returns
    their CRC-32s."""
    import struct
    import zlib
    from concurrent.futures import ThreadPoolExecutor
    fn = fn if fn.endswith(".npz") else fn + ".npz"
    comb = _crc32_combine()
    members = []
    off = 0
    for name, arr in arrays.items():
        if isinstance(arr, Deferred):
            hd = {"descr": np.lib.format.dtype_to_descr(arr.dtype), "fortran_order": False, "shape": (arr.n,)}
            body, blen = None, arr.n * arr.dtype.itemsize
        else:
            a = np.ascontiguousarray(arr)
            hd = np.lib.format.header_data_from_array_1_0(a)
            body = a.reshape(-1).view(np.uint8) if a.size else np.zeros(0, np.uint8)
            blen = body.shape[0]
        hb = io.BytesIO()
        np.lib.format.write_array_header_1_0(hb, hd)
        head = hb.getvalue()
        zname = (name + ".npy").encode()
        lh = 30 + len(zname) + 20                       # local header + ZIP64 extra (sizes)
        members.append([zname, head, body, off, lh, blen])
        off += lh + len(head) + blen
    fd = os.open(fn, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
    try:
        tasks = []
        for mi, (zname, head, body, moff, lh, blen) in enumerate(members):
            d0 = moff + lh + len(head)
            if body is not None:
                for p in range(0, blen, NPZ_PIECE):
                    tasks.append((mi, p, body[p:p + NPZ_PIECE], d0 + p))

        def work(t):
            mi, p, piece, at = t
            mv = memoryview(piece)
            done = 0
            while done < len(mv):
                done += os.pwrite(fd, mv[done:], at + done)
            return mi, p, zlib.crc32(mv), len(mv)
        crcs = {}
        if tasks:
            with ThreadPoolExecutor(max_workers=min(16, len(tasks), os.cpu_count() or 4)) as ex:
                for mi, p, c, n in ex.map(work, tasks):
                    crcs[(mi, p)] = (c, n)
        deferred = [mi for mi, m in enumerate(members) if m[2] is None]
        if deferred:
            got = fill(fd, [members[mi][3] + members[mi][4] + len(members[mi][1]) for mi in deferred])
            for mi, c in zip(deferred, got):
                crcs[(mi, 0)] = (int(c), members[mi][5])
        cdir = bytearray()
        dt = (0 << 11) | (0 << 5), (1 << 5) | 1        # 00:00:00, 1980-01-01
        for mi, (zname, head, body, moff, lh, blen) in enumerate(members):
            crc = zlib.crc32(head)
            for p in (range(0, blen, NPZ_PIECE) if body is not None else [0] if blen else []):
                c, n = crcs[(mi, p)]
                crc = comb(crc, c, n)
            size = len(head) + blen
            local = struct.pack("<IHHHHHIIIHH", 0x04034B50, 45, 0, 0, dt[0], dt[1], crc, 0xFFFFFFFF, 0xFFFFFFFF,
                                len(zname), 20) + zname + struct.pack("<HHQQ", 1, 16, size, size) + head
            done = 0
            while done < len(local):
                done += os.pwrite(fd, local[done:], moff + done)
            cdir += struct.pack("<IHHHHHHIIIHHHHHII", 0x02014B50, 45, 45, 0, 0, dt[0], dt[1], crc, 0xFFFFFFFF,
                                0xFFFFFFFF, len(zname), 28, 0, 0, 0, 0, 0xFFFFFFFF) + zname + \
                struct.pack("<HHQQQ", 1, 24, size, size, moff)
        n = len(members)
        tail = bytes(cdir) + struct.pack("<IQHHIIQQQQ", 0x06064B50, 44, 45, 45, 0, 0, n, n, len(cdir), off) + \
            struct.pack("<IIQI", 0x07064B50, 0, off + len(cdir), 1) + \
            struct.pack("<IHHHHIIH", 0x06054B50, 0, 0, min(n, 0xFFFF), min(n, 0xFFFF), 0xFFFFFFFF, 0xFFFFFFFF, 0)
        done = 0
        while done < len(tail):
            done += os.pwrite(fd, tail[done:], off + done)
    finally:
        os.close(fd)


def write_db_npz(fn: str, capacity: int, size: int, keys, values, counts, offset: int = 0):
    """dump() for an oakht (:243-261): parameters [capacity, load * 1e9, size,
    ksize, vsize, offset] and the keys / values / counts slot arrays."""
    fn = fn[:-4] if fn.endswith(".npz") else fn
    params = np.asarray([capacity, DB_LOAD, size, 1, 1, offset], dtype=np.uint64)
    # members stored (np.savez's format) rather than the reference's
    # savez_compressed: the same zip of .npy members, read identically by
    # np.load / the reference's load_on_disk, ~1.4x the bytes, but deflate ran
    # at ~30 MB/s on the slot arrays (C3: 26 s of a 42 s CLI run)
    savez_stored(fn, parameters=params, keys=keys, values=values, counts=counts)


def write_db_npz_from(fn: str, capacity: int, size: int, fill, offset: int = 0):
    """write_db_npz with the slot arrays written by `fill(fd, offsets)` (the
    device's pg_dbg_dump_fd): the same file, no host copy of the arrays."""
    fn = fn[:-4] if fn.endswith(".npz") else fn
    params = np.asarray([capacity, DB_LOAD, size, 1, 1, offset], dtype=np.uint64)
    savez_stored(fn, fill, parameters=params, keys=Deferred(np.uint64, capacity),
                 values=Deferred(np.uint16, capacity), counts=Deferred(np.uint8, capacity))


def read_db_npz(fn: str):
    """load_on_disk (:289-335) of an oakht dump: (offset, keys, values, counts)
    of the occupied (counts > 0) slots, the entries iteritems yields (:623-631).
    The file is read with numpy's non-pickling loader."""
    with np.load(fn, allow_pickle=False) as z:
        params = np.asarray(z["parameters"])
        if params.shape[0] != 6:
            raise ValueError("%s: not an oakht dump (parameters %r)" % (fn, params.tolist()))
        if int(params[3]) != 1 or int(params[4]) != 1:
            raise ValueError("%s: ksize/vsize %d/%d, the dBG uses 1/1" % (fn, int(params[3]), int(params[4])))
        counts = np.asarray(z["counts"])
        sel = counts > 0
        keys = np.asarray(z["keys"])[sel].astype(np.uint64)
        values = np.asarray(z["values"])[sel].astype(np.uint16)
        return int(params[5]), keys, values, np.minimum(counts[sel], 255).astype(np.uint8)


def resume_position(offset: int, rec_ptr: np.ndarray) -> int:
    """The record a checkpoint's `offset` (seqio's ptr when record r was
    yielded, :1255-1259) restarts at: r + 1.  Offset 0 is a fresh start."""
    if offset == 0:
        return 0
    hit = np.flatnonzero(rec_ptr == offset)
    if hit.shape[0] == 0:
        raise ValueError("checkpoint offset %d is not a record boundary of this input" % offset)
    return int(hit[0]) + 1


def write_edge_npz(fn: str, tuples, counts, offset: int):
    """dump(jit=True, ksize=4, vsize=1) of the edge Dict (:243-250): parameters
    [4, 1, offset], then dict2array's popitem order (:221-235) - the Dict's
    iteration order reversed.  `tuples` / `counts` are in iteration order."""
    fn = fn[:-4] if fn.endswith(".npz") else fn
    t = np.ascontiguousarray(np.asarray(tuples, dtype=np.uint64)[::-1]).reshape(-1)
    c = np.ascontiguousarray(np.asarray(counts)[::-1]).astype(np.uint64)
    savez_stored(fn, parameters=np.asarray([4, 1, offset], dtype=np.uint64), keys=t, values=c)


def read_edge_npz(fn: str):
    """load_on_disk(jit=True) (:305-309) of an edge checkpoint: (offset,
    tuples[N, 4] uint64, counts[N]) in file order — array2dict's insertion
    order (:264-286)."""
    with np.load(fn, allow_pickle=False) as z:
        params = np.asarray(z["parameters"])
        if params.shape[0] != 3 or int(params[0]) != 4 or int(params[1]) != 1:
            raise ValueError("%s: not an edge checkpoint (parameters %r)" % (fn, params.tolist()))
        keys = np.asarray(z["keys"]).astype(np.uint64)
        values = np.asarray(z["values"])
        n = min(keys.shape[0] // 4, values.shape[0])
        return int(params[2]), keys[:4 * n].reshape(n, 4), values[:n].astype(np.int64)


def merge_edges(loaded_t, loaded_c, tuples, counts, walk_first, segment_of_record, n_checkpoints):
    """The edge Dict of a resumed seq2graph (:1859-1887): the loaded items in
    file order, then the walks' edges by first occurrence — a known edge adds
    its walk count in place, a new one is appended — and the whole Dict
    reversed at every further checkpoint dump/reload."""
    d = {}
    for t, c in zip(map(tuple, loaded_t.tolist()), loaded_c.tolist()):
        d[t] = c
    seg = segment_of_record[walk_first // 2] if walk_first.shape[0] else np.zeros(0, np.int64)
    tl, cl = tuples.tolist(), counts.tolist()
    for s in range(n_checkpoints + 1):
        for i in np.flatnonzero(seg == s).tolist():
            t = tuple(tl[i])
            d[t] = d.get(t, 0) + cl[i]
        if s < n_checkpoints:
            d = dict(reversed(list(d.items())))
    out_t = np.array(list(d.keys()), dtype=np.uint64).reshape(-1, 4)
    out_c = np.array(list(d.values()), dtype=np.int64)
    return out_t, out_c

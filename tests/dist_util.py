"""Test infrastructure for the multi-rank paths (pangenome_amd/dist.py).

* seqio_records  numpy restatement of readline_jit_ / seqio_jit_'s record
                 table (kmer_numba.py:122-172);
* NumpyTable     CPU stand-in for the GPU table's owner partition / OR-merge /
                 rdBG rule (the exchange's 16-byte canonical records);
* oak_*          oakht.pointer (:521-538) and a slot layout built the way
                 __setitem__ does, oakht's capacity growth (:355-372, :551-558);
* OracleShard    the shard backend of dist.DistRun on the CPU: the C oracle
                 builds each shard's dBG, counts and walks; NumpyTable does the
                 exchange.  It supports the default pass plans (every record,
                 no -n / checkpoint / resume), which is what the CPU tests run;
                 the GPU tests cover the rest through GpuShard.
"""
import ctypes
import os
import socket

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PRES_A, B_SHIFT = 1 << 12, 13
M64 = (1 << 64) - 1
SENTINEL = 2 ** 64 - 1


# ----------------------------------------------------------------- records
def seqio_records(buf: bytes):
    """readline_jit_ (:122-132) + seqio_jit_ (:135-172), isfasta, offset 0:
    [(seq_len, hdr_start, hdr_len, ptr), ...]."""
    a = np.frombuffer(buf, dtype=np.uint8)
    n = a.shape[0]
    nl = np.flatnonzero(a == 10)
    starts = np.concatenate([[0], nl + 1])[: nl.shape[0]]
    ends = nl + 1
    if n and nl.shape[0]:
        st = int(nl[-1]) + 1
        if n - 1 > st > 0:                                   # end > start > 0
            starts = np.append(starts, st)
            ends = np.append(ends, n)
    recs = []
    cur = None
    for st, ed in zip(starts.tolist(), ends.tolist()):
        if a[st] == 62:
            if cur is not None:
                recs.append((cur[0], cur[1], cur[2], st))
            cur = [0, st, ed - 1 - st]
        elif cur is not None:
            cur[0] += ed - st - 1
    if cur is not None:
        recs.append((cur[0], cur[1], cur[2], int(starts[-1])))
    return recs


# ------------------------------------------------------------------- oakht
def oak_fnv(x):
    a = 0xCBF29CE484222325
    for i in range(4):
        a ^= (x >> (8 * i)) & 0xFF
        a = (a * 0x100000001B3) & M64
    return a


def oak_slot(keys, counts, x):
    """oakht.pointer (:521-538): j, j, j+1, j+4, ... until the key or an empty slot."""
    M = keys.shape[0]
    j0 = oak_fnv(x) % M
    j = j0
    for k in range(M):
        if int(keys[j]) == x or counts[j] == 0:
            break
        j = (j0 + k * k) % M
    return j


def oak_place(keys_in, vals_in, cnts_in, M):
    """A valid oakht layout built the way __setitem__ does (test helper)."""
    keys = np.zeros(M, np.uint64)
    vals = np.zeros(M, np.uint16)
    cnts = np.zeros(M, np.uint8)
    for x, v, c in zip(keys_in.tolist(), vals_in.tolist(), cnts_in.tolist()):
        j = oak_slot(keys, cnts, x)
        keys[j], vals[j], cnts[j] = x, v, c
    return keys, vals, cnts


def oak_place_rounds(keys_in, vals_in, cnts_in, M):
    """pg_dbg_dump's deterministic placement restated (test helper): in
    rounds, every unplaced key proposes the first still-empty slot of its
    oakht.pointer probe sequence from where it stands, and the smallest key
    proposing a slot takes it; then the n<k sentinel at the first empty slot
    of its sequence."""
    keys = np.zeros(M, np.uint64)
    vals = np.zeros(M, np.uint16)
    cnts = np.zeros(M, np.uint8)
    trip = list(zip(keys_in.tolist(), vals_in.tolist(), cnts_in.tolist()))
    sent = [t for t in trip if t[0] == SENTINEL]
    pend = [(int(x), int(v), int(c), 0) for x, v, c in trip if x != SENTINEL]
    while pend:
        prop, nxt = {}, []
        for i, (x, v, c, kk) in enumerate(pend):
            j0 = oak_fnv(x) % M
            while cnts[(j0 + kk * kk) % M]:
                kk += 1
            pend[i] = (x, v, c, kk)
            s = (j0 + kk * kk) % M
            prop[s] = min(prop.get(s, x), x)
        for x, v, c, kk in pend:
            s = (oak_fnv(x) % M + kk * kk) % M
            if prop[s] == x:
                keys[s], vals[s], cnts[s] = x, v, c
            else:
                nxt.append((x, v, c, kk + 1))
        pend = nxt
    for x, v, c in sent:
        j = oak_slot(keys, cnts, x)
        keys[j], vals[j], cnts[j] = x, v, c
    return keys, vals, cnts


def _isprime(n):
    if n <= 1 or n % 2 == 0 or n % 3 == 0:
        return False
    i = 5
    while i * i <= n:
        if n % i == 0 or n % (i + 2) == 0:
            return False
        i += 6
    return True


def oak_capacity(size):
    """init_dict(2**20) then resize to find_prime(int(cap * 1.62)) past load 0.75."""
    def find_prime(n):
        while not _isprime(n):
            n += 1
        return n
    cap = find_prime(1 << 20)
    while size / cap > 0.75:
        cap = find_prime(int(cap * 1.62))
    return cap


# ------------------------------------------------------------ numpy table
def rc_key_np(x: np.ndarray, k: int) -> np.ndarray:
    x = x.astype(np.uint64).copy()
    r = np.zeros_like(x)
    for _ in range(k):
        d = x % np.uint64(5)
        x //= np.uint64(5)
        rd = np.where(d < 4, np.uint64(3) - d, np.uint64(4))
        r = r * np.uint64(5) + rd
    return r


def popcount6(m):
    return np.array([bin(i).count("1") for i in range(64)])[m & 63]


class NumpyTable:
    """CPU stand-in for the GPU table (test infrastructure)."""

    def __init__(self, k):
        self.k = k
        self.c = np.zeros(0, np.uint64)
        self.mw = np.zeros(0, np.uint64)
        self.sentinel = False

    def load_dbg(self, keys, masks):
        keys = keys.astype(np.uint64)
        sent = keys == np.uint64(SENTINEL)
        self.sentinel = bool(sent.any())
        keys, masks = keys[~sent], masks[~sent].astype(np.uint64)
        rc = rc_key_np(keys, self.k)
        c = np.minimum(keys, rc)
        word = np.where(keys == c, masks | PRES_A, (masks | PRES_A) << np.uint64(B_SHIFT))
        self._set(c, word)

    def _set(self, c, word):
        order = np.argsort(c, kind="stable")
        c, word = c[order], word[order]
        uniq, start = np.unique(c, return_index=True)
        self.c, self.mw = uniq, np.bitwise_or.reduceat(word, start) if c.size else word

    def _owner(self, nparts, routed=False):
        z = self.c * np.uint64(0x9E3779B97F4A7C15 if not routed else 0xC2B2AE3D27D4EB4F)
        return ((z >> np.uint64(40)) % np.uint64(nparts)).astype(np.int64)

    def partition(self, nparts, ptr=None, cap=0, routed=False):
        """routed: 12-byte rows {key + 1 (two 32-bit words), mask word}, as
        pg_route_scatter lays them out; else 16-byte records {key + 1, mask}."""
        from pangenome_amd.dist import row_check_sum
        own = self._owner(nparts, routed)
        counts = np.bincount(own, minlength=nparts).astype(np.uint64)
        if ptr is not None:
            order = np.argsort(own, kind="stable")
            if routed:
                buf = np.ctypeslib.as_array((ctypes.c_uint32 * (3 * cap)).from_address(ptr)).reshape(cap, 3)
                k1 = self.c[order] + np.uint64(1)
                buf[:, 0] = (k1 & np.uint64(0xFFFFFFFF)).astype(np.uint32)
                buf[:, 1] = (k1 >> np.uint64(32)).astype(np.uint32)
                buf[:, 2] = self.mw[order].astype(np.uint32)
            else:
                buf = np.ctypeslib.as_array((ctypes.c_int64 * (2 * cap)).from_address(ptr)).reshape(cap, 2)
                buf[:, 0] = (self.c[order] + np.uint64(1)).view(np.int64)
                buf[:, 1] = self.mw[order].view(np.int64)
            off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
            self.psums = np.array([row_check_sum(buf[off[i]:off[i + 1]]) for i in range(nparts)], np.uint64)
        return counts

    def partition_sums(self, nparts):
        return self.psums[:nparts]

    def entries(self):
        return int(self.c.shape[0])

    def merge(self, ptr, n, sentinel=False, routed=False):
        from pangenome_amd.dist import row_check_sum
        if n and routed:
            buf = np.ctypeslib.as_array((ctypes.c_uint32 * (3 * n)).from_address(ptr)).reshape(n, 3)
            k1 = buf[:, 0].astype(np.uint64) | (buf[:, 1].astype(np.uint64) << np.uint64(32))
            self.mcheck = (int(np.count_nonzero(k1)), row_check_sum(buf))
            self._set(k1 - np.uint64(1), buf[:, 2].astype(np.uint64))
        elif n:
            buf = np.ctypeslib.as_array((ctypes.c_int64 * (2 * n)).from_address(ptr)).reshape(n, 2)
            self.mcheck = (int(np.count_nonzero(buf[:, 0])), row_check_sum(buf))
            self._set(buf[:, 0].view(np.uint64) - np.uint64(1), buf[:, 1].view(np.uint64))
        else:
            self.mcheck = (0, 0)
            self.c, self.mw = np.zeros(0, np.uint64), np.zeros(0, np.uint64)
        self.sentinel = sentinel

    def merge_check(self):
        return self.mcheck

    def _members(self):
        a = (self.mw & np.uint64(0xFFF)).astype(np.int64)
        b = ((self.mw >> np.uint64(B_SHIFT)) & np.uint64(0xFFF)).astype(np.int64)
        pa = (self.mw & np.uint64(PRES_A)) != 0
        pb = (self.mw & np.uint64(PRES_A << B_SHIFT)) != 0
        ma = pa & ~((popcount6(a >> 6) == 1) & (popcount6(a) == 1))
        mb = pb & ~((popcount6(b >> 6) == 1) & (popcount6(b) == 1))
        return pa, pb, ma, mb

    def build_rdbg(self):
        pa, pb, ma, mb = self._members()

        class St:
            pass
        st = St()
        st.n_dbg = int(pa.sum() + pb.sum()) + int(self.sentinel)
        st.n_rdbg = int(ma.sum() + mb.sum()) + int(self.sentinel)
        return st

    def rdbg_keys(self):
        _, _, ma, mb = self._members()
        keys = [self.c[ma], rc_key_np(self.c[mb], self.k)]
        if self.sentinel:
            keys.append(np.array([SENTINEL], np.uint64))
        return np.sort(np.concatenate(keys))


# ------------------------------------------------------- oracle shard backend
class OracleShard:
    """dist.DistRun's shard backend on the CPU (test infrastructure)."""

    def __init__(self, k):
        self.k = k
        self.table = NumpyTable(k)

    def load(self, data):
        self.data = bytes(np.asarray(data, np.uint8))
        recs = seqio_records(self.data)
        cols = list(zip(*recs)) if recs else [(), (), (), ()]
        self.meta = {name: np.asarray(col, np.int64)
                     for name, col in zip(("seq_len", "hdr_start", "hdr_len", "ptr"), cols)}
        self.run = None
        return self.meta

    def stage(self, keys, masks=None, counts=None):
        raise NotImplementedError("OracleShard: staged npz slots are covered by the GPU tests")

    def build(self, flags, extra, rc0):
        """All records (the default plan), or a contiguous run of them (a
        chunk of the streaming exchange: the run's bytes parse exactly as in
        the shard, since they end before a header line or at the end)."""
        from oracle import oracle
        flags = np.asarray(flags)
        assert extra == 0, "OracleShard runs the default pass plan only"
        self.rc0 = bool(rc0)
        if np.all(flags == 1):
            self.run = self.cnt = oracle.OracleRun(self.data, self.k, 2 if rc0 else 0)
        else:
            idx = np.flatnonzero(flags)
            if idx.size == 0:
                self.cnt = None
                self.table.load_dbg(np.zeros(0, np.uint64), np.zeros(0, np.uint16))
                return self.table.sentinel
            assert np.all(np.diff(idx) == 1), "a chunk is a contiguous run of records"
            hs = self.meta["hdr_start"]
            end = int(hs[idx[-1] + 1]) if idx[-1] + 1 < hs.shape[0] else len(self.data)
            self.cnt = oracle.OracleRun(self.data[int(hs[idx[0]]):end], self.k, 2 if rc0 else 0)
        keys, masks = self.cnt.dbg()
        self.table.load_dbg(keys, masks)
        return self.table.sentinel

    def counts(self):
        if self.cnt is None:
            return np.zeros(0, np.uint64), np.zeros(0, np.uint16), np.zeros(0, np.uint8)
        return self.cnt.dbg_counts()

    def partition(self, nparts, ptr=None, cap=0):
        return self.table.partition(nparts, ptr, cap)

    def partition_sums(self, nparts):
        return self.table.partition_sums(nparts)

    def entries(self):
        return self.table.entries()

    def merge(self, ptr, n, sentinel=False):
        self.table.merge(ptr, n, sentinel)

    def merge_check(self):
        return self.table.merge_check()

    # the routed exchange: the local table's entries stand in for the held
    # stage A records, grouped by an owner function of their own
    def route_stage_a(self, flags, extra, rc0, nparts):
        sent = self.build(flags, extra, rc0)
        self.route_n = nparts
        return self.table.partition(nparts, routed=True), sent

    def route_scatter(self, nparts, ptr, cap):
        assert nparts == self.route_n
        self.table.partition(nparts, ptr, cap, routed=True)
        return self.table.partition_sums(nparts)

    def route_finish(self):
        return self.table.build_rdbg()

    def route_merge(self, ptr, n, nparts, sentinel=False):
        self.table.merge(ptr, n, sentinel, routed=True)
        return self.table.build_rdbg()

    def route_merge_segs(self, segs, nparts, sentinel=False):
        rows = [np.ctypeslib.as_array((ctypes.c_uint32 * (3 * n)).from_address(p)).reshape(n, 3)
                for p, n in segs if n]
        buf = np.ascontiguousarray(np.concatenate(rows)) if rows else np.zeros((1, 3), np.uint32)
        self.table.merge(buf.ctypes.data, buf.shape[0] if rows else 0, sentinel, routed=True)
        return self.table.build_rdbg()

    def route_rows_checksum(self, d_rows, seg_off):
        from pangenome_amd.dist import row_check_sum
        off = np.asarray(seg_off, np.int64)
        n = int(off[-1]) if off.size else 0
        buf = np.ctypeslib.as_array((ctypes.c_uint32 * (3 * max(n, 1))).from_address(d_rows)).reshape(-1, 3)
        return [row_check_sum(buf[off[i]:off[i + 1]]) for i in range(off.size - 1)]

    def build_rdbg(self):
        return self.table.build_rdbg()

    def owner_rdbg(self):
        return self.table.rdbg_keys()

    def members(self, keys, n_records, rc0):
        if self.run is None:                       # a streamed build ran chunks only
            from oracle import oracle
            self.run = oracle.OracleRun(self.data, self.k, 2 if rc0 else 0)
        self.run.set_rdbg(keys)

    def edges(self, flags, rc1):
        assert np.all(np.asarray(flags) == 1)
        self.run.c = (2 if self.rc0 else 0) | (1 if rc1 else 0)
        t, c = self.run.edges()
        return t, c, np.zeros(c.shape[0], np.int64)

    def rows_text(self, labels, flags, rc1, names):
        assert np.all(np.asarray(flags) == 1)
        self.run.c = (2 if self.rc0 else 0) | (1 if rc1 else 0)
        lines = self.run.rows(labels)
        return "".join(x + "\n" for x in lines).encode()

    def dump_global(self, keys, masks, counts, k, device):
        keys = np.asarray(keys, np.uint64)
        u, inv = np.unique(keys, return_inverse=True)
        v = np.zeros(u.shape[0], np.uint16)
        np.bitwise_or.at(v, inv.ravel(), np.asarray(masks, np.uint16))
        c = np.zeros(u.shape[0], np.int64)
        np.add.at(c, inv.ravel(), np.asarray(counts, np.int64))
        M = oak_capacity(u.shape[0])
        K, V, C = oak_place(u, v, np.minimum(c, 255).astype(np.uint8), M)
        return M, u.shape[0], K, V, C


# ---------------------------------------------------------------- spawning
def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(world, target, args, timeout=300):
    """Run target(rank, world, port, q, *args) in `world` spawned processes;
    returns {rank: what the rank put on q}."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + tuple(args)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            r, res = q.get(timeout=timeout)
            out[r] = res
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for p in procs:
        assert p.exitcode == 0, "rank process failed (exit %s)" % p.exitcode
    return out

"""The N>1 exchange protocol (pangenome_amd/dist.py) on CPU with gloo, world 2.

Each rank owns half the records of a small pangenome; its local dBG comes from
the oracle, in the same 16-byte canonical record format the GPU exchanges
(key+1, 26-bit mask word of both orientations).  A numpy table stands in for
the GPU table's partition / merge / degree scan.  The sharded totals must equal
the single-process build over all records.
"""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PRES_A, B_SHIFT = 1 << 12, 13


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

    def load_dbg(self, keys, masks):
        keys = keys.astype(np.uint64)
        sent = keys == np.uint64(2 ** 64 - 1)
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

    def _owner(self, nparts):
        z = self.c * np.uint64(0x9E3779B97F4A7C15)
        return ((z >> np.uint64(40)) % np.uint64(nparts)).astype(np.int64)

    def partition(self, nparts, ptr=None, cap=0):
        own = self._owner(nparts)
        counts = np.bincount(own, minlength=nparts).astype(np.uint64)
        if ptr is not None:
            buf = np.ctypeslib.as_array((ctypes.c_int64 * (2 * cap)).from_address(ptr)).reshape(cap, 2)
            order = np.argsort(own, kind="stable")
            buf[:, 0] = (self.c[order] + np.uint64(1)).view(np.int64)
            buf[:, 1] = self.mw[order].view(np.int64)
        return counts

    def merge(self, ptr, n, sentinel=False):
        if n:
            buf = np.ctypeslib.as_array((ctypes.c_int64 * (2 * n)).from_address(ptr)).reshape(n, 2)
            self._set(buf[:, 0].view(np.uint64) - np.uint64(1), buf[:, 1].view(np.uint64))
        else:
            self.c, self.mw = np.zeros(0, np.uint64), np.zeros(0, np.uint64)
        self.sentinel = sentinel

    def build_rdbg(self):
        a = (self.mw & np.uint64(0xFFF)).astype(np.int64)
        b = ((self.mw >> np.uint64(B_SHIFT)) & np.uint64(0xFFF)).astype(np.int64)
        pa = (self.mw & np.uint64(PRES_A)) != 0
        pb = (self.mw & np.uint64(PRES_A << B_SHIFT)) != 0
        ma = pa & ~((popcount6(a >> 6) == 1) & (popcount6(a) == 1))
        mb = pb & ~((popcount6(b >> 6) == 1) & (popcount6(b) == 1))

        class St:
            pass
        st = St()
        st.n_dbg = int(pa.sum() + pb.sum()) + int(self.sentinel)
        st.n_rdbg = int(ma.sum() + mb.sum()) + int(self.sentinel)
        return st


def _records(fasta: bytes):
    parts = fasta.split(b"\n>")
    return [p if i == 0 else b">" + p for i, p in enumerate(parts)]


def _worker(rank, world, port, fasta, k, q):
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from oracle import oracle
    from pangenome_amd.dist import exchange_and_reduce
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    recs = _records(fasta)
    mine = b"".join(r if r.endswith(b"\n") else r + b"\n" for r in recs[rank::world])
    keys, masks = oracle.OracleRun(mine, k, 2).dbg()
    t = NumpyTable(k)
    t.load_dbg(keys, masks)
    res = exchange_and_reduce(t, world, rank, "cpu", t.sentinel)
    q.put((rank, res))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_exchange_matches_single_process(oracle_mod, world):
    from pangenome_amd import synth
    k = 27
    fasta = synth.pangenome(6, 30_000, snp=0.01, indel=1e-3, seed=41) + b">tiny\nACG\n"
    ref = oracle_mod.OracleRun(fasta, k, 2)
    ref_dbg = ref.dbg()[0].shape[0]
    ref_rdbg = ref.rdbg().shape[0]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fasta, k, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        n_dbg, n_rdbg, _, _ = out[r]
        assert n_dbg == ref_dbg
        assert n_rdbg == ref_rdbg
    # owners hold disjoint partitions
    assert sum(out[r][2] for r in range(world)) == ref_rdbg

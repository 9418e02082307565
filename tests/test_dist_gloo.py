"""The N>1 exchange protocol (pangenome_amd/dist.py) on CPU with gloo, world 2.

Each rank owns half the records of a small pangenome; its local dBG comes from
the oracle, in the same 16-byte canonical record format the GPU exchanges
(key+1, 26-bit mask word of both orientations).  A numpy table stands in for
the GPU table's partition / merge / degree scan.  The sharded totals must equal
the single-process build over all records.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from dist_util import ROOT, NumpyTable


def _records(fasta: bytes):
    parts = fasta.split(b"\n>")
    return [p if i == 0 else b">" + p for i, p in enumerate(parts)]


def _worker(rank, world, port, fasta, k, q, a2a_rows=None):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist
    from oracle import oracle
    from pangenome_amd import dist as pdist
    from pangenome_amd.dist import exchange_and_reduce
    if a2a_rows:
        pdist.A2A_ROWS = a2a_rows                 # the piecewise all-to-all (RCCL's 1 GiB limit)
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


@pytest.mark.parametrize("world,a2a_rows", [(2, None), (3, None), (3, 1000)])
def test_sharded_exchange_matches_single_process(oracle_mod, world, a2a_rows):
    from pangenome_amd import synth
    k = 27
    fasta = synth.pangenome(6, 30_000, snp=0.01, indel=1e-3, seed=41) + b">tiny\nACG\n"
    ref = oracle_mod.OracleRun(fasta, k, 2)
    ref_dbg = ref.dbg()[0].shape[0]
    ref_rdbg = ref.rdbg().shape[0]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fasta, k, q, a2a_rows)) for r in range(world)]
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


def _routed_worker(rank, world, port, fasta, k, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist
    from dist_util import OracleShard
    from pangenome_amd.dist import exchange_routed
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    recs = _records(fasta)
    mine = b"".join(r if r.endswith(b"\n") else r + b"\n" for r in recs[rank::world])
    sh = OracleShard(k)
    meta = sh.load(np.frombuffer(mine, np.uint8))
    flags = np.ones(meta["seq_len"].shape[0], np.uint8)
    tm = {}
    res = exchange_routed(sh, world, rank, "cpu", flags, 0, True, tm=tm)
    q.put((rank, res + (sorted(tm),)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2, 4])
def test_routed_exchange_matches_single_process(oracle_mod, world):
    """exchange_routed (the owners build once from routed stage A records):
    the sharded totals equal the single-process build; world 1 builds where
    the records lie, with no exchange at all."""
    from pangenome_amd import synth
    k = 27
    fasta = synth.pangenome(6, 30_000, snp=0.01, indel=1e-3, seed=43) + b">tiny\nACG\n"
    ref = oracle_mod.OracleRun(fasta, k, 2)
    ref_dbg = ref.dbg()[0].shape[0]
    ref_rdbg = ref.rdbg().shape[0]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_routed_worker, args=(r, world, port, fasta, k, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        n_dbg, n_rdbg, _, sent, phases = out[r]
        assert (n_dbg, n_rdbg) == (ref_dbg, ref_rdbg)
        assert phases == (["merge"] if world == 1 else ["all_to_all", "merge", "partition", "rows"])
    assert sum(out[r][2] for r in range(world)) == ref_rdbg


def _stream_worker(rank, world, port, q, fasta, k, routed=False):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist
    from dist_util import OracleShard
    from pangenome_amd.dist import exchange_stream, stream_chunks
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    recs = _records(fasta)
    per = -(-len(recs) // world)
    mine = b"".join(r if r.endswith(b"\n") else r + b"\n" for r in recs[rank * per:(rank + 1) * per])
    sh = OracleShard(k)
    meta = sh.load(np.frombuffer(mine, np.uint8))
    R = int(meta["seq_len"].shape[0])
    chunks = stream_chunks(np.ones(R, np.uint8), meta["seq_len"], 1)     # one record per round
    tm = {}
    if routed:
        res = exchange_stream(sh, world, rank, "cpu", chunks, R, True, tm=tm)
    else:
        res = exchange_stream(sh, world, rank, "cpu", chunks, R, True, compact_at=1, tm=tm, routed=False)
    q.put((rank, res[:5] + (sorted(k_ for k_ in tm if k_ != "start"),)))
    dist.destroy_process_group()


def test_streamed_exchange_many_rounds_world3(oracle_mod):
    """World 3 with 18 rounds: the sub-log count stays within world x P <= 64
    (P = 16, not the 32 that rounding 18 up would give: pg_dbg_partition
    takes at most 64 parts)."""
    from dist_util import spawn_ranks
    from pangenome_amd import synth
    k = 27
    fasta = synth.pangenome(54, 2_000, snp=0.01, indel=1e-3, seed=43)
    ref = oracle_mod.OracleRun(fasta, k, 2)
    out = spawn_ranks(3, _stream_worker, (fasta, k))
    for r in range(3):
        n_dbg, n_rdbg, _, _, rounds, phases = out[r]
        assert rounds == 18
        assert phases == ["build", "compact", "final", "log", "route", "setup"]
        assert (n_dbg, n_rdbg) == (ref.dbg()[0].shape[0], ref.rdbg().shape[0])
    assert sum(out[r][2] for r in range(3)) == ref.rdbg().shape[0]


@pytest.mark.parametrize("world", [1, 2, 4])
def test_routed_streamed_exchange_matches_single_process(oracle_mod, world):
    """exchange_stream's routed form (no local table: every round's stage A
    records straight to their owners' sub-logs, each sub-log one owner table
    at the end from its received segments, pg_route_merge_segs): the sharded
    totals equal the single-process build, every rank runs the same rounds,
    and the owners' rdBG partitions are disjoint."""
    from dist_util import spawn_ranks
    from pangenome_amd import synth
    k = 27
    fasta = synth.pangenome(12, 3_000, snp=0.01, indel=1e-3, seed=47) + b">tiny\nACG\n"
    ref = oracle_mod.OracleRun(fasta, k, 2)
    out = spawn_ranks(world, _stream_worker, (fasta, k, True))
    for r in range(world):
        n_dbg, n_rdbg, _, _, rounds, phases = out[r]
        assert rounds == -(-13 // world)
        assert (n_dbg, n_rdbg) == (ref.dbg()[0].shape[0], ref.rdbg().shape[0])
        assert phases == ["build", "flag", "keys", "log", "merge", "route", "setup", "tail"]
    assert sum(out[r][2] for r in range(world)) == ref.rdbg().shape[0]


def _diagnose_worker(rank, world, port, q):
    """_diagnose called directly with send/receive splits whose A2A_ROWS piece
    counts differ between the ranks (rank 0: 2 pieces, rank 1: 1)."""
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from pangenome_amd import dist as pdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pdist.A2A_ROWS = 100
    # rows sent [to 0, to 1]: rank 0 [150, 50], rank 1 [50, 50]
    counts = np.array([[150], [50]] if rank == 0 else [[50], [50]], np.int64)
    rh = np.array([[150], [50]] if rank == 0 else [[50], [50]], np.int64)
    g = torch.Generator().manual_seed(rank)
    send = torch.randint(0, 1 << 40, (int(counts.sum()), 2), generator=g, dtype=torch.int64)
    recv = torch.randint(0, 1 << 40, (int(rh.sum()), 2), generator=g, dtype=torch.int64)
    sums = np.zeros(2, np.uint64)
    bad = [(0, 0)] if rank == 0 else []
    try:
        pdist._diagnose(None, send, recv, counts, sums, rh, bad, world, 1, rank, "cpu", torch.device("cpu"), None,
                        "diag")
        q.put((rank, None))
    except pdist.ExchangeIntegrityError as e:
        q.put((rank, str(e)))
    dist.destroy_process_group()


def test_diagnose_with_uneven_piece_counts_raises_everywhere():
    """the piece count is agreed collectively (MAX all-reduce)
    before any rank diverges, so ranks with fewer pieces pad with empty ones
    and every rank raises instead of one rank waiting in an all-gather."""
    from dist_util import spawn_ranks
    out = spawn_ranks(2, _diagnose_worker, (), timeout=60)
    assert out[0] is not None and "from rank 0" in out[0], out
    assert out[1] is not None and "rank 1" in out[1], out


@pytest.mark.parametrize("world,rounds,subparts,want", [(1, 3, None, 4), (3, 17, None, 16), (3, 18, None, 16),
                                                        (5, 9, None, 8), (6, 9, None, 8), (8, 4, None, 4),
                                                        (8, 40, None, 8), (3, 2, 64, 16), (2, 1, None, 1)])
def test_sublog_count(world, rounds, subparts, want):
    from pangenome_amd.dist import sublog_count
    P = sublog_count(world, rounds, subparts)
    assert P == want and world * P <= 64 and P & (P - 1) == 0


def _corrupt_worker(rank, world, port, q, fasta, k, mode):
    """exchange_and_reduce with one record changed after the sender summed it
    (mode "send": in rank 1's send buffer, between partition and all-to-all)
    or in the owner's receive buffer before its merge (mode "merge")."""
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import ctypes
    import torch.distributed as dist
    from oracle import oracle
    from pangenome_amd import dist as pdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pdist.A2A_ROWS = 500                          # several pieces per message

    class Bad(NumpyTable):
        def partition(self, nparts, ptr=None, cap=0):
            c = super().partition(nparts, ptr, cap)
            if ptr is not None and mode == "send" and rank == 1 and cap > 1200:
                buf = np.ctypeslib.as_array((ctypes.c_int64 * (2 * cap)).from_address(ptr)).reshape(cap, 2)
                buf[1200, 1] ^= 1 << 3              # one mask bit of one record
            return c

        def merge(self, ptr, n, sentinel=False):
            if mode == "merge" and rank == 0 and n > 10:
                buf = np.ctypeslib.as_array((ctypes.c_int64 * (2 * n)).from_address(ptr)).reshape(n, 2)
                buf[10, 0] += 1                     # one key
            super().merge(ptr, n, sentinel)

    if mode == "wire":                            # a piece damaged in flight (the collective's output)
        real = pdist._all_to_all_rows

        def lossy(recv, send, rsplit, ssplit, *a, **kw):
            real(recv, send, rsplit, ssplit, *a, **kw)
            if rank == 0 and rsplit[1] > 1200:
                recv[int(rsplit[0]) + 1200, 0] += 2
        pdist._all_to_all_rows = lossy

    recs = _records(fasta)
    mine = b"".join(r if r.endswith(b"\n") else r + b"\n" for r in recs[rank::world])
    keys, masks = oracle.OracleRun(mine, k, 2).dbg()
    t = Bad(k)
    t.load_dbg(keys, masks)
    try:
        pdist.exchange_and_reduce(t, world, rank, "cpu", t.sentinel)
        q.put((rank, None))
    except pdist.ExchangeIntegrityError as e:
        q.put((rank, str(e)))
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["send", "wire", "merge"])
def test_exchange_integrity_check_raises(oracle_mod, mode):
    """A record changed anywhere between the sender's partition and the
    owner's merge fails the exchange loudly on every rank, never as a silently
    wrong count: a change in the sender's buffer after its partition sums
    (named by the sender), a piece damaged on the wire (the receiver names
    the source rank and the piece), a change in the owner's log (at the
    owner's merge)."""
    from dist_util import spawn_ranks
    from pangenome_amd import synth
    fasta = synth.pangenome(6, 30_000, snp=0.01, indel=1e-3, seed=41)
    out = spawn_ranks(2, _corrupt_worker, (fasta, 27, mode))
    if mode in ("send", "wire"):
        for r in range(2):
            assert out[r] is not None, out
        owner = [r for r in range(2) if "from rank 1" in out[r]]
        assert len(owner) == 1 and "stage: all_to_all" in out[owner[0]], out
        if mode == "send":
            assert "stage: send buffer" in out[1], out
        else:
            assert "pieces [2] of 500 rows each differ on the wire" in out[owner[0]], out
    else:
        assert out[0] is not None and "stage: merge" in out[0], out

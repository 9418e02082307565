"""The multi-rank CLI path (pangenome_amd/dist.py) on CPU with gloo.

Every rank takes its byte shard of a golden input, builds its dBG with the C
oracle (OracleShard, tests/dist_util.py), exchanges entries with its owners,
all-gathers the rdBG, walks its own records, and rank 0 reduces the edges,
writes `.xyz`, builds the label table and prints the gathered rows — the
orchestration the GPU path runs, with the oracle in place of the kernels.
The `.xyz`, the rows and the `<in>_db.npz` must equal what the reference
itself produced for the whole file (tests/golden, make_goldens.py).
"""
import io
import os
import sys

import numpy as np
import pytest

from dist_util import ROOT, OracleShard, seqio_records, spawn_ranks
from golden_util import Fixture


def _cli_rank(rank, world, port, q, qry, argv, kw=None):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist
    from pangenome_amd import dist as pdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = io.StringIO()
    used = []                                       # which owner exchange the rdBG step ran

    def spy(name):
        real = getattr(pdist, name)

        def f(*a, **k):
            used.append("%s(%s)" % (name, type(a[0]).__name__))
            return real(*a, **k)
        setattr(pdist, name, f)
    spy("exchange_routed")
    spy("exchange_and_reduce")
    try:
        pdist.entry_point(argv, out=out, shard_factory=OracleShard,
                          **{k_: v for k_, v in (kw or {}).items() if k_ != "report"})
    finally:
        dist.destroy_process_group()
    q.put((rank, out.getvalue() if kw is None or not kw.get("report") else (out.getvalue(), used)))


def rows_of(text):
    return [ln for ln in text.split("\n") if len(ln.split("\t")) == 5 and ln.split("\t")[3] in ("+", "-")]


@pytest.mark.parametrize("name,world", [("pan8_k27_c2", 2), ("pan8_k27_c3", 3), ("pan8_k27_c0", 2),
                                        ("pan8_k15", 4), ("edge_k27", 2), ("test_k27", 2)])
def test_dist_cli_matches_reference(name, world, tmp_path):
    fx = Fixture(name)
    if fx.ns is not None or fx.meta["chunk"]:
        pytest.skip("the oracle stand-in runs the default pass plan")
    q = tmp_path / "input.fsa"
    q.write_bytes(fx.fasta)
    (tmp_path / "input.fsa_rdbg_weight.xyz.mcl").write_text(fx.mcl)
    argv = ["kmer_numba.py", "-i", str(q), "-k", str(fx.k), "-c", str(fx.c)]
    got = spawn_ranks(world, _cli_rank, (str(q), argv, {"report": True}))
    outs = {r: got[r][0] for r in got}
    # the rdBG step: the routed owner exchange (the bench's N>1 step) at a
    # power-of-two world, the local-table exchange otherwise
    for r in got:
        assert got[r][1] == ["exchange_routed(OracleShard)", "exchange_and_reduce(%s)"
                             % ("_Routed" if world & (world - 1) == 0 else "OracleShard")], got[r][1]
    assert (tmp_path / "input.fsa_rdbg_weight.xyz").read_text() == fx.xyz
    assert rows_of(outs[0]) == fx.rows
    assert all(rows_of(outs[r]) == [] for r in range(1, world))           # rank 0 prints
    assert "# the mcl has been ran" in outs[0]
    # the global dBG dump: the reference's keys / values / counts
    z = np.load(str(q) + "_db.npz")
    sel = z["counts"] > 0
    o = np.argsort(z["keys"][sel], kind="stable")
    assert np.array_equal(z["keys"][sel][o], fx.dbg_keys)
    assert np.array_equal(z["values"][sel][o], fx.dbg_masks)
    assert np.array_equal(z["counts"][sel][o], fx.dbg_counts)
    assert z["parameters"].tolist() == fx.db_params.tolist()


@pytest.mark.parametrize("name,world,stream,compact", [("pan8_k27_c2", 2, 30_000, 1), ("pan8_k27_c2", 3, 1, 1),
                                                        ("pan8_k15", 2, 50_000, 1 << 26), ("edge_k27", 2, 1, 1)])
def test_dist_cli_streamed_exchange(name, world, stream, compact, tmp_path):
    """The streaming exchange (exchange_stream, the C5 form of SURVEY 8(e)):
    each rank's records in chunks of at most `stream` bases, one all-to-all
    per chunk into the owner's record log, the log compacted (merged and
    re-exported) whenever it doubles past `compact` records; the dump from
    the counts gathered chunk by chunk.  Same outputs as the reference's."""
    fx = Fixture(name)
    q = tmp_path / "input.fsa"
    q.write_bytes(fx.fasta)
    (tmp_path / "input.fsa_rdbg_weight.xyz.mcl").write_text(fx.mcl)
    argv = ["kmer_numba.py", "-i", str(q), "-k", str(fx.k), "-c", str(fx.c)]
    outs = spawn_ranks(world, _cli_rank, (str(q), argv, {"stream_bases": stream, "compact_at": compact}))
    assert (tmp_path / "input.fsa_rdbg_weight.xyz").read_text() == fx.xyz
    assert rows_of(outs[0]) == fx.rows
    z = np.load(str(q) + "_db.npz")
    sel = z["counts"] > 0
    o = np.argsort(z["keys"][sel], kind="stable")
    assert np.array_equal(z["keys"][sel][o], fx.dbg_keys)
    assert np.array_equal(z["values"][sel][o], fx.dbg_masks)
    assert np.array_equal(z["counts"][sel][o], fx.dbg_counts)


def test_stream_chunks():
    from pangenome_amd.dist import stream_chunks
    seq_len = np.array([5, 7, 3, 10, 2, 2], np.int64)
    flags = np.array([1, 1, 0, 1, 1, 1], np.uint8)
    ch = stream_chunks(flags, seq_len, 8)
    assert [np.flatnonzero(c).tolist() for c in ch] == [[0], [1], [3], [4, 5]]
    assert stream_chunks(np.zeros(3, np.uint8), seq_len[:3], 8) == []
    assert [np.flatnonzero(c).tolist() for c in stream_chunks(flags, seq_len, 100)] == [[0, 1, 3, 4, 5]]


def _bounds_case(buf, world):
    from pangenome_amd.dist import shard_bounds
    b = shard_bounds(np.frombuffer(buf, np.uint8), world)
    assert b[0] == 0 and b[-1] == len(buf) and all(x <= y for x, y in zip(b, b[1:]))
    whole = seqio_records(buf)
    parts = []
    for r in range(world):
        lo, hi = b[r], b[r + 1]
        if lo > 0 and lo < len(buf):
            assert buf[lo - 1:lo + 1] == b"\n>"                     # a header line start
        for sl, hs, hl, ptr in seqio_records(buf[lo:hi]):
            parts.append((sl, hs + lo, hl, ptr + lo, hi))
    # shard-local parses concatenate to the whole file's records; a shard's
    # last record reports ptr at the next shard's header (dist.Shards)
    assert [p[:3] for p in parts] == [w[:3] for w in whole]
    for p, w in zip(parts, whole):
        assert p[3] == w[3] or p[4] == w[3]


@pytest.mark.parametrize("world", [1, 2, 3, 5, 8])
def test_shard_bounds_parse_like_the_whole_file(world):
    cases = [b">a\nACGT\nACG\n>b\nTTTT\n>c\nGG\n>d\nA\n",
             b"JUNK\nACGT\n>a\nAC\n>b\nGG",                       # bases before the first header, no final '\n'
             b">a\nAC\n>bb",                                       # a header-only unterminated tail
             b">a\nAC\n>b\n>c\n\n>d\nAC\n",
             b"\n\n>a\nACGT\n",
             b"",
             b">only\nACGTACGTACGT\n",
             b">a\r\nAC\r\n>b\r\nGT\r\n"]
    for buf in cases:
        _bounds_case(buf, world)
    from pangenome_amd import synth
    _bounds_case(synth.pangenome(7, 3000, seed=5), world)


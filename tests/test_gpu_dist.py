"""The multi-GPU path (pangenome_amd/dist.py) through the HIP library, with
2-3 ranks sharing one MI355X; the collectives run on gloo with host staging
(RCCL needs one GPU per rank — the 8-GPU bench uses it).

* the exchange kernels (pg_dbg_partition / pg_dbg_merge / the rdBG rule on the
  owner partition) against the C oracle's dBG / rdBG of the whole input;
* the whole CLI (`python -m torch.distributed.run ... -m pangenome_amd`) against
  what the reference itself produced (tests/golden): `.xyz` in edge order,
  region rows, the `<in>_db.npz` dump, with -n limits, checkpoint chunks,
  -r / -R resumes from the reference's own checkpoints, -d and -D reloads, and
  a rank whose shard holds no record.
"""
import io
import os
import sys

import numpy as np
import pytest

from dist_util import ROOT, spawn_ranks
from golden_util import Fixture, ResumeFixture

pytestmark = pytest.mark.gpu


def _exchange_rank(rank, world, port, q, shard):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from pangenome_amd._lib import Context
    from pangenome_amd.dist import exchange_and_reduce
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = Context(27, 0)
    ctx.set_fasta(shard)
    ctx.parse()
    st = ctx.build_dbg(None, 0, True)
    res = exchange_and_reduce(ctx, world, rank, torch.device("cuda", 0), bool(st.sentinel))
    q.put((rank, (res, ctx.rdbg())))
    dist.destroy_process_group()


def test_two_rank_exchange_vs_oracle(oracle_mod):
    from pangenome_amd import synth
    fasta = synth.pangenome(8, 200_000, snp=0.005, indel=5e-4, seed=99)
    recs = [b">" + r for r in fasta.split(b">")[1:]]
    shards = [b"".join(recs[0::2]), b"".join(recs[1::2]) + b">short\nACGTA\n"]
    ref = oracle_mod.OracleRun(shards[0] + shards[1], 27, 2)
    ref_dbg, ref_rdbg = ref.dbg()[0].shape[0], ref.rdbg()
    res = spawn_ranks(2, _exchange_rank_sharded, (shards,))
    for r in range(2):
        n_dbg, n_rdbg, _, _ = res[r][0]
        assert n_dbg == ref_dbg and n_rdbg == ref_rdbg.shape[0]
    union = np.sort(np.concatenate([res[0][1], res[1][1]]))
    assert np.array_equal(union, ref_rdbg)


def _exchange_rank_sharded(rank, world, port, q, shards):
    _exchange_rank(rank, world, port, q, shards[rank])


def _routed_rank(rank, world, port, q, shards, force):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from pangenome_amd._lib import Context
    from pangenome_amd.dist import exchange_routed
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = Context(27, 0)
    out = []
    for rep in range(2):                                    # (the second build reuses the context's buffers)
        ctx.set_fasta(shards[rank])
        ctx.parse()
        res = exchange_routed(ctx, world, rank, torch.device("cuda", 0), None, 0, True, force=force)
        keys, masks = ctx.dbg()
        out.append((res, keys, masks, ctx.rdbg()))
    q.put((rank, out))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,force", [(1, False), (1, True), (2, False), (4, False)])
def test_routed_exchange_vs_oracle(oracle_mod, world, force):
    """dist.exchange_routed through the library: stage A held and routed by
    the top bits of h (pg_route_stage_a / pg_route_scatter), each owner's
    stages A-C over what it received on h rotated into its domain
    (pg_route_merge), or at world 1 stages B/C where the records lie
    (pg_route_finish).  The owners' dBG (keys and masks) and rdBG are
    disjoint and their union is the oracle's, twice in a row."""
    from pangenome_amd import synth
    fasta = synth.pangenome(8, 200_000, snp=0.005, indel=5e-4, seed=97)
    recs = [b">" + r for r in fasta.split(b">")[1:]] + [b">short\nACGTA\n", b">tiny\nAC\n"]
    shards = [b"".join(recs[r::world]) for r in range(world)]
    ref = oracle_mod.OracleRun(b"".join(recs), 27, 2)
    ref_keys, ref_masks = ref.dbg()
    ref_rdbg = ref.rdbg()
    res = spawn_ranks(world, _routed_rank, (shards, force))
    for rep in range(2):
        for r in range(world):
            n_dbg, n_rdbg, _, _ = res[r][rep][0]
            assert (n_dbg, n_rdbg) == (ref_keys.shape[0], ref_rdbg.shape[0])
        keys = np.concatenate([res[r][rep][1] for r in range(world)])
        masks = np.concatenate([res[r][rep][2] for r in range(world)])
        o = np.argsort(keys, kind="stable")
        assert np.array_equal(keys[o], ref_keys) and np.array_equal(masks[o], ref_masks)
        union = np.sort(np.concatenate([res[r][rep][3] for r in range(world)]))
        assert np.array_equal(union, ref_rdbg)


def _cli_rank(rank, world, port, q, argv, chunk, cwd, dbg_chunk=2 ** 33, stream=None):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from pangenome_amd import dist as pdist
    os.chdir(cwd)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = io.StringIO()
    try:
        kw = {} if stream is None else {"stream_bases": stream[0], "compact_at": stream[1]}
        pdist.entry_point(argv, out=out, device=torch.device("cuda", 0), dev_index=0, edge_chunk=chunk,
                          dbg_chunk=dbg_chunk, **kw)
    finally:
        dist.destroy_process_group()
    q.put((rank, out.getvalue()))


def rows_of(text):
    return [ln for ln in text.split("\n") if len(ln.split("\t")) == 5 and ln.split("\t")[3] in ("+", "-")]


def _run(tmp_path, world, argv, chunk=2 ** 33, dbg_chunk=2 ** 33, stream=None):
    outs = spawn_ranks(world, _cli_rank, (argv, chunk, str(tmp_path), dbg_chunk, stream))
    assert all(rows_of(outs[r]) == [] for r in range(1, world))
    return outs[0]


def _check_dump(path, dbg_keys, dbg_masks, dbg_counts, params=None):
    z = np.load(path)
    sel = z["counts"] > 0
    o = np.argsort(z["keys"][sel], kind="stable")
    assert np.array_equal(z["keys"][sel][o], dbg_keys)
    assert np.array_equal(z["values"][sel][o], dbg_masks)
    assert np.array_equal(z["counts"][sel][o], dbg_counts)
    if params is not None:
        assert z["parameters"].tolist() == params.tolist()


@pytest.mark.parametrize("name,world", [("pan8_k27_c3", 2), ("pan8_k27_n", 3), ("pan8_k27_chunk", 2),
                                        ("edge_k27", 3), ("pan8_k27_mcl", 2)])
def test_dist_cli_vs_reference(name, world, tmp_path):
    fx = Fixture(name)
    q = tmp_path / "input.fsa"
    q.write_bytes(fx.fasta)
    (tmp_path / "input.fsa_rdbg_weight.xyz.mcl").write_text(fx.mcl)
    argv = ["kmer_numba.py", "-i", str(q), "-k", str(fx.k), "-c", str(fx.c)]
    if fx.ns is not None:
        argv += ["-n", str(fx.meta["n"])]
    text = _run(tmp_path, world, argv, fx.edge_chunk)
    assert (tmp_path / "input.fsa_rdbg_weight.xyz").read_text() == fx.xyz
    assert rows_of(text) == fx.rows
    _check_dump(str(q) + "_db.npz", fx.dbg_keys, fx.dbg_masks, fx.dbg_counts, fx.db_params)


# the streaming exchange (dist.exchange_stream, SURVEY 8(e)'s C5 form) with
# tiny chunks: (stream_bases, compact_at) -> every few records a chunk, the
# owner log compacted through pg_dbg_merge + pg_dbg_partition(1)
STREAMS = [(20_000, 1), (60_000, 1 << 26)]


@pytest.mark.parametrize("name,world,stream", [("pan8_k27_c3", 2, STREAMS[0]), ("pan8_k27_n", 3, STREAMS[0]),
                                               ("pan8_k27_chunk", 2, STREAMS[1]), ("edge_k27", 2, (1, 1))])
def test_dist_cli_streamed_vs_reference(name, world, stream, tmp_path):
    fx = Fixture(name)
    q = tmp_path / "input.fsa"
    q.write_bytes(fx.fasta)
    (tmp_path / "input.fsa_rdbg_weight.xyz.mcl").write_text(fx.mcl)
    argv = ["kmer_numba.py", "-i", str(q), "-k", str(fx.k), "-c", str(fx.c)]
    if fx.ns is not None:
        argv += ["-n", str(fx.meta["n"])]
    text = _run(tmp_path, world, argv, fx.edge_chunk, stream=stream)
    assert (tmp_path / "input.fsa_rdbg_weight.xyz").read_text() == fx.xyz
    assert rows_of(text) == fx.rows
    _check_dump(str(q) + "_db.npz", fx.dbg_keys, fx.dbg_masks, fx.dbg_counts, fx.db_params)


def test_dist_cli_streamed_resume_and_checkpoints(tmp_path):
    """Streamed: a -r resume (rank 0's staged checkpoint slots go into the
    first chunk only) and a run writing <in>_db_brkpt.npz from chunked
    builds, both against the reference's own files."""
    fx = ResumeFixture("pan8_k27_r")
    q = tmp_path / "input.fsa"
    q.write_bytes(fx.fasta)
    (tmp_path / "input.fsa_rdbg_weight.xyz.mcl").write_text("")
    text = _run(tmp_path, 2, ["kmer_numba.py", "-i", str(q), "-k", str(fx.k), "-c", str(fx.c), fx.flag, fx.brkpt],
                stream=STREAMS[0])
    assert (tmp_path / "input.fsa_rdbg_weight.xyz").read_text() == fx.xyz
    assert rows_of(text) == fx.rows
    if fx.graph is not None:
        _check_dump(str(q) + "_db.npz", fx.graph["dbg_keys"], fx.graph["dbg_masks"], fx.graph["dbg_counts"])
    d2 = tmp_path / "ck"
    d2.mkdir()
    q2 = d2 / "input.fsa"
    q2.write_bytes(fx.fasta)
    (d2 / "input.fsa_rdbg_weight.xyz.mcl").write_text("")
    _run(d2, 2, ["kmer_numba.py", "-i", str(q2), "-k", "27", "-c", "3"], chunk=30000, dbg_chunk=100000,
         stream=STREAMS[0])
    z, ref = np.load(str(q2) + "_db_brkpt.npz"), np.load(fx.brkpt)
    assert z["parameters"].tolist() == ref["parameters"].tolist()
    sel, rsel = z["counts"] > 0, ref["counts"] > 0
    o, ro = np.argsort(z["keys"][sel], kind="stable"), np.argsort(ref["keys"][rsel], kind="stable")
    for a in ("keys", "values", "counts"):
        assert np.array_equal(z[a][sel][o], ref[a][rsel][ro]), a


def test_dist_cli_reload_d_and_D(tmp_path):
    """-d reloads the dump the distributed run wrote; -D an rdBG key file."""
    from dist_util import oak_place
    from pangenome_amd import host
    fx = Fixture("pan8_k27_c3")
    q = tmp_path / "input.fsa"
    q.write_bytes(fx.fasta)
    (tmp_path / "input.fsa_rdbg_weight.xyz.mcl").write_text("")
    base = ["kmer_numba.py", "-i", str(q), "-k", "27", "-c", "3"]
    assert rows_of(_run(tmp_path, 2, base)) == fx.rows
    text = _run(tmp_path, 2, base + ["-d", str(q) + "_db.npz"])
    assert "load dBG from disk" in text.split("\n") and rows_of(text) == fx.rows
    keys = fx.rdbg_keys
    M = 1048583
    kk, vv, cc = oak_place(keys, np.full(keys.shape[0], 7, np.uint16), np.ones(keys.shape[0], np.uint8), M)
    host.write_db_npz(str(tmp_path / "rdbg"), M, keys.shape[0], kk, vv, cc)
    assert rows_of(_run(tmp_path, 3, base + ["-D", str(tmp_path / "rdbg.npz")])) == fx.rows


@pytest.mark.parametrize("name", __import__("golden_util").resume_names())
def test_dist_cli_resumes_reference_checkpoint(name, tmp_path):
    fx = ResumeFixture(name)
    q = tmp_path / "input.fsa"
    q.write_bytes(fx.fasta)
    (tmp_path / "input.fsa_rdbg_weight.xyz.mcl").write_text("")
    text = _run(tmp_path, 2, ["kmer_numba.py", "-i", str(q), "-k", str(fx.k), "-c", str(fx.c), fx.flag, fx.brkpt])
    assert (tmp_path / "input.fsa_rdbg_weight.xyz").read_text() == fx.xyz
    assert rows_of(text) == fx.rows
    if fx.graph is not None:
        _check_dump(str(q) + "_db.npz", fx.graph["dbg_keys"], fx.graph["dbg_masks"], fx.graph["dbg_counts"])


def test_dist_cli_empty_shard_vs_oracle(oracle_mod, tmp_path):
    """Two records over three ranks: one rank's shard is empty."""
    from oracle import oracle
    from pangenome_amd import synth
    fasta = synth.pangenome(2, 5000, snp=0.01, seed=3)
    q = tmp_path / "input.fsa"
    q.write_bytes(fasta)
    (tmp_path / "input.fsa_rdbg_weight.xyz.mcl").write_text("")
    text = _run(tmp_path, 3, ["kmer_numba.py", "-i", str(q), "-k", "27", "-c", "3"])
    ref = oracle.run_pipeline(fasta, 27, 3)
    assert (tmp_path / "input.fsa_rdbg_weight.xyz").read_text() == ref["xyz"]
    assert rows_of(text) == ref["rows"]


def test_torchrun_launch(tmp_path):
    """The launch line itself: `python -m torch.distributed.run --nproc-per-node 2
    -m pangenome_amd ...` (gloo, both ranks on cuda:0 for this one-GPU box)."""
    import subprocess
    fx = Fixture("pan8_k27_c2")
    q = tmp_path / "input.fsa"
    q.write_bytes(fx.fasta)
    (tmp_path / "input.fsa_rdbg_weight.xyz.mcl").write_text("")
    from dist_util import free_port
    env = dict(os.environ, PG_DIST_BACKEND="gloo", PG_DIST_ONE_GPU="1", PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           "-m", "pangenome_amd", "-i", str(q), "-k", "27", "-c", "2"]
    p = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    assert rows_of(p.stdout) == fx.rows
    assert (tmp_path / "input.fsa_rdbg_weight.xyz").read_text() == fx.xyz


def test_dist_cli_writes_reference_checkpoints(tmp_path):
    """The sharded CLI with passes crossing their chunk leaves the
    <in>_db_brkpt.npz (dBG chunk 100000, :1255-1259) and <in>_rdb_brkpt.npz
    (edge chunk 30000, :1880-1887) the reference itself wrote
    (tests/golden/resume), and still prints the reference's rows."""
    fr, fR = ResumeFixture("pan8_k27_r"), ResumeFixture("pan8_k27_R")
    assert (fr.meta["chunk"], fR.meta["chunk"], fr.c, fR.c) == (100000, 30000, 3, 3)
    q = tmp_path / "input.fsa"
    q.write_bytes(fr.fasta)
    (tmp_path / "input.fsa_rdbg_weight.xyz.mcl").write_text("")
    text = _run(tmp_path, 2, ["kmer_numba.py", "-i", str(q), "-k", "27", "-c", "3"], chunk=30000, dbg_chunk=100000)
    assert rows_of(text) == fR.rows
    z, ref = np.load(str(q) + "_db_brkpt.npz"), np.load(fr.brkpt)
    assert z["parameters"].tolist() == ref["parameters"].tolist()
    sel, rsel = z["counts"] > 0, ref["counts"] > 0
    o, ro = np.argsort(z["keys"][sel], kind="stable"), np.argsort(ref["keys"][rsel], kind="stable")
    for a in ("keys", "values", "counts"):
        assert np.array_equal(z[a][sel][o], ref[a][rsel][ro]), a
    z, ref = np.load(str(q) + "_rdb_brkpt.npz"), np.load(fR.brkpt)
    for a in ("parameters", "keys", "values"):
        assert z[a].tolist() == ref[a].tolist(), a


def _budget_rank(rank, world, port, q, fasta, mode, cap):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from pangenome_amd._lib import PG_TUNE_DEVICE_CAP, PangenomeError, load
    from pangenome_amd.dist import GpuShard, exchange_and_reduce, exchange_stream, stream_chunks
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    sh = GpuShard(27, 0)
    meta = sh.load(np.frombuffer(fasta, np.uint8))
    R = meta["seq_len"].shape[0]
    sh.ctx.tune(PG_TUNE_DEVICE_CAP, cap)                   # (restarts the peak)
    try:
        if mode == "whole":
            sentinel = sh.build(np.ones(R, np.uint8), 0, True)
            res = exchange_and_reduce(sh, world, rank, dev, sentinel)
            keys = sh.owner_rdbg()
        else:
            chunks = stream_chunks(np.ones(R, np.uint8), meta["seq_len"], int(meta["seq_len"][0]))
            res = exchange_stream(sh, world, rank, dev, chunks, R, True, compact_at=1)
            keys = res[5]
        q.put((rank, ("ok", res[0], res[1], np.sort(keys), int(load().pg_device_bytes(1)))))
    except PangenomeError as e:
        q.put((rank, ("error", str(e))))
    finally:
        sh.ctx.tune(PG_TUNE_DEVICE_CAP, 0)
        dist.destroy_process_group()


def test_streamed_exchange_device_budget(oracle_mod):
    """ADVICE r2 (the C5 form's memory): the streamed exchange keeps the
    owner's record log in sub-logs and merges one at a time, so the
    library's device buffers stay near one chunk's build instead of the whole
    shard's.  At a scaled-down size (16 x 200 kbp at 1 % SNP, one genome per
    chunk): both forms give the oracle's dBG / rdBG; the streamed one peaks
    lower; under a device cap between the two peaks (PG_TUNE_DEVICE_CAP) the
    streamed run still completes and the whole-shard build fails with
    PG_ENOMEM."""
    from pangenome_amd import synth
    fasta = synth.pangenome(16, 200_000, snp=0.01, indel=1e-3, seed=31)
    ref = oracle_mod.OracleRun(fasta, 27, 2)
    n_dbg, rdbg = ref.dbg()[0].shape[0], ref.rdbg()
    whole = spawn_ranks(1, _budget_rank, (fasta, "whole", 0))[0]
    strm = spawn_ranks(1, _budget_rank, (fasta, "stream", 0))[0]
    for r in (whole, strm):
        assert r[0] == "ok", r
        assert (r[1], r[2]) == (n_dbg, rdbg.shape[0])
        assert np.array_equal(r[3], rdbg)
    assert strm[4] < whole[4], (strm[4], whole[4])
    cap = (strm[4] + whole[4]) // 2
    capped = spawn_ranks(1, _budget_rank, (fasta, "stream", cap))[0]
    assert capped[0] == "ok" and np.array_equal(capped[3], rdbg), capped[:2]
    failed = spawn_ranks(1, _budget_rank, (fasta, "whole", cap))[0]
    assert failed[0] == "error" and "device memory cap" in failed[1], failed

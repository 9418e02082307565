"""C5's form on one GPU: SURVEY 8(d)'s C5 workload (10 x 3 Gbp genomes written
as 125 Mbp records, 1 % SNP, 0.1 % indel; pangenome_amd/synth.c5_record) and
8(e)'s streamed owner exchange (dist.exchange_stream), which a C5 shard of
3.75 Gbp per GPU needs because its whole local table does not fit beside the
owner partition.

* ``c5s`` (records 0-1 of genomes 0-1 in the file's genome-major order,
  0.5 Gbp, 725 M dBG keys — far less redundant than C3: two distinct 125 Mbp
  segments, each twice at 1 % SNP): the whole build and the streamed exchange
  at world 1 (one record per chunk, a compaction after every chunk) against
  the oracle's digest (tests/golden/scale/c5s.json: n_dbg, n_rdbg, SHA-256 of
  the sorted dBG and rdBG).  Over gloo (host-staged collectives) and over the
  nccl backend, i.e. RCCL's all_to_all_single on device buffers with one rank.
* ``c5m`` (genome 0's records 0-7, then genome 1's 0-1: 1.25 Gbp, ~2.3 G dBG
  keys): the streamed exchange at the production chunk size, 2^30 forward
  bases, so the first round builds 8 records (1.0 Gbp) at once — the shape
  whose counts came back wrong in round 4 — against the oracle's digest
  (tests/golden/scale/c5m.json, digested key range by key range:
  make_scale_digests.py).  Three forms: the rank's own run as a device copy
  (the product path), through RCCL (PG_EXCHANGE_SELF_RCCL=1: at world 1
  every byte of the ~37 GB exchanged crosses RCCL in 512 MiB pieces), and
  with every new library and exchange buffer poisoned (PG_TUNE_POISON 0xA5:
  a read of memory no kernel wrote changes the result).  Plus the whole
  1.25 Gbp build in one table, dBG SHA-256 included.
* the C5 shard one rank holds at N = 8 (3.75 Gbp: genome 0's 24 records and
  genome 1's first 6, 3.8 GB of FASTA; ~1 min: 17 s to generate, ~1 s per
  streamed build): against the oracle's digest of it
  (tests/golden/scale/c5shard.json, key ranges as for c5m) at 2^30 bases per
  chunk over RCCL and at 2^29 as a device copy; the dBG is closed under
  reverse complement (no N and odd k: n_dbg is even).  PG_RUN_C5_GLOO=1 adds
  the ~30 s gloo run.

Every exchange runs with dist.py's integrity checks (per-run sums of the
exchanged records from the sender's scatter to the owner's merge, record
conservation): a record changed anywhere on the way raises instead of
giving a wrong count.
"""
import json
import os
import sys
import time

import numpy as np
import pytest

from dist_util import ROOT, spawn_ranks
from scale_util import load_digest

pytestmark = pytest.mark.gpu
TESTS = os.path.dirname(os.path.abspath(__file__))


def _c5_rank(rank, world, port, q, path, backend, chunk_bases, compact_at, whole, subparts, form="copy"):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, TESTS)
    if form == "rccl":
        os.environ["PG_EXCHANGE_SELF_RCCL"] = "1"       # (read when dist is imported)
    if form == "poison":
        os.environ["PG_DEBUG_POISON"] = "0xA5"
    import torch
    import torch.distributed as dist
    from pangenome_amd import kmer
    from pangenome_amd.dist import GpuShard, exchange_stream, stream_chunks
    from scale_util import dbg_digest, rdbg_digest
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    out = {"backend": dist.get_backend()}
    sh = GpuShard(27, 0)
    if form == "poison":
        from pangenome_amd._lib import PG_TUNE_POISON
        sh.ctx.tune(PG_TUNE_POISON, 0xA5)
    out["form"] = form
    from pangenome_amd import dist as pdist
    out["self_copy"] = pdist.SELF_COPY
    if os.environ.get("PG_TEST_K3_COVER"):          # (tools/c5_forms.py: the coverage form under test)
        from pangenome_amd._lib import PG_TUNE_K3_COVER
        sh.ctx.tune(PG_TUNE_K3_COVER, int(os.environ["PG_TEST_K3_COVER"]))
    t0 = time.time()
    meta = sh.load(kmer.seq2bytes(path))
    R = int(meta["seq_len"].shape[0])
    out["records"], out["bases"] = R, int(meta["seq_len"].sum())
    out["parse_s"] = time.time() - t0
    print("c5 rank: %s parsed %d records, %d bases in %.1f s" % (backend, R, out["bases"], out["parse_s"]), flush=True)
    if whole:
        t0 = time.time()
        st = sh.ctx.build_dbg(np.ones(R, np.uint8), 0, True)
        st = sh.ctx.build_rdbg()
        out["whole_s"] = time.time() - t0
        keys, masks = sh.ctx.dbg()
        out["whole"] = [int(st.n_dbg), int(st.n_rdbg), dbg_digest(keys, masks), rdbg_digest(sh.ctx.rdbg())]
        del keys, masks
        if whole == "only":
            q.put((rank, out))
            dist.barrier()
            dist.destroy_process_group()
            return
    t0 = time.time()
    chunks = stream_chunks(np.ones(R, np.uint8), meta["seq_len"], chunk_bases)
    lib = {}
    res = exchange_stream(sh, world, rank, dev, chunks, R, True, compact_at=compact_at, subparts=subparts,
                          routed=False if form == "local" else None, lib_stats=lib)
    out["stream_s"] = time.time() - t0
    out["routed"] = bool(lib)
    out["stream"] = [int(res[0]), int(res[1]), int(res[4]), rdbg_digest(np.sort(res[5]))]
    print("c5 rank: %s streamed in %.1f s: %s" % (backend, out["stream_s"], out["stream"][:3]), flush=True)
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


@pytest.fixture(scope="module")
def c5s_file(tmp_path_factory):
    from pangenome_amd import synth
    dg = load_digest("c5s")
    assert dg is not None, "tests/golden/scale/c5s.json missing (make_scale_digests.py c5s)"
    p = str(tmp_path_factory.mktemp("c5") / "c5s.fa")
    n = synth.write_c5(p, pairs=[(g, r) for g in (0, 1) for r in (0, 1)], workers=4)
    assert n == dg["fasta_bytes"]
    return p, dg


@pytest.mark.timeout(900)
@pytest.mark.parametrize("backend,form", [("gloo", "local"), ("nccl", "local"), ("nccl", "copy")])
def test_c5_form_streamed_vs_oracle_digest(c5s_file, backend, form):
    """The local-table form (compaction after every chunk) and the routed
    form (stage A records straight to the owner's sub-logs)."""
    path, dg = c5s_file
    out = spawn_ranks(1, _c5_rank, (path, backend, 125_000_000, 1 if form == "local" else None, backend == "gloo",
                                    None, form), timeout=600)[0]
    assert out["backend"] == backend and out["routed"] == (form != "local")
    assert (out["records"], out["bases"]) == (4, dg["n_bases"])
    if "whole" in out:
        assert out["whole"] == [dg["n_dbg"], dg["n_rdbg"], dg["dbg_sha256"], dg["rdbg_sha256"]]
    n_dbg, n_rdbg, rounds, rsha = out["stream"]
    assert rounds == 4
    assert (n_dbg, n_rdbg, rsha) == (dg["n_dbg"], dg["n_rdbg"], dg["rdbg_sha256"])


@pytest.fixture(scope="module")
def c5m_file(tmp_path_factory):
    from pangenome_amd import synth
    from scale_util import INPUTS
    dg = load_digest("c5m")
    assert dg is not None, "tests/golden/scale/c5m.json missing (make_scale_digests.py c5m)"
    p = str(tmp_path_factory.mktemp("c5m") / "c5m.fa")
    n = synth.write_c5(p, pairs=INPUTS["c5m"]["pairs"], workers=10)
    assert n == dg["fasta_bytes"]
    return p, dg


@pytest.mark.timeout(900)
@pytest.mark.parametrize("form", ["copy", "rccl", "poison", "local"])
def test_c5m_streamed_at_2p30_vs_oracle_digest(c5m_file, form):
    """The streamed exchange at 2^30 forward bases per chunk (round 1 builds 8
    records of 125 Mbp at once) against the oracle: the product path (routed:
    at world 1 the scatter's buffer is the owner's log), RCCL carrying the
    rank's own run, poisoned buffers, and the local-table form."""
    path, dg = c5m_file
    out = spawn_ranks(1, _c5_rank, (path, "nccl", 1 << 30, None, False, None, form), timeout=800)[0]
    print("c5m %s: %s" % (form, json.dumps(out, sort_keys=True)))
    assert out["self_copy"] == (form != "rccl")
    assert out["routed"] == (form != "local")
    assert (out["records"], out["bases"]) == (10, dg["n_bases"])
    n_dbg, n_rdbg, rounds, rsha = out["stream"]
    assert rounds == 2
    assert (n_dbg, n_rdbg, rsha) == (dg["n_dbg"], dg["n_rdbg"], dg["rdbg_sha256"])


@pytest.mark.timeout(900)
def test_c5m_whole_build_vs_oracle_digest(c5m_file):
    """The 1.25 Gbp of c5m in one table (2^31 buckets), dBG SHA-256 included."""
    path, dg = c5m_file
    out = spawn_ranks(1, _c5_rank, (path, "nccl", 1 << 30, None, "only", None), timeout=800)[0]
    assert out["whole"] == [dg["n_dbg"], dg["n_rdbg"], dg["dbg_sha256"], dg["rdbg_sha256"]]


@pytest.mark.timeout(900)
def test_c5_shard_full_size_vs_oracle_digest(tmp_path):
    from pangenome_amd import synth
    from scale_util import INPUTS
    dg = load_digest("c5shard")
    assert dg is not None, "tests/golden/scale/c5shard.json missing (make_scale_digests.py c5shard)"
    p = str(tmp_path / "c5_shard0.fa")
    t0 = time.time()
    nbytes = synth.write_c5(p, pairs=INPUTS["c5shard"]["pairs"], workers=10)
    assert nbytes == dg["fasta_bytes"]
    print("c5 shard: %d bytes generated in %.0f s" % (nbytes, time.time() - t0), flush=True)
    forms = [("nccl_2^30_rccl", "nccl", 1 << 30, "rccl"), ("nccl_2^29_copy", "nccl", 1 << 29, "copy"),
             ("nccl_2^30_local", "nccl", 1 << 30, "local")]
    if os.environ.get("PG_RUN_C5_GLOO") == "1":
        forms += [("gloo_2^30", "gloo", 1 << 30, "copy")]
    runs = {}
    for tag, backend, chunk, form in forms:
        runs[tag] = spawn_ranks(1, _c5_rank, (p, backend, chunk, None, False, None, form), timeout=800)[0]
        print("c5 shard %s: %s" % (tag, json.dumps(runs[tag], sort_keys=True)), flush=True)
    a, b = runs["nccl_2^30_rccl"], runs["nccl_2^29_copy"]
    assert a["records"] == 30 and a["bases"] == dg["n_bases"]
    assert a["stream"][2] == 4 and b["stream"][2] == 8 and runs["nccl_2^30_local"]["stream"][2] == 4
    assert a["routed"] and b["routed"] and not runs["nccl_2^30_local"]["routed"]
    for r in runs.values():
        assert [r["stream"][0], r["stream"][1], r["stream"][3]] == [dg["n_dbg"], dg["n_rdbg"], dg["rdbg_sha256"]]
    # both strands of every window, no N, odd k: closed under reverse complement
    assert a["stream"][0] % 2 == 0 and a["stream"][1] > 0

"""Parity at benchmark scale: the default (no-knob) production path on the exact
C3 and C2 inputs bench.py measures, against digests of the pinned oracle's
results (tests/golden/make_scale_digests.py -> tests/golden/scale/*.json).

C3 is too slow for the oracle inside a test (minutes of one core), so the
oracle ran once in the build container and its dBG / rdBG are compared here
through SHA-256 digests of the sorted arrays (bit-exact, any difference in any
key or mask changes them).  C2 (one 4.64 Mbp record) is also walked: `.xyz`
and region rows with an empty `.mcl`.
"""
import io
import os

import numpy as np
import pytest

from scale_util import dbg_digest, load_digest, make_input, rdbg_digest, text_digest

pytestmark = pytest.mark.gpu

_INPUTS = {}


def _input(name):
    if name not in _INPUTS:
        _INPUTS.clear()                       # one C3-sized input in host memory at a time
        _INPUTS[name] = make_input(name)
    return _INPUTS[name]


def _check_graph(ctx, st, dg):
    assert st.n_bases == dg["n_bases"]
    assert (st.n_dbg, st.n_rdbg) == (dg["n_dbg"], dg["n_rdbg"])
    keys, masks = ctx.dbg()
    assert keys.shape[0] == dg["n_dbg"]
    assert dbg_digest(keys, masks) == dg["dbg_sha256"]
    del keys, masks
    assert rdbg_digest(ctx.rdbg()) == dg["rdbg_sha256"]


@pytest.mark.parametrize("name", ["c3a", "c3b"])
def test_c3_default_path_vs_oracle_digest(name):
    """pg_build (K5 behind K3) twice on device-resident input — the bench's
    exact call sequence — then the two-call pg_build_dbg + pg_build_rdbg path
    on host input, all against the oracle's digest."""
    import torch
    from pangenome_amd._lib import Context
    dg = load_digest(name)
    assert dg is not None, "tests/golden/scale/%s.json missing (make_scale_digests.py)" % name
    fasta = _input(name)
    assert len(fasta) == dg["fasta_bytes"]
    d = torch.frombuffer(bytearray(fasta), dtype=torch.uint8).to("cuda:0")
    torch.cuda.synchronize()
    ctx = Context(27)
    for _ in range(2):                        # cold, then warm (learned sizes, cached tiles)
        ctx.set_fasta_device(d.data_ptr(), d.numel(), keepalive=d)
        ctx.parse()
        st = ctx.build(None, 0, True)
        _check_graph(ctx, st, dg)
    ctx.close()
    del d
    two = Context(27)
    two.set_fasta(fasta)
    two.parse()
    two.build_dbg(None, 0, True)
    st = two.build_rdbg()
    _check_graph(two, st, dg)
    two.close()


def test_c3_alternating_batches():
    """The bench's steady state: one context fed batch A, B, A, B; every
    build against its own oracle digest (nothing carried over is allowed to
    change a result)."""
    import torch
    from pangenome_amd._lib import Context
    digests = [load_digest("c3a"), load_digest("c3b")]
    devs = []
    for name in ("c3a", "c3b"):
        fasta = make_input(name)
        devs.append(torch.frombuffer(bytearray(fasta), dtype=torch.uint8).to("cuda:0"))
        del fasta
    torch.cuda.synchronize()
    ctx = Context(27)
    for i in range(4):
        d, dg = devs[i % 2], digests[i % 2]
        ctx.set_fasta_device(d.data_ptr(), d.numel(), keepalive=d)
        ctx.parse()
        st = ctx.build(None, 0, True)
        assert (st.n_dbg, st.n_rdbg) == (dg["n_dbg"], dg["n_rdbg"])
        assert rdbg_digest(ctx.rdbg()) == dg["rdbg_sha256"]
    keys, masks = ctx.dbg()
    assert dbg_digest(keys, masks) == digests[1]["dbg_sha256"]
    ctx.close()


def test_c2_pipeline_vs_oracle_digest(tmp_path):
    """C2 (one long record: no dedup reference) through the CLI passes:
    dBG, rdBG, `.xyz` and rows (empty `.mcl`)."""
    from pangenome_amd import kmer
    dg = load_digest("c2")
    fasta = make_input("c2")
    q = tmp_path / "c2.fa"
    q.write_bytes(fasta)
    (tmp_path / "c2.fa_rdbg_weight.xyz.mcl").write_text("")
    g = kmer.seq2rdbg(str(q), 27, 5, 2 ** 63, brkpt="", chunk=2 ** 33, rc=True)
    keys, masks = g.dbg_items()
    assert keys.shape[0] == dg["n_dbg"]
    assert dbg_digest(keys, masks) == dg["dbg_sha256"]
    kmer.dbg2rdbg(g)
    assert rdbg_digest(g.rdbg_keys()) == dg["rdbg_sha256"]
    out = io.StringIO()
    kmer.seq2graph(str(q), kmer=27, bits=5, Ns=2 ** 63, rdbg_dict=g, chunk=2 ** 33, brkpt="", rc=False, out=out)
    xyz = open(str(q) + "_rdbg_weight.xyz").read()
    assert text_digest(xyz) == dg["xyz_sha256"]
    rows = [ln for ln in out.getvalue().split("\n") if ln.count("\t") == 4]
    assert len(rows) == dg["n_rows"]
    assert text_digest("".join(x + "\n" for x in rows)) == dg["rows_sha256"]


class _Out:
    """stdout stand-in: `#` lines through write(), row text through .buffer -
    in memory, or a file (a descriptor: the rows go to it from the device)."""

    def __init__(self, path=None):
        import io
        self.buffer = io.BytesIO() if path is None else open(path, "w+b")
        self.lines = []

    def write(self, s):
        self.lines.append(s)
        self.buffer.write(s.encode())

    def flush(self):
        self.buffer.flush()

    def getvalue(self):
        if hasattr(self.buffer, "getvalue"):
            return self.buffer.getvalue()
        self.buffer.flush()
        self.buffer.seek(0)
        return self.buffer.read()


@pytest.mark.parametrize("name", ["c3a_c2", "c3a_c3"])
def test_c3_cli_region_table_vs_oracle_digest(tmp_path, name):
    """The whole CLI (kmer.entry_point: dBG, `<in>_db.npz`, rdBG, edges, `.xyz`,
    labels from an empty `.mcl`, region rows) on C3 batch A at -c 2 and -c 3,
    against the oracle's digests of the `.xyz` text and the region rows
    (seq2graph :1853-1951, rdbg_edge_weight :1446-1518, seq2path_jit_
    :1523-1573 on 100 records and 1.93 M rdBG keys).  The stage times the CLI
    prints go to $PG_TIMING_LOG when set."""
    import json
    import time
    from pangenome_amd import kmer
    dg = load_digest(name)
    assert dg is not None, "tests/golden/scale/%s.json missing (make_scale_digests.py)" % name
    fasta = _input("c3a")
    assert len(fasta) == dg["fasta_bytes"]
    q = tmp_path / "c3.fa"
    q.write_bytes(fasta)
    (tmp_path / "c3.fa_rdbg_weight.xyz.mcl").write_text("")
    out = _Out(tmp_path / "stdout.txt" if dg["c"] == 2 else None)   # -c 2: rows to a descriptor
    t0 = time.time()
    kmer.entry_point(["kmer_numba.py", "-i", str(q), "-k", "27", "-c", str(dg["c"])], out=out)
    wall = time.time() - t0
    text = out.getvalue()
    lines = text.split(b"\n")
    rows = [ln for ln in lines if ln.count(b"\t") == 4]
    assert len(rows) == dg["n_rows"]
    assert text_digest(b"".join(x + b"\n" for x in rows)) == dg["rows_sha256"]
    xyz = (tmp_path / "c3.fa_rdbg_weight.xyz").read_bytes()
    assert xyz.count(b"\n") == dg["n_edges"]
    assert text_digest(xyz) == dg["xyz_sha256"]
    # stage times: each "# finished in X seconds" follows its stage's name
    stages, cur = {}, None
    for ln in lines:
        if ln.startswith(b"# finished in"):
            stages[cur] = float(ln.split()[3])
        elif ln.startswith(b"#"):
            cur = ln[2:].decode()
    log = os.environ.get("PG_TIMING_LOG")
    if log:
        with open(log, "a") as f:
            f.write(json.dumps({"test": name, "stages_s": stages, "cli_wall_s": round(wall, 3),
                                "n_edges": dg["n_edges"], "n_rows": dg["n_rows"]}) + "\n")


def test_c4_past_4gib_vs_oracle_digest(tmp_path):
    """C4 (1000 x 5 Mbp, 5.08 GB of FASTA: byte offsets, class-stream offsets
    and record regions past 2^32) on one MI355X through the CLI's dBG pass
    (kmer.seq2rdbg: the file memory-mapped, staged through the pinned ring,
    pg_build_host), then the rdBG; n_dbg / n_rdbg and the SHA-256 of the sorted
    dBG and rdBG against the oracle's digest (tests/golden/scale/c4.json, 31
    min of one core in the build container).  The FASTA is written by
    `python -m pangenome_amd.synth c4` (spawned workers, ~20 s), or taken from
    $PG_C4_FASTA."""
    import subprocess
    import sys
    import time
    from pangenome_amd import kmer
    dg = load_digest("c4")
    assert dg is not None, "tests/golden/scale/c4.json missing (make_scale_digests.py c4)"
    path = os.environ.get("PG_C4_FASTA")
    if not path or not os.path.isfile(path):
        path = str(tmp_path / "c4.fa")
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        subprocess.run([sys.executable, "-m", "pangenome_amd.synth", "c4", path, "16"], cwd=root, check=True,
                       timeout=600)
    assert os.path.getsize(path) == dg["fasta_bytes"] > 2 ** 32
    t0 = time.time()
    g = kmer.seq2rdbg(path, 27, 5, 2 ** 63, brkpt="", chunk=2 ** 33, rc=True)
    build_s = time.time() - t0
    assert g.stats.n_bases == dg["n_bases"]
    assert (g.stats.n_dbg, g.stats.n_rdbg) == (dg["n_dbg"], dg["n_rdbg"])
    keys, masks = g.dbg_items()
    assert dbg_digest(keys, masks) == dg["dbg_sha256"]
    del keys, masks
    kmer.dbg2rdbg(g)
    assert rdbg_digest(g.rdbg_keys()) == dg["rdbg_sha256"]
    log = os.environ.get("PG_TIMING_LOG")
    if log:
        import json
        with open(log, "a") as f:
            f.write(json.dumps({"test": "c4", "seq2rdbg_s": round(build_s, 3), "n_dbg": dg["n_dbg"],
                                "n_rdbg": dg["n_rdbg"], "n_records_a": g.stats.n_records_a}) + "\n")
    g.ctx.close()

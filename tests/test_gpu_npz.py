"""npz persistence (dump / load_on_disk, kmer_numba.py:243-335) on the GPU.

The dumped `<in>_db.npz` is compared with the dump the reference itself wrote
for every golden fixture (its keys / values / counts slots, capacity and
size, tests/golden/graphs/*), and its slot layout is checked with a
restatement of oakht.pointer (:521-538): every key is found by the probe walk
a reference lookup does.  -d, -D and -r then reproduce the reference's region
rows from those files.
"""
import io
import os

import numpy as np
import pytest

from dist_util import oak_place, oak_slot
from golden_util import Fixture, fixture_names

pytestmark = pytest.mark.gpu
def rows_of(text):
    return [ln for ln in text.split("\n") if len(ln.split("\t")) == 5 and ln.split("\t")[3] in ("+", "-")]


def _graph_fixtures():
    seen, out = set(), []
    for n in fixture_names():
        g = Fixture(n).meta["graph"]
        if g not in seen:
            seen.add(g)
            out.append(n)
    return out


@pytest.mark.parametrize("name", _graph_fixtures())
def test_dump_matches_reference_dump(name, tmp_path):
    from pangenome_amd import host, kmer
    fx = Fixture(name)
    q = tmp_path / "input.fsa"
    q.write_bytes(fx.fasta)
    Ns = fx.ns if fx.ns is not None else 2 ** 63
    g = kmer.seq2rdbg(str(q), fx.k, 5, Ns, brkpt="", chunk=2 ** 33, rc=(fx.c >> 1) == 1)
    kmer.dump(g, str(q) + "_db")
    z = np.load(str(q) + "_db.npz")
    params = z["parameters"]
    assert params.tolist() == fx.db_params.tolist()          # capacity, load, size, ksize, vsize, offset
    keys, vals, cnts = z["keys"], z["values"], z["counts"]
    assert keys.dtype == np.uint64 and vals.dtype == np.uint16 and cnts.dtype == np.uint8
    sel = cnts > 0
    o = np.argsort(keys[sel], kind="stable")
    assert np.array_equal(keys[sel][o], fx.dbg_keys)
    assert np.array_equal(vals[sel][o], fx.dbg_masks)
    assert np.array_equal(cnts[sel][o], fx.dbg_counts)
    # the layout: every key sits where oakht.pointer looks for it
    idx = np.flatnonzero(sel)
    sample = idx if idx.shape[0] <= 20000 else idx[np.random.default_rng(0).choice(idx.shape[0], 20000, False)]
    for j in sample.tolist():
        assert oak_slot(keys, cnts, int(keys[j])) == j
    off, k2, v2, c2 = host.read_db_npz(str(q) + "_db.npz")
    assert off == 0 and k2.shape[0] == int(params[2])


@pytest.mark.parametrize("name", _graph_fixtures())
def test_native_dump_file_equals_host_write(name, tmp_path):
    """pg_dbg_dump_fd (slot arrays streamed from the device into the file,
    kmer.dump) writes what pg_dbg_dump + host.write_db_npz write, byte for
    byte: a valid zip (every CRC), the same parameters and (key, value,
    count) slots, the n<k sentinel's included, each where oakht.pointer looks
    for it.  The slot placement is deterministic (the smallest proposing key
    takes a contested slot), so a dump of the same input from a fresh build
    in a fresh context is byte-equal too, and equals the host restatement of
    the placement rule (dist_util.oak_place_rounds)."""
    import zipfile
    from pangenome_amd import host, kmer
    fx = Fixture(name)
    q = tmp_path / "input.fsa"
    q.write_bytes(fx.fasta)
    Ns = fx.ns if fx.ns is not None else 2 ** 63
    g = kmer.seq2rdbg(str(q), fx.k, 5, Ns, brkpt="", chunk=2 ** 33, rc=(fx.c >> 1) == 1)
    kmer.dump(g, str(tmp_path / "a_db"))
    cap, size, keys, vals, cnts = g.ctx.dbg_dump()
    host.write_db_npz(str(tmp_path / "b_db"), cap, size, keys, vals, cnts)
    assert zipfile.ZipFile(str(tmp_path / "a_db.npz")).testzip() is None
    za, zb = np.load(str(tmp_path / "a_db.npz")), np.load(str(tmp_path / "b_db.npz"))
    assert za["parameters"].tolist() == zb["parameters"].tolist()
    ka, va, ca = za["keys"], za["values"], za["counts"]
    kb_, vb, cb = zb["keys"], zb["values"], zb["counts"]
    assert ka.shape == kb_.shape == (cap,) and va.dtype == np.uint16 and ca.dtype == np.uint8
    sa, sb = ca > 0, cb > 0
    oa, ob = np.argsort(ka[sa], kind="stable"), np.argsort(kb_[sb], kind="stable")
    assert np.array_equal(ka[sa][oa], kb_[sb][ob])
    assert np.array_equal(va[sa][oa], vb[sb][ob]) and np.array_equal(ca[sa][oa], cb[sb][ob])
    idx = np.flatnonzero(sa)
    sample = idx if idx.shape[0] <= 5000 else idx[np.random.default_rng(1).choice(idx.shape[0], 5000, False)]
    for j in sample.tolist():
        assert oak_slot(ka, ca, int(ka[j])) == j
    a_bytes = (tmp_path / "a_db.npz").read_bytes()
    assert a_bytes == (tmp_path / "b_db.npz").read_bytes()
    g2 = kmer.seq2rdbg(str(q), fx.k, 5, Ns, brkpt="", chunk=2 ** 33, rc=(fx.c >> 1) == 1)
    kmer.dump(g2, str(tmp_path / "c_db"))
    assert (tmp_path / "c_db.npz").read_bytes() == a_bytes
    if sa.sum() <= 20000:
        from dist_util import oak_place_rounds
        K, V, C = oak_place_rounds(ka[sa], va[sa], ca[sa], cap)
        assert np.array_equal(K, ka) and np.array_equal(V, va) and np.array_equal(C, ca)


def _run_cli(argv):
    from pangenome_amd import kmer
    out = io.StringIO()
    kmer.entry_point(argv, out=out)
    return out.getvalue()


def test_cli_writes_db_npz_and_d_reloads_it(tmp_path):
    fx = Fixture("pan8_k27_c3")
    q = tmp_path / "in.fa"
    q.write_bytes(fx.fasta)
    (tmp_path / "in.fa_rdbg_weight.xyz.mcl").write_text("")
    text = _run_cli(["kmer_numba.py", "-i", str(q), "-k", "27", "-c", "3"])
    assert "# save dBG to disk" in text and rows_of(text) == fx.rows
    db = str(q) + "_db.npz"
    assert os.path.isfile(db)
    text = _run_cli(["kmer_numba.py", "-i", str(q), "-k", "27", "-c", "3", "-d", db])
    assert "load dBG from disk" in text.split("\n")
    assert rows_of(text) == fx.rows


def test_cli_D_loads_an_rdbg(tmp_path):
    """-D: rdBG keys in an oakht file (values are not consulted, :1538 has_key)."""
    fx = Fixture("pan8_k27_c1")
    q = tmp_path / "in.fa"
    q.write_bytes(fx.fasta)
    (tmp_path / "in.fa_rdbg_weight.xyz.mcl").write_text("")
    from pangenome_amd import host
    keys = fx.rdbg_keys
    M = 1048583
    kk, vv, cc = oak_place(keys, np.full(keys.shape[0], 7, np.uint16), np.ones(keys.shape[0], np.uint8), M)
    host.write_db_npz(str(tmp_path / "rdbg"), M, keys.shape[0], kk, vv, cc)
    text = _run_cli(["kmer_numba.py", "-i", str(q), "-k", "27", "-c", "1", "-D", str(tmp_path / "rdbg.npz")])
    assert rows_of(text) == fx.rows


def test_cli_r_resumes_a_checkpoint(tmp_path):
    """-r: the dBG of records 0..3 with the offset seqio reports after record 3
    (:1255-1259); resuming inserts records 4.. and ends at the full dBG, counts
    included, and the reference's rows."""
    from pangenome_amd import host, kmer
    from pangenome_amd._lib import Context
    fx = Fixture("pan8_k27_c3")
    q = tmp_path / "in.fa"
    q.write_bytes(fx.fasta)
    (tmp_path / "in.fa_rdbg_weight.xyz.mcl").write_text("")
    ctx = Context(27)
    ctx.set_fasta(np.frombuffer(fx.fasta, np.uint8))
    R, _ = ctx.parse()
    ptr = ctx.records()["ptr"]
    flags = np.zeros(R, np.uint8)
    flags[:4] = 1
    ctx.build_dbg(flags, 0, True)
    cap, size, keys, vals, cnts = ctx.dbg_dump()
    ctx.close()
    brk = str(tmp_path / "in.fa_db_brkpt")
    host.write_db_npz(brk, cap, size, keys, vals, cnts, offset=int(ptr[3]))
    g = kmer.seq2rdbg(str(q), 27, 5, 2 ** 63, brkpt=brk + ".npz", chunk=2 ** 33, rc=True)
    kmer.dump(g, str(tmp_path / "resumed"))
    z = np.load(str(tmp_path / "resumed.npz"))
    sel = z["counts"] > 0
    o = np.argsort(z["keys"][sel], kind="stable")
    assert np.array_equal(z["keys"][sel][o], fx.dbg_keys)
    assert np.array_equal(z["values"][sel][o], fx.dbg_masks)
    assert np.array_equal(z["counts"][sel][o], fx.dbg_counts)
    text = _run_cli(["kmer_numba.py", "-i", str(q), "-k", "27", "-c", "3", "-r", brk + ".npz"])
    assert rows_of(text) == fx.rows


@pytest.mark.parametrize("name", __import__("golden_util").resume_names())
def test_cli_resumes_reference_checkpoint(name, tmp_path):
    """-r / -R from a checkpoint the reference wrote itself: same .xyz (edge
    order included), rows and, for -r, the dumped dBG."""
    from golden_util import ResumeFixture
    fx = ResumeFixture(name)
    q = tmp_path / "input.fsa"
    q.write_bytes(fx.fasta)
    (tmp_path / "input.fsa_rdbg_weight.xyz.mcl").write_text("")
    text = _run_cli(["kmer_numba.py", "-i", str(q), "-k", str(fx.k), "-c", str(fx.c), fx.flag, fx.brkpt])
    assert (tmp_path / "input.fsa_rdbg_weight.xyz").read_text() == fx.xyz
    assert rows_of(text) == fx.rows
    if fx.graph is not None:
        z = np.load(str(q) + "_db.npz")
        sel = z["counts"] > 0
        o = np.argsort(z["keys"][sel], kind="stable")
        assert np.array_equal(z["keys"][sel][o], fx.graph["dbg_keys"])
        assert np.array_equal(z["values"][sel][o], fx.graph["dbg_masks"])
        assert np.array_equal(z["counts"][sel][o], fx.graph["dbg_counts"])


@pytest.mark.parametrize("name", __import__("golden_util").resume_names())
def test_writes_reference_checkpoint(name, tmp_path):
    """The mid-run checkpoint side files: a pass crossing `chunk` bases dumps
    the state so far to <in>_db_brkpt.npz (seq2rdbg :1255-1259) or
    <in>_rdb_brkpt.npz (seq2graph :1880-1887); the file left behind equals
    the one the reference itself wrote with the same chunk (the fixture's
    brkpt.npz): oakht parameters and slot contents, or the edge Dict in
    popitem order with its walk counts and offset."""
    from golden_util import ResumeFixture
    from pangenome_amd import kmer
    fx = ResumeFixture(name)
    q = tmp_path / "input.fsa"
    q.write_bytes(fx.fasta)
    (tmp_path / "input.fsa_rdbg_weight.xyz.mcl").write_text("")
    ref = np.load(fx.brkpt)
    chunk = int(fx.meta["chunk"])
    if fx.flag == "-r":
        kmer.seq2rdbg(str(q), fx.k, 5, 2 ** 63, brkpt="", chunk=chunk, rc=(fx.c >> 1) == 1)
        z = np.load(str(q) + "_db_brkpt.npz")
        assert z["parameters"].tolist() == ref["parameters"].tolist()
        sel, rsel = z["counts"] > 0, ref["counts"] > 0
        o, ro = np.argsort(z["keys"][sel], kind="stable"), np.argsort(ref["keys"][rsel], kind="stable")
        assert np.array_equal(z["keys"][sel][o], ref["keys"][rsel][ro])
        assert np.array_equal(z["values"][sel][o], ref["values"][rsel][ro])
        assert np.array_equal(z["counts"][sel][o], ref["counts"][rsel][ro])
    else:
        g = kmer.seq2rdbg(str(q), fx.k, 5, 2 ** 63, brkpt="", chunk=2 ** 33, rc=(fx.c >> 1) == 1)
        kmer.dbg2rdbg(g)
        kmer.seq2graph(str(q), kmer=fx.k, bits=5, Ns=2 ** 63, rdbg_dict=g, chunk=chunk, brkpt="",
                       rc=(fx.c & 1) == 1, out=io.StringIO())
        z = np.load(str(q) + "_rdb_brkpt.npz")
        for a in ("parameters", "keys", "values"):
            assert z[a].tolist() == ref[a].tolist(), a

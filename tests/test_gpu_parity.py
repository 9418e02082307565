"""GPU parity: libpangenome_hip.so against the reference's goldens and the oracle.

Every test here goes through the C ABI (pangenome_amd._lib -> pangenome.h) on
an MI355X.  Integer/byte work: all comparisons are bit-exact.
"""
import io
import os

import numpy as np
import pytest

from golden_util import Fixture, fixture_names

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def km():
    from pangenome_amd import kmer
    return kmer


def rows_of(text):
    return [ln for ln in text.split("\n") if len(ln.split("\t")) == 5 and ln.split("\t")[3] in ("+", "-")]


def run_stages(km, fasta: bytes, k, c, ns, mcl_text, tmp_path, edge_chunk=2 ** 33):
    q = tmp_path / "input.fsa"
    q.write_bytes(fasta)
    (tmp_path / "input.fsa_rdbg_weight.xyz.mcl").write_text(mcl_text)
    Ns = ns if ns is not None else 2 ** 63
    out = io.StringIO()
    g = km.seq2rdbg(str(q), k, 5, Ns, brkpt="", chunk=2 ** 33, rc=(c >> 1) == 1)
    dk, dm = g.dbg_items()
    km.dbg2rdbg(g)
    rk = g.rdbg_keys()
    km.seq2graph(str(q), kmer=k, bits=5, Ns=Ns, rdbg_dict=g, chunk=edge_chunk, brkpt="", rc=(c & 1) == 1, out=out)
    xyz = (tmp_path / "input.fsa_rdbg_weight.xyz").read_text()
    return dict(dbg_keys=dk, dbg_masks=dm, rdbg_keys=rk, xyz=xyz, rows=rows_of(out.getvalue()), graph=g)


@pytest.mark.parametrize("name", fixture_names())
def test_golden(km, name, tmp_path):
    fx = Fixture(name)
    got = run_stages(km, fx.fasta, fx.k, fx.c, fx.ns, fx.mcl, tmp_path, fx.edge_chunk)
    assert np.array_equal(got["dbg_keys"], fx.dbg_keys)
    assert np.array_equal(got["dbg_masks"], fx.dbg_masks)
    assert np.array_equal(got["rdbg_keys"], fx.rdbg_keys)
    assert got["xyz"] == fx.xyz
    assert got["rows"] == fx.rows


def test_cli_entry_point(km, tmp_path):
    fx = Fixture("pan8_k27_c3")
    q = tmp_path / "in.fa"
    q.write_bytes(fx.fasta)
    (tmp_path / "in.fa_rdbg_weight.xyz.mcl").write_text("")
    out = io.StringIO()
    km.entry_point(["kmer_numba.py", "-i", str(q), "-k27", "-c", "3", "--unknown"], out=out)
    text = out.getvalue()
    assert "# the mcl has been ran" in text
    assert rows_of(text) == fx.rows


@pytest.mark.parametrize("sink", ["file", "append", "pipe"])
def test_cli_rows_to_descriptor(km, tmp_path, sink):
    """stdout with a descriptor under it: the rows go straight from the device
    to it (pg_rows_format_fd) - a regular file in parallel pieces at its
    position, an O_APPEND file and a pipe in order - between the `#` lines
    printed before and after them, as the StringIO path prints them."""
    import threading
    fx = Fixture("pan8_k27_c3")
    q = tmp_path / "in.fa"
    q.write_bytes(fx.fasta)
    (tmp_path / "in.fa_rdbg_weight.xyz.mcl").write_text("")
    argv = ["kmer_numba.py", "-i", str(q), "-k27", "-c", "3"]
    ref = io.StringIO()
    km.entry_point(argv, out=ref)
    xyz_ref = (tmp_path / "in.fa_rdbg_weight.xyz").read_bytes()

    def shape(text):                                  # the text without its timings
        return [ln for ln in text.split("\n") if not ln.startswith("# finished in")]

    if sink == "pipe":
        r, w = os.pipe()
        got = []
        th = threading.Thread(target=lambda: got.append(os.fdopen(r, "rb").read()))
        th.start()
        with os.fdopen(w, "w") as out:
            out.write("# before\n")
            km.entry_point(argv, out=out)
        th.join()
        text = got[0].decode()
    else:
        fn = tmp_path / "out.txt"
        fn.write_text("# before\n")
        with open(fn, "a" if sink == "append" else "r+") as out:
            out.seek(0, os.SEEK_END)
            km.entry_point(argv, out=out)
        text = fn.read_text()
    assert text.startswith("# before\n")
    assert shape(text[len("# before\n"):]) == shape(ref.getvalue())
    assert rows_of(text) == fx.rows
    assert (tmp_path / "in.fa_rdbg_weight.xyz").read_bytes() == xyz_ref


def _random_fasta(rng, n_rec, k):
    """Random records exercising every length class around k and odd bytes."""
    alphabet = np.frombuffer(b"ACGTACGTACGTACGTacgtNnRY$#", dtype=np.uint8)
    parts = []
    for r in range(n_rec):
        n = int(rng.choice([0, 1, k - 1, k, k + 1, k + 2, k + 3, 2 * k, 500, 3000]))
        seq = alphabet[rng.integers(0, alphabet.shape[0], n)].tobytes()
        width = int(rng.choice([7, 60, 1000]))
        body = b"".join(seq[i:i + width] + b"\n" for i in range(0, n, width))
        parts.append(b">r%d desc\n" % r + body)
    return b"".join(parts)


@pytest.mark.parametrize("k", [1, 5, 11, 27])
@pytest.mark.parametrize("c", [0, 3])
def test_random_vs_oracle(km, oracle_mod, tmp_path, k, c):
    rng = np.random.default_rng(1000 * k + c)
    fasta = _random_fasta(rng, 40, k)
    ref = oracle_mod.run_pipeline(fasta, k, c)
    got = run_stages(km, fasta, k, c, None, "", tmp_path)
    assert np.array_equal(got["dbg_keys"], ref["dbg_keys"])
    assert np.array_equal(got["dbg_masks"], ref["dbg_masks"])
    assert np.array_equal(got["rdbg_keys"], ref["rdbg_keys"])
    assert got["xyz"] == ref["xyz"]
    assert got["rows"] == ref["rows"]


@pytest.mark.parametrize("c", [0, 1, 2, 3])
def test_pangenome_vs_oracle(km, oracle_mod, tmp_path, c):
    from pangenome_amd import synth
    fasta = synth.pangenome(12, 60_000, snp=0.005, indel=5e-4, seed=77 + c)
    ref = oracle_mod.run_pipeline(fasta, 27, c)
    got = run_stages(km, fasta, 27, c, None, "", tmp_path)
    assert np.array_equal(got["dbg_keys"], ref["dbg_keys"])
    assert np.array_equal(got["dbg_masks"], ref["dbg_masks"])
    assert np.array_equal(got["rdbg_keys"], ref["rdbg_keys"])
    assert got["xyz"] == ref["xyz"]
    assert got["rows"] == ref["rows"]


@pytest.mark.parametrize("chunks", [1, 4])
@pytest.mark.parametrize("rc0", [True, False])
def test_k3_ragged_vs_oracle(oracle_mod, chunks, rc0):
    """The partitioned K3 (coverage + work passes, stage A bins, split, range
    merge with the fused degree scan) on a pangenome with ragged record
    lengths, including records shorter than a stripe and records of n <= k+1,
    with the tile list in one chunk and in four."""
    from pangenome_amd import synth
    from pangenome_amd._lib import Context, PG_TUNE_K3_CHUNKS
    fasta = synth.pangenome(11, 70_000, snp=0.004, indel=6e-4, seed=31)
    fasta += b">s1\nACGTACGTACGTACGTACGTACGTACGT\n>s2\nACGT\n>s3\n" + b"A" * 700 + b"\n"
    c = 2 if rc0 else 0
    ref = oracle_mod.OracleRun(fasta, 27, c)
    ctx = Context(27)
    ctx.tune(PG_TUNE_K3_CHUNKS, chunks)
    ctx.set_fasta(fasta)
    ctx.parse()
    ctx.build_dbg(None, 0, rc0)
    keys, masks = ctx.dbg()
    ctx.build_rdbg()
    rk, rm = ref.dbg()
    assert np.array_equal(keys, rk)
    assert np.array_equal(masks, rm)
    assert np.array_equal(ctx.rdbg(), ref.rdbg())
    ctx.close()


@pytest.mark.parametrize("k", [15, 27])
def test_overflow_and_rerun_paths_vs_oracle(oracle_mod, k):
    """Forced slow paths give the same dBG: a table 8x smaller than sized
    (LDS overflow sets fill, spill to the HBM overflow table, re-run with
    more buckets) and tiny stage A regions (records dropped, re-run with the
    exact region counts)."""
    from pangenome_amd import synth
    from pangenome_amd._lib import Context, PG_TUNE_BUCKET_SHIFT, PG_TUNE_REGION_CAP
    fasta = synth.pangenome(6, 90_000, snp=0.01, indel=1e-3, seed=17)
    ref = oracle_mod.OracleRun(fasta, k, 2)
    rk, rm = ref.dbg()
    for what, val in ((PG_TUNE_BUCKET_SHIFT, 3), (PG_TUNE_BUCKET_SHIFT, 8), (PG_TUNE_REGION_CAP, 64)):
        ctx = Context(k)
        ctx.tune(what, val)
        ctx.set_fasta(fasta)
        ctx.parse()
        st = ctx.build(None, 0, True)
        keys, masks = ctx.dbg()
        assert np.array_equal(keys, rk) and np.array_equal(masks, rm), (what, val)
        assert np.array_equal(ctx.rdbg(), ref.rdbg()), (what, val)
        assert st.n_rdbg == len(ref.rdbg())
        ctx.close()


def _cover_forms():
    """The coverage-pass forms this library was built with: the packed form
    (0); rounds 2-3's class-byte forms (1: LDS-staged members, 2: quad
    compare) only in a PG_COVER_LEGACY test build."""
    from pangenome_amd._lib import Context, PangenomeError, PG_TUNE_K3_COVER
    ctx = Context(27)
    forms = [0]
    for f in (1, 2):
        try:
            ctx.tune(PG_TUNE_K3_COVER, f)
            forms.append(f)
        except PangenomeError:
            pass
    ctx.close()
    return forms


@pytest.mark.parametrize("form", [0, 1, 2])
@pytest.mark.parametrize("c", [0, 2])
def test_k3_reference_dedup_vs_oracle(oracle_mod, c, form):
    """The coverage pass skips a follower window whose k+2 context bytes equal
    the lead record's at some drift: copies of the lead with insertions (drift
    inside and beyond the +-512 search), deletions, SNPs, an N run, lowercase
    bytes, shorter copies (reference windows near its ends) and a reverse
    complement; every form of the pass (packed 2-bit stream, LDS-staged
    members, quad compare)."""
    from pangenome_amd import synth
    from pangenome_amd._lib import Context, PG_TUNE_K3_COVER
    rng = np.random.default_rng(7 + c)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    lead = acgt[rng.integers(0, 4, 30_000)]
    copies = [lead.copy()]
    for ins in (1, 37, 300, 511, 513, 900):
        g = lead.copy()
        pos = int(rng.integers(1000, 20_000))
        g = np.concatenate([g[:pos], acgt[rng.integers(0, 4, ins)], g[pos:]])
        snp = rng.integers(0, g.shape[0], 20)
        g[snp] = acgt[rng.integers(0, 4, 20)]
        copies.append(g)
    g = lead.copy()
    g = np.concatenate([g[:5000], g[5100:]])                 # deletion
    g[12000:12040] = ord("N")
    g[20000:20010] = np.frombuffer(b"acgtacgtac", np.uint8)
    copies.append(g)
    copies.append(lead[3:29_000].copy())                     # shorter, shifted
    copies.append(lead[:4100].copy())                        # ends inside the lead's first stripe
    comp = np.frombuffer(bytes.maketrans(b"ACGT", b"TGCA"), np.uint8)
    copies.append(comp[lead[::-1]])                          # reverse complement
    fasta = b"".join(b">g%d\n" % i + g.tobytes() + b"\n" for i, g in enumerate(copies))
    if form not in _cover_forms():
        pytest.skip("coverage form %d: built only with PG_COVER_LEGACY" % form)
    ref = oracle_mod.OracleRun(fasta, 27, c)
    ctx = Context(27)
    ctx.tune(PG_TUNE_K3_COVER, form)
    ctx.set_fasta(fasta)
    ctx.parse()
    ctx.build_dbg(None, 0, c == 2)
    keys, masks = ctx.dbg()
    rk, rm = ref.dbg()
    assert np.array_equal(keys, rk)
    assert np.array_equal(masks, rm)
    ctx.build_rdbg()
    assert np.array_equal(ctx.rdbg(), ref.rdbg())
    ctx.close()


@pytest.mark.parametrize("k", [5, 15, 21, 27])
def test_k3_cover_forms_vs_oracle(oracle_mod, k):
    """Every coverage-pass form gives the oracle's dBG and rdBG at several k
    (the window masks depend on k and on each record's start modulo 4 (quad
    form) or 16 (packed form): odd line widths and headers shift it); the
    packed form, exact per base, leaves no more stage A records than the quad
    form, and neither leaves more than 2 % more than the LDS-staged one."""
    from pangenome_amd import synth
    from pangenome_amd._lib import Context, PG_TUNE_K3_COVER
    fasta = synth.pangenome(9, 120_000, snp=2e-3, indel=3e-4, seed=400 + k, width=61)
    ref = oracle_mod.OracleRun(fasta, k, 2)
    rk, rm = ref.dbg()
    recs = []
    forms = _cover_forms()
    for form in forms:
        ctx = Context(k)
        ctx.tune(PG_TUNE_K3_COVER, form)
        ctx.set_fasta(fasta)
        ctx.parse()
        st = ctx.build(None, 0, True)
        keys, masks = ctx.dbg()
        assert np.array_equal(keys, rk) and np.array_equal(masks, rm), form
        assert np.array_equal(ctx.rdbg(), ref.rdbg()), form
        recs.append(st.n_records_a)
        ctx.close()
    if forms == [0, 1, 2]:
        assert recs[0] <= recs[2] and recs[2] <= recs[1] * 1.02 + 64, recs


@pytest.mark.parametrize("k", [15, 27])
def test_k3_anchor_counts_vs_oracle(oracle_mod, k):
    """The packed coverage pass at 3, 4, 6 and 8 anchors per tile and reference
    (PG_TUNE_K3_ANCHORS) gives the oracle's dBG and rdBG; with indels dense
    enough for several drift changes per tile, more anchors leave fewer stage A
    records (the runs between two indels that an anchor falls in are covered)."""
    from pangenome_amd import synth
    from pangenome_amd._lib import Context, PG_TUNE_K3_ANCHORS
    fasta = synth.pangenome(9, 150_000, snp=1e-3, indel=5e-4, seed=470 + k, width=61)
    ref = oracle_mod.OracleRun(fasta, k, 2)
    rk, rm = ref.dbg()
    recs = {}
    for na in (3, 4, 6, 8, 0):
        ctx = Context(k)
        ctx.tune(PG_TUNE_K3_ANCHORS, na)
        ctx.set_fasta(fasta)
        ctx.parse()
        st = ctx.build(None, 0, True)
        keys, masks = ctx.dbg()
        assert np.array_equal(keys, rk) and np.array_equal(masks, rm), na
        assert np.array_equal(ctx.rdbg(), ref.rdbg()), na
        recs[na] = st.n_records_a
        ctx.close()
    assert recs[8] < recs[6] < recs[4] < recs[3], recs
    assert abs(recs[0] - recs[4]) <= recs[4] // 100, recs      # 0 = 4 (hints may differ run to run)


@pytest.mark.parametrize("k", [15, 27])
def test_k3_packed_exceptions_vs_oracle(oracle_mod, k):
    """The packed coverage pass around bases that are not ACGT (their 2-bit
    code is not their class): N runs, IUPAC codes in both cases and '$' in
    members and in the lead and second reference records, at every alignment
    of a 16-base word - the oracle's dBG and rdBG in every form."""
    from pangenome_amd import synth
    from pangenome_amd._lib import Context, PG_TUNE_K3_COVER
    fasta = bytearray(synth.pangenome(8, 90_000, snp=2e-3, indel=3e-4, seed=700 + k, width=57))
    rng = np.random.default_rng(k)
    seq = np.zeros(len(fasta), bool)                 # sequence bytes (not headers, not newlines)
    hdr = False
    for i, b in enumerate(fasta):
        if b == ord(">") and (i == 0 or fasta[i - 1] == ord("\n")):
            hdr = True
        if b == ord("\n"):
            hdr = False
        seq[i] = not hdr and b != ord("\n")
    pos = np.flatnonzero(seq)
    for p in rng.choice(pos, 400, replace=False).tolist():        # single odd bases
        fasta[p] = rng.choice([ord(c) for c in "NnRYkmSWbdhv$"])
    for p in rng.choice(pos[: pos.shape[0] // 8], 6, replace=False).tolist():   # N runs, some in the lead
        for q in range(p, min(p + int(rng.integers(1, 70)), len(fasta))):
            if seq[q]:
                fasta[q] = ord("N")
    fasta = bytes(fasta)
    ref = oracle_mod.OracleRun(fasta, k, 2)
    rk, rm = ref.dbg()
    for form in _cover_forms():
        ctx = Context(k)
        ctx.tune(PG_TUNE_K3_COVER, form)
        ctx.set_fasta(fasta)
        ctx.parse()
        ctx.build(None, 0, True)
        keys, masks = ctx.dbg()
        assert np.array_equal(keys, rk) and np.array_equal(masks, rm), form
        assert np.array_equal(ctx.rdbg(), ref.rdbg()), form
        ctx.close()


def test_edge_checkpoint_reversal_vs_oracle(km, oracle_mod, tmp_path):
    from pangenome_amd import synth
    fasta = b"junk before header\n" + synth.pangenome(9, 20_000, snp=0.01, indel=1e-3, seed=5)
    ref = oracle_mod.run_pipeline(fasta, 21, 3, edge_chunk=25_000)
    got = run_stages(km, fasta, 21, 3, None, "", tmp_path, edge_chunk=25_000)
    assert got["xyz"] == ref["xyz"]
    assert got["rows"] == ref["rows"]


def test_device_resident_input_and_repeat(km):
    """Input already in HBM (the bench path): two builds are identical."""
    import torch
    from pangenome_amd import synth
    from pangenome_amd._lib import Context
    fasta = synth.pangenome(20, 100_000, seed=9)
    d = torch.frombuffer(bytearray(fasta), dtype=torch.uint8).to("cuda:0")
    torch.cuda.synchronize()
    ctx = Context(27)
    res = []
    for _ in range(2):
        ctx.set_fasta_device(d.data_ptr(), d.numel(), keepalive=d)
        ctx.parse()
        ctx.build_dbg(None, 0, True)
        st = ctx.build_rdbg()
        res.append((st.n_dbg, st.n_rdbg, ctx.rdbg()))
    assert res[0][0] == res[1][0] and res[0][1] == res[1][1]
    assert np.array_equal(res[0][2], res[1][2])


def test_build_device_empty_input():
    """pg_build_device of an empty input, on a fresh context and
    after a real build, succeeds with an empty dBG and zero parse time."""
    import torch
    from pangenome_amd import synth
    from pangenome_amd._lib import Context
    d = torch.frombuffer(bytearray(synth.pangenome(2, 20_000, seed=5)), dtype=torch.uint8).to("cuda:0")
    e = torch.zeros(16, dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()
    for warm in (False, True):
        ctx = Context(27)
        if warm:
            assert ctx.build_device(d.data_ptr(), d.numel(), True, keepalive=d).n_dbg > 0
        st = ctx.build_device(e.data_ptr(), 0, True, keepalive=e)
        assert (st.n_records, st.n_bases, st.n_dbg, st.n_rdbg, st.ms_parse) == (0, 0, 0, 0, 0.0)
        ctx.close()


def test_full_size_properties(km):
    """C3-shaped input (100 genomes is too slow for the oracle; use 40 x 5 Mbp):
    size-independent invariants of the reference's dBG."""
    from pangenome_amd import synth
    from pangenome_amd._lib import Context
    fasta = synth.pangenome(40, 5_000_000, seed=123)
    ctx = Context(27)
    ctx.set_fasta(fasta)
    R, B = ctx.parse()
    assert R == 40
    ctx.build_dbg(None, 0, True)
    st = ctx.build_rdbg()
    keys, masks = ctx.dbg()
    assert st.n_dbg == keys.shape[0]
    # both strands inserted: the key set is closed under reverse complement
    # (no N here, so no palindromes at odd k): n_dbg == 2 * occupied slots
    assert st.n_dbg == 2 * st.n_slots
    # every key has a nonzero mask with at most one '#' start (pred 0) ... and
    # the rdBG is exactly the keys whose mask is not (1 pred bit and 1 succ bit)
    pc = np.array([bin(i).count("1") for i in range(64)], np.int64)
    member = ~((pc[(masks >> 6) & 63] == 1) & (pc[masks & 63] == 1))
    assert np.array_equal(np.sort(keys[member]), ctx.rdbg())
    # record lengths agree with a host parse
    lens = [len(b"".join(rec.split(b"\n")[1:])) for rec in fasta.split(b">")[1:]]
    assert ctx.records()["seq_len"].tolist() == lens


@pytest.mark.parametrize("chunks", [1, 3, 4])
@pytest.mark.parametrize("c", [0, 2])
def test_k3_chunked_two_references_vs_oracle(oracle_mod, chunks, c):
    """The two-pass K3 on two streams (coverage of chunk i+1 beside the work
    pass of chunk i), with the lead and a second reference record: genomes
    sharing the lead's variant sites (so ref2 covers them), an N run, a
    lowercase stretch and records shorter than a stripe."""
    from pangenome_amd import synth
    from pangenome_amd._lib import Context, PG_TUNE_K3_CHUNKS
    fasta = synth.pangenome(12, 150_000, snp=2e-3, indel=3e-4, seed=77 + chunks)
    recs = [b">" + r for r in fasta.split(b">")[1:]]
    body = bytearray(recs[3])
    body[5000:5040] = b"N" * 40
    body[9000:9100] = bytes(body[9000:9100]).lower()
    recs[3] = bytes(body)
    fasta = b"".join(recs) + b">short\n" + b"ACGT" * 300 + b"\n"
    ref = oracle_mod.OracleRun(fasta, 27, c)
    ctx = Context(27)
    ctx.tune(PG_TUNE_K3_CHUNKS, chunks)
    ctx.set_fasta(fasta)
    ctx.parse()
    ctx.build_dbg(None, 0, c == 2)
    keys, masks = ctx.dbg()
    rk, rm = ref.dbg()
    assert np.array_equal(keys, rk)
    assert np.array_equal(masks, rm)
    ctx.build_rdbg()
    assert np.array_equal(ctx.rdbg(), ref.rdbg())
    ctx.close()


def test_pg_build_sequence_vs_oracle(oracle_mod):
    """One context over inputs of different shape: a first build (no learned
    stage A size), a repeat, then a larger, more varied input whose records
    per window outgrow the learned size (stage A re-run), a single record,
    and back — pg_build and the two-call path against the oracle."""
    from pangenome_amd import synth
    from pangenome_amd._lib import Context
    small = synth.pangenome(4, 40_000, snp=1e-4, indel=0.0, seed=5)
    large = synth.pangenome(10, 120_000, snp=3e-2, indel=5e-3, seed=6)
    single = synth.ecoli_like(300_000)
    ctx, two = Context(27), Context(27)
    for fasta in (small, small, large, large, single, small):
        ref = oracle_mod.OracleRun(fasta, 27, 2)
        ctx.set_fasta(fasta)
        ctx.parse()
        st = ctx.build(None, 0, True)
        two.set_fasta(fasta)                       # the two-call path
        two.parse()
        two.build_dbg(None, 0, True)
        st2 = two.build_rdbg()
        assert (st.n_dbg, st.n_rdbg) == (st2.n_dbg, st2.n_rdbg)
        assert np.array_equal(ctx.rdbg(), ref.rdbg())
        assert st.n_rdbg == len(ref.rdbg())
        keys, masks = ctx.dbg()
        rk, rm = ref.dbg()
        assert np.array_equal(keys, rk) and np.array_equal(masks, rm)
    ctx.close()
    two.close()

"""K1 (FASTA parse) parity on adversarial byte streams.

The record table (sequence length, header span, seqio's `ptr`) is checked
against a numpy restatement of readline_jit_ / seqio_jit_
(kmer_numba.py:122-172); the bases themselves through the k=1 and k=5 dBG
against the C oracle (every base's class and both neighbours are in a k=1
mask).  Inputs cover unterminated last lines of every length, '>' at the end,
CRLF, empty lines and records, bases before the first header, lines and
headers longer than the kernel's 16 KiB wave span, and random byte soup.
"""
import numpy as np
import pytest

from dist_util import seqio_records

pytestmark = pytest.mark.gpu


CASES = {
    "plain": b">a\nACGT\nACG\n>b\nTTTT\n",
    "tail2": b">a\nACGT\nAC",
    "tail1": b">a\nACGT\nA",
    "tail_hdr": b">a\nACGT\n>b",
    "tail_gt": b">a\nACGT\n>",
    "tail_hdr_only": b">a\nAC\n>bb",
    "no_newline": b">a ACGT",
    "only_newlines": b"\n\n\n",
    "single_nl": b"\n",
    "crlf": b">a\r\nACGT\r\nGG\r\n>b\r\nTT\r\n",
    "empty_lines": b"\n\n>a\n\nAC\n\n\n>b\n\n",
    "empty_records": b">a\n>b\n>c\nACG\n>d\n",
    "before_header": b"ACGTACGT\nGG\n>a\nCCCC\n",
    "headers_only": b">a\n>b\n>c\n",
    "gt_in_seq": b">a\nAC>GT\n>b\nG>\n",
    "dollar_n": b">a\nAC$GTNNnnacgtRYK\n",
}


def _long_cases():
    rng = np.random.default_rng(5)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    one_line = acgt[rng.integers(0, 4, 70_000)].tobytes()
    long_hdr = b">" + b"h" * 40_000
    return {
        "one_line_70k": b">x\n" + one_line + b"\n>y\n" + one_line[:33_333] + b"\n",
        "long_header": long_hdr + b"\nACGTTGCA\n" + long_hdr + b"\nGG\n",
        "long_tail": b">x\n" + one_line,
        "long_tail_hdr": b">x\nACGT\n" + long_hdr,
    }


def _soup(seed, n, alphabet):
    rng = np.random.default_rng(seed)
    a = np.frombuffer(alphabet, dtype=np.uint8)
    return a[rng.integers(0, a.shape[0], n)].tobytes()


SOUPS = [(s, n, alpha) for s, (n, alpha) in enumerate([
    (1, b">\nA"), (2, b">\nA"), (3, b">\nAC"), (17, b">\nACGTN"), (1000, b">\nACGT\r"),
    (16_383, b"ACGT\n>"), (16_385, b"ACGTACGTACGT\n>"), (50_000, b"ACGTACGTACGTACGTACGT\n>x"),
    (120_000, b"A" * 60 + b"\n>"), (33_000, b"\n>"),
])]


def _check(buf, oracle_mod, k1=None):
    from pangenome_amd._lib import PG_TUNE_K1, Context

    def make(k):
        c = Context(k)
        if k1 is not None:
            c.tune(PG_TUNE_K1, k1)
        return c
    ctx = make(5)
    ctx.set_fasta(buf)
    R, B = ctx.parse()
    exp = seqio_records(buf)
    assert R == len(exp)
    if R:
        got = ctx.records()
        assert got["seq_len"].tolist() == [e[0] for e in exp]
        assert got["hdr_start"].tolist() == [e[1] for e in exp]
        assert got["hdr_len"].tolist() == [e[2] for e in exp]
        assert got["ptr"].tolist() == [e[3] for e in exp]
    assert B == sum(e[0] for e in exp)
    ctx.close()
    for k in (1, 5):
        ctx = make(k)
        ctx.set_fasta(buf)
        ctx.parse()
        ctx.build_dbg(None, 0, True)
        keys, masks = ctx.dbg()
        ctx.close()
        rk, rm = oracle_mod.OracleRun(buf, k, 2).dbg()
        assert np.array_equal(keys, rk)
        assert np.array_equal(masks, rm)


# K1's forms (PG_TUNE_K1): per-step / whole-span span pass, one / two steps
# of emission loads in flight
K1_FORMS = [0, 1, 2, 3, 4, 5]


@pytest.mark.parametrize("name", sorted(CASES))
def test_parse_cases(oracle_mod, name):
    _check(CASES[name], oracle_mod)


@pytest.mark.parametrize("k1", K1_FORMS)
@pytest.mark.parametrize("name", ["one_line_70k", "long_header", "long_tail", "long_tail_hdr"])
def test_parse_long_lines(oracle_mod, name, k1):
    _check(_long_cases()[name], oracle_mod, k1)


@pytest.mark.parametrize("k1", K1_FORMS)
@pytest.mark.parametrize("seed,n,alphabet", SOUPS)
def test_parse_soup(oracle_mod, seed, n, alphabet, k1):
    _check(_soup(seed, n, alphabet), oracle_mod, k1)


@pytest.mark.parametrize("k1", K1_FORMS)
def test_parse_span_boundaries(oracle_mod, k1):
    """Line and header boundaries on every side of the 16 KiB span edge;
    spans with no newline, with the line open at the span start a header
    line or a sequence line, and a header line continuing across a span."""
    span = 16 * 1024
    for shift in (-2, -1, 0, 1, 2):
        body = b"A" * (span + shift - 4)
        _check(b">a\n" + body + b"\n>b\nCC\n", oracle_mod, k1)
        _check(b">a\nC\n" + b"G" * (span + shift - 6) + b">c\nAC\n", oracle_mod, k1)
        _check(b">" + b"h" * (span + shift) + b"\n" + b"ACGT" * 9000 + b"\n>c\nAC\n", oracle_mod, k1)
        _check(b">a\n" + b"T" * (3 * span + shift) + b"\n" + b">" + b"h" * (2 * span) + b"x\nGA\n", oracle_mod, k1)


def _mixed_fasta(seed, widths, nrec=12, reclen=40_000):
    """Records of ACGT with lowercase stretches, N runs and a rare '$', wrapped
    at the given line widths: most 1 KiB wave steps take K1's fast step (no
    '>', at most one '\\n' per 16 bytes, ACGTacgt only), the rest its general
    step, switching at every kind of boundary."""
    rng = np.random.default_rng(seed)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    out = []
    for r in range(nrec):
        s = acgt[rng.integers(0, 4, reclen)].copy()
        for _ in range(6):                                   # lowercase stretches
            a = int(rng.integers(0, reclen - 500))
            s[a:a + int(rng.integers(1, 500))] |= 0x20
        if r % 3 == 0:                                       # an N run (general steps)
            a = int(rng.integers(0, reclen - 100))
            s[a:a + int(rng.integers(1, 100))] = ord("N")
        if r % 5 == 1:
            s[int(rng.integers(0, reclen))] = ord("$")
        w = int(widths[r % len(widths)])
        body = b"\n".join(s[i:i + w].tobytes() for i in range(0, reclen, w))
        out.append(b">rec%d some description\n" % r + body + b"\n")
    return b"".join(out)


@pytest.mark.parametrize("k1", K1_FORMS)
@pytest.mark.parametrize("widths", [(60,), (15, 16, 17), (61, 80, 1000), (16, 7, 60, 33)])
def test_parse_fast_steps(oracle_mod, widths, k1):
    _check(_mixed_fasta(sum(widths), widths), oracle_mod, k1)
    # unterminated last line, and a record longer than a 16 KiB span
    _check(_mixed_fasta(7, widths, nrec=3, reclen=50_000)[:-1], oracle_mod, k1)


def _rec_table(buf):
    """The record table restated from readline_jit_ / seqio_jit_ (numpy)."""
    exp = seqio_records(buf)
    cols = list(zip(*exp)) if exp else [(), (), (), ()]
    return {key: np.array(col, np.int64) for key, col in zip(("seq_len", "hdr_start", "hdr_len", "ptr"), cols)}


def _check_records(ctx, exp):
    got = ctx.records()
    for key in exp:
        assert np.array_equal(got[key], exp[key]), key


@pytest.mark.parametrize("chunk", [16 * 1024, 3 * 16 * 1024, 0])
def test_parse_host_pipelined(oracle_mod, chunk):
    """pg_parse_host: the upload in chunks of whole K1 spans on a side stream
    (pageable bytes through the pinned staging ring), K1 on each chunk as it
    lands.  The record table against the seqio restatement and the class
    stream (via the k=5 dBG) against the oracle, with chunk edges on every
    span edge."""
    from pangenome_amd._lib import Context, PG_TUNE_H2D_CHUNK
    # (> 64 records: the first parse of a context re-runs the emission with the exact record count)
    buf = _mixed_fasta(3, (60, 17), nrec=70, reclen=3_000) + CASES["empty_records"] + _long_cases()["long_header"]
    exp = _rec_table(buf)
    rk, rm = oracle_mod.OracleRun(buf, 5, 2).dbg()
    ctx = Context(5)
    ctx.tune(PG_TUNE_H2D_CHUNK, chunk)
    for _ in range(2):                              # the second parse reuses the record capacity
        assert ctx.parse_host(buf) == (exp["seq_len"].shape[0], int(exp["seq_len"].sum()))
        _check_records(ctx, exp)
        ctx.build_dbg(None, 0, True)
        keys, masks = ctx.dbg()
        assert np.array_equal(keys, rk) and np.array_equal(masks, rm)
    ctx.close()


def _oracle_ref(buf, k=27):
    """(record table, dBG, rdBG) of the restatement and the pinned oracle."""
    from oracle import oracle
    o = oracle.OracleRun(buf, k, 2)
    dk, dm = o.dbg()
    return _rec_table(buf), (dk, dm), o.rdbg()


def _check_build(ctx, st, ref):
    rec, (rk, rm), rr = ref
    assert (st.n_dbg, st.n_rdbg) == (rk.shape[0], rr.shape[0])
    _check_records(ctx, rec)
    keys, masks = ctx.dbg()
    assert np.array_equal(keys, rk) and np.array_equal(masks, rm)
    assert np.array_equal(ctx.rdbg(), rr)


@pytest.mark.parametrize("case", ["pangenome", "mixed", "few_long", "tiny_records"])
def test_build_host_streamed(case):
    """pg_build_host: stage A over each chunk's completed records under the
    chunked upload (the lead and second reference picked among the first
    completed records) - the record table of the seqio restatement and the
    oracle's dBG and rdBG, cold and warm, with chunk edges inside records and
    records spanning many chunks."""
    from pangenome_amd import synth
    from pangenome_amd._lib import Context, PG_TUNE_H2D_CHUNK
    if case == "pangenome":
        buf, chunks = synth.pangenome(12, 150_000, snp=1e-3, indel=1e-4, seed=11), (64 * 1024, 16 * 1024)
    elif case == "mixed":
        buf, chunks = _mixed_fasta(5, (60, 17, 1000), nrec=10, reclen=20_000), (16 * 1024, 3 * 16 * 1024)
    elif case == "few_long":                       # never three long records before the last chunk
        buf, chunks = _mixed_fasta(9, (60,), nrec=2, reclen=60_000), (16 * 1024,)
    else:                                          # records of length < k, = k, k+1, k+2 between long ones
        rng = np.random.default_rng(3)
        acgt = np.frombuffer(b"ACGT", np.uint8)
        recs = [acgt[rng.integers(0, 4, m)].tobytes() for m in (40_000, 5, 27, 28, 29, 40_000, 0, 30_000, 26, 35_000)]
        buf, chunks = b"".join(b">r%d\n%s\n" % (i, r) for i, r in enumerate(recs)), (16 * 1024,)
    ref = _oracle_ref(buf)
    for chunk in chunks:
        ctx = Context(27)
        ctx.tune(PG_TUNE_H2D_CHUNK, chunk)
        for _ in range(2):                          # cold, then warm (sized from the first build)
            st = ctx.build_host(buf, True)
            _check_build(ctx, st, ref)
        ctx.close()


@pytest.mark.parametrize("threads,register", [(1, 0), (3, 0), (0, 0), (0, 1)])
def test_build_host_mmap_and_pinned(tmp_path, threads, register):
    """The input kinds pg_build_host meets: a read-only np.memmap of the file
    (kmer.seq2bytes, what the CLI passes: through the pinned staging ring,
    40+ chunks so the ring's slots and the 16 chunk events are reused many
    times), a pinned torch buffer (DMA'd directly) and a pinned buffer at an
    offset; all against the oracle, with 1, 3 and the default staging threads,
    and with the mmap's chunks registered and DMA'd directly (the default)."""
    import torch
    from pangenome_amd import kmer, synth
    from pangenome_amd._lib import Context, PG_TUNE_H2D_CHUNK, PG_TUNE_HOST_REGISTER, PG_TUNE_HOST_THREADS
    buf = synth.pangenome(10, 120_000, snp=2e-3, indel=2e-4, seed=21)
    q = tmp_path / "in.fa"
    q.write_bytes(buf)
    ref = _oracle_ref(buf)
    mm = kmer.seq2bytes(str(q))
    pin = torch.empty(len(buf) + 64, dtype=torch.uint8, pin_memory=True)
    pin.numpy()[:len(buf)] = np.frombuffer(buf, np.uint8)
    pin2 = torch.empty(len(buf) + 64, dtype=torch.uint8, pin_memory=True)
    pin2.numpy()[5:5 + len(buf)] = np.frombuffer(buf, np.uint8)
    ctx = Context(27)
    ctx.tune(PG_TUNE_H2D_CHUNK, 16 * 1024 * 2)
    ctx.tune(PG_TUNE_HOST_THREADS, threads)
    ctx.tune(PG_TUNE_HOST_REGISTER, register)
    for src in ("mmap", "pinned", "mmap", "pinned_offset"):
        if src == "mmap":
            st = ctx.build_host(mm, True)
        elif src == "pinned":
            st = ctx.build_host_ptr(pin.data_ptr(), len(buf), True)
        else:
            st = ctx.build_host_ptr(pin2.data_ptr() + 5, len(buf), True)
        _check_build(ctx, st, ref)
    # pg_set_fasta (the bare staged upload) + parse
    ctx.set_fasta(mm)
    assert ctx.parse() == (ref[0]["seq_len"].shape[0], int(ref[0]["seq_len"].sum()))
    ctx.close()


@pytest.mark.parametrize("tail", [16384, 3 * 16384, 100_000])
def test_build_host_small_last_chunk(tmp_path, tail):
    """pg_build_host with a last H2D chunk smaller than the others
    (PG_TUNE_H2D_TAIL: the chunk bounds are no longer uniform, a body
    remainder shorter than a quarter chunk joins its neighbour), from the mmap
    and from pinned memory, three builds each (the early split and the
    speculative stage C of the warm builds): the oracle's dBG and rdBG."""
    import torch
    from pangenome_amd import kmer, synth
    from pangenome_amd._lib import Context, PG_TUNE_H2D_CHUNK, PG_TUNE_H2D_TAIL
    buf = synth.pangenome(12, 90_000, snp=2e-3, indel=2e-4, seed=23)
    q = tmp_path / "in.fa"
    q.write_bytes(buf)
    ref = _oracle_ref(buf)
    mm = kmer.seq2bytes(str(q))
    pin = torch.empty(len(buf) + 64, dtype=torch.uint8, pin_memory=True)
    pin.numpy()[:len(buf)] = np.frombuffer(buf, np.uint8)
    ctx = Context(27)
    ctx.tune(PG_TUNE_H2D_CHUNK, 8 * 16384)
    ctx.tune(PG_TUNE_H2D_TAIL, tail)
    for _ in range(3):
        _check_build(ctx, ctx.build_host(mm, True), ref)
        _check_build(ctx, ctx.build_host_ptr(pin.data_ptr(), len(buf), True), ref)
    ctx.close()


def test_cli_build_uses_streamed_path(tmp_path):
    """kmer.seq2rdbg on a file no -n / checkpoint touches builds through
    pg_build_host (the stats of a streamed build: stage A records counted
    while the upload ran) and equals the oracle."""
    from pangenome_amd import kmer, synth
    buf = synth.pangenome(8, 100_000, snp=2e-3, indel=2e-4, seed=22)
    q = tmp_path / "in.fa"
    q.write_bytes(buf)
    ref = _oracle_ref(buf)
    g = kmer.seq2rdbg(str(q), 27, 5, 2 ** 63, brkpt="", chunk=2 ** 33, rc=True)
    _check_build(g.ctx, g.stats, ref)
    # a -n limit below the file size: the planned path (parse, then the build
    # of the records the plan takes), against the oracle under the same -n
    from oracle import oracle
    g2 = kmer.seq2rdbg(str(q), 27, 5, 300_000, brkpt="", chunk=2 ** 33, rc=True)
    dk, dm = oracle.OracleRun(buf, 27, 2, ns=300_000).dbg()
    keys, masks = g2.dbg_items()
    assert 0 < keys.shape[0] < ref[1][0].shape[0]
    assert np.array_equal(keys, dk) and np.array_equal(masks, dm)


def test_build_device_one_call(oracle_mod):
    """pg_build_device (set_fasta_device + parse + build in one call, the
    bench's step): the oracle's dBG / rdBG, the record table of parse, with
    the context alternating between inputs of different record counts (the
    kept device copy of the record flags, the overflow table's skipped
    clear, the one-launch readback)."""
    import torch
    from oracle import oracle
    from pangenome_amd import synth
    from pangenome_amd._lib import Context
    rng = np.random.default_rng(5)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    recs = [acgt[rng.integers(0, 4, m)].tobytes() for m in (40_000, 5, 27, 28, 29, 40_000, 0, 30_000, 26)]
    bufs = [synth.pangenome(12, 150_000, snp=1e-3, indel=1e-4, seed=11),
            b"".join(b">r%d\n%s\n" % (i, r) for i, r in enumerate(recs)),
            _mixed_fasta(5, (60, 17, 1000), nrec=10, reclen=20_000),
            synth.pangenome(7, 90_000, snp=2e-3, indel=1e-4, seed=12)]
    refs = []
    for b in bufs:
        o = oracle.OracleRun(b, 27, 2)
        dk, dm = o.dbg()
        refs.append((_rec_table(b), dk, dm, o.rdbg()))
    ctx = Context(27)
    dev = [torch.frombuffer(bytearray(b), dtype=torch.uint8).to("cuda") for b in bufs]
    torch.cuda.synchronize()
    for i in (0, 1, 2, 3, 0, 0, 3, 1):
        st = ctx.build_device(dev[i].data_ptr(), dev[i].numel(), True, keepalive=dev[i])
        rec, dk, dm, rk = refs[i]
        assert (st.n_dbg, st.n_rdbg) == (dk.shape[0], rk.shape[0]), i
        got = ctx.records()
        for key in rec:
            assert np.array_equal(got[key], rec[key]), (i, key)
        keys, masks = ctx.dbg()
        assert np.array_equal(keys, dk) and np.array_equal(masks, dm), i
        assert np.array_equal(ctx.rdbg(), rk), i
    ctx.close()



def test_build_host_early_split():
    """Stage B under the upload (PG_TUNE_EARLY_SPLIT): a warm pg_build_host
    splits each landed chunk's records into the table's partitions (geometry
    from the first build) and stage C reads them (build_flags bit 0) - the
    oracle's dBG and rdBG either way, and with the early split turned off."""
    from pangenome_amd import synth
    from pangenome_amd._lib import Context, PG_TUNE_EARLY_SPLIT, PG_TUNE_H2D_CHUNK
    buf = synth.pangenome(24, 250_000, snp=1e-2, indel=1e-3, seed=31)   # > 2^19 stage A records: a split level
    ref = _oracle_ref(buf)
    ctx = Context(27)
    ctx.tune(PG_TUNE_H2D_CHUNK, 256 * 1024)
    used = []
    for early in (1, 1, 1, 0, 1):
        ctx.tune(PG_TUNE_EARLY_SPLIT, early)
        st = ctx.build_host(buf, True)
        _check_build(ctx, st, ref)
        used.append(int(st.build_flags) & 1)
    ctx.close()
    # build 1 may still fall back (its capacity estimate comes from build 0's
    # ratios alone); from build 2 on the estimate holds
    assert used[0] == 0 and used[2] == 1 and used[3] == 0 and used[4] == 1, used


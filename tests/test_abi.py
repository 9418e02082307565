"""CPU-side checks of the drop-in boundary and the host logic (no GPU calls)."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "pangenome.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|uint64_t|const char\*)\s+(pg_\w+)\s*\(", text, re.M)))


def test_library_exports_every_declared_symbol():
    from pangenome_amd import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    syms = declared_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
    # and the ctypes binding covers exactly the header
    assert sorted(_lib.SIGNATURES) == syms


def test_binding_marshals_round6_entry_points():
    """The ctypes argument lists of the round-6 entry points accept what the
    Context methods pass (a NULL context: each returns PG_EINVAL, no device
    touched)."""
    from pangenome_amd import _lib
    lib = _lib.load()

    class Fake:
        pass
    f = Fake()
    f.lib, f.h = lib, None
    with pytest.raises(_lib.PangenomeError, match="pg_route_merge_segs"):
        _lib.Context.route_merge_segs(f, [(0x1000, 3), (0, 0)], 4, True)
    with pytest.raises(_lib.PangenomeError, match="pg_stream_wait"):
        _lib.Context.stream_wait(f, 0)
    with pytest.raises(_lib.PangenomeError, match="pg_route_rows_checksum"):
        _lib.Context.route_rows_checksum(f, 0x1000, np.array([0, 3, 5], np.uint64))


def test_routed_row_hash_matches_the_16_byte_form():
    """A 12-byte routed row {h, mask word} hashes as the 16-byte record
    {h, mask word, 0} (the senders' sums and the receivers' checks agree
    across the two layouts)."""
    from pangenome_amd.dist import row_check_sum
    rng = np.random.default_rng(6)
    h = rng.integers(0, 2 ** 63, 1000, dtype=np.uint64)
    m = rng.integers(0, 2 ** 26, 1000, dtype=np.uint64)
    r16 = np.stack([h, m], axis=1).view(np.int64)
    r12 = np.stack([(h & np.uint64(0xFFFFFFFF)).astype(np.uint32), (h >> np.uint64(32)).astype(np.uint32),
                    m.astype(np.uint32)], axis=1)
    assert row_check_sum(r12) == row_check_sum(r16) == row_check_sum(r16.view(np.int32).reshape(-1, 4))
    assert row_check_sum(r12[:0]) == 0


def test_no_device_fails_loudly():
    """Without a GPU the product raises; it never falls back to a CPU path."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from pangenome_amd import _lib
    with pytest.raises(_lib.PangenomeError):
        _lib.Context(27)


def test_eval_number():
    from pangenome_amd.host import eval_number
    assert eval_number("2**63") == 2 ** 63
    assert eval_number("5e8") == 500000000
    assert eval_number("1000") == 1000
    with pytest.raises(ValueError):
        eval_number("__import__('os')")


def test_parse_args_reference_forms():
    from pangenome_amd.kmer import parse_args
    a = parse_args(["x", "-i", "f.fa", "-k27", "--weird", "-c", "3"])
    assert a["-i"] == "f.fa" and a["-k"] == "27" and a["-c"] == "3" and a["-n"] == "2**63"


def test_plan_dbg_checkpoints():
    from pangenome_amd import host
    lens = np.array([10, 10, 10, 10], np.int64)
    shape_gt = host.FileShape(ord(">"), True, 0, False)
    shape_junk = host.FileShape(ord("j"), True, 20, False)
    # chunk 25 with rc (20 per record): checkpoint after record 1 and record 3
    f, extra = host.plan_dbg(lens, shape_gt, True, 2 ** 63, chunk=25)
    assert f.tolist() == [1, 1, 1, 1] and extra == 1           # resume at EOF -> empty record
    f, extra = host.plan_dbg(lens, shape_junk, True, 2 ** 63, chunk=25)
    assert f.tolist() == [1, 1, 0, 1] and extra == 0           # record after the checkpoint lost
    # -n: the dBG pass counts both strands; stops after the record that crosses
    f, _ = host.plan_dbg(lens, shape_gt, True, 30)
    assert f.tolist() == [1, 1, 0, 0]
    f, _ = host.plan_dbg(lens, shape_gt, False, 30)
    assert f.tolist() == [1, 1, 1, 1]


def test_plan_checkpoint_states():
    """The state of the last <in>_db_brkpt / <in>_rdb_brkpt dump (:1255-1259,
    :1880-1887): records inserted when it was written, and the record whose
    seqio ptr is its offset; None without a checkpoint."""
    from pangenome_amd import host
    lens = np.array([10, 10, 10, 10], np.int64)
    shape_gt = host.FileShape(ord(">"), True, 0, False)
    f, extra, ck = host.plan_dbg(lens, shape_gt, True, 2 ** 63, chunk=25, checkpoint=True)
    assert f.tolist() == [1, 1, 1, 1] and extra == 1
    cf, ce, last = ck                                          # dumps after records 1 and 3: the last wins
    assert cf.tolist() == [1, 1, 1, 1] and ce == 0 and last == 3
    f, _, ck = host.plan_dbg(lens, shape_gt, True, 2 ** 63, chunk=45, checkpoint=True)
    assert ck[0].tolist() == [1, 1, 1, 0] and ck[2] == 2
    assert host.plan_dbg(lens, shape_gt, True, 2 ** 63, checkpoint=True)[2] is None
    f, seg, ncp, last = host.plan_edges(lens, shape_gt, 2 ** 63, chunk=15, checkpoint=True)
    assert seg.tolist() == [0, 0, 1, 1] and ncp == 2 and last == 3     # dumps after records 1 and 3
    assert host.plan_edges(lens, shape_gt, 2 ** 63, checkpoint=True)[3] is None


def test_write_edge_npz_popitem_order(tmp_path):
    from pangenome_amd import host
    t = np.arange(12, dtype=np.uint64).reshape(3, 4)
    host.write_edge_npz(str(tmp_path / "e"), t, np.array([5, 6, 7]), 99)
    off, lt, lc = host.read_edge_npz(str(tmp_path / "e.npz"))
    assert off == 99 and lt.tolist() == t[::-1].tolist() and lc.tolist() == [7, 6, 5]


def test_plan_edges_and_rows():
    from pangenome_amd import host
    lens = np.array([10, 10, 10], np.int64)
    shape = host.FileShape(ord(">"), True, 0, False)
    f, seg, ncp = host.plan_edges(lens, shape, 2 ** 63, chunk=15)
    assert f.tolist() == [1, 1, 1] and seg.tolist() == [0, 0, 1] and ncp == 1
    assert host.plan_rows(lens, shape, b">a\n", 15).tolist() == [1, 1, 0]
    # a file starting with '\n' then record 0's header: lost in the label pass
    assert host.plan_rows(lens, host.FileShape(10, True, 1, False), b"\n>a\n", 2 ** 63).tolist() == [0, 1, 1]


def test_edge_order_reversal():
    from pangenome_amd import host
    walk_first = np.array([0, 0, 2, 4, 4], np.int64)        # records 0, 0, 1, 2, 2
    seg = np.array([0, 1, 1], np.int64)
    order = host.edge_order(walk_first, seg, 1)
    # segment 0 = [0, 1] reversed -> [1, 0], then append [2, 3, 4]
    assert order.tolist() == [1, 0, 2, 3, 4]


def test_label_dict_matches_oracle(oracle_mod):
    from pangenome_amd import host
    xyz = "1_2\t3_4\t1\n3_4\t5_6\t2\n7_8\t1_2\t1\n"
    mcl = "3_4\t9_9\n"
    a = host.label_dict(mcl, xyz.splitlines(keepends=True))
    k, v, i = oracle_mod.label_table(xyz, mcl)
    assert a == {(int(x), int(y)): int(z) for x, y, z in zip(k, v, i)}


def test_oakht_capacity_chain_matches_oracle(oracle_mod):
    """pg_oakht_capacity (host-only) against the oracle's faithful oakht growth
    (find_prime(2^20), x1.62 at load 0.75, kmer_numba.py:423-474) at sizes on
    both sides of the first two resizes."""
    from pangenome_amd import _lib, synth
    lib = ctypes.CDLL(_lib.LIB_PATH)
    lib.pg_oakht_capacity.restype = ctypes.c_uint64
    lib.pg_oakht_capacity.argtypes = [ctypes.c_uint64]
    assert lib.pg_oakht_capacity(0) == 1048583
    assert lib.pg_oakht_capacity(786437) == 1048583        # 0.75 * 1048583 = 786437.25
    assert lib.pg_oakht_capacity(786438) > 1048583
    for n_bases in (380_000, 420_000, 700_000):
        fa = synth.to_fasta_lines(b"g", synth.base_genome(n_bases, seed=n_bases))
        run = oracle_mod.OracleRun(fa, 27, 2)
        keys, _ = run.dbg()
        assert lib.pg_oakht_capacity(keys.shape[0]) == run.dbg_capacity()


def test_db_npz_roundtrip(tmp_path):
    """write_db_npz / read_db_npz: dump()'s parameters row and slot arrays
    (:243-261); only counts > 0 slots come back (iteritems :623-631)."""
    from pangenome_amd import host
    keys = np.array([0, 5, 0, 2 ** 64 - 1, 9], np.uint64)
    vals = np.array([0, 3, 0, 32, 65], np.uint16)
    cnts = np.array([0, 2, 0, 1, 255], np.uint8)
    host.write_db_npz(str(tmp_path / "x_db"), 5, 3, keys, vals, cnts, offset=77)
    z = np.load(str(tmp_path / "x_db.npz"))
    assert z["parameters"].tolist() == [5, 750000000, 3, 1, 1, 77]
    off, k, v, c = host.read_db_npz(str(tmp_path / "x_db.npz"))
    assert off == 77 and k.tolist() == [5, 2 ** 64 - 1, 9] and v.tolist() == [3, 32, 65] and c.tolist() == [2, 1, 255]
    np.savez_compressed(str(tmp_path / "edges"), parameters=np.array([4, 1, 0], np.uint64),
                        keys=np.zeros(8, np.uint64), values=np.zeros(2, np.int64))
    with pytest.raises(ValueError):
        host.read_db_npz(str(tmp_path / "edges.npz"))
    assert host.resume_position(0, np.array([10, 20])) == 0
    assert host.resume_position(20, np.array([10, 20])) == 2
    with pytest.raises(ValueError):
        host.resume_position(15, np.array([10, 20]))


def test_reference_checkpoint_files_parse():
    """The checkpoints the reference wrote (tests/golden/resume) read back in
    both layouts: oakht (-r) and the jit edge Dict (-R)."""
    from golden_util import ResumeFixture, resume_names
    from pangenome_amd import host
    seen = set()
    for name in resume_names():
        fx = ResumeFixture(name)
        if fx.flag == "-r":
            off, k, v, c = host.read_db_npz(fx.brkpt)
            assert off > 0 and k.shape[0] == v.shape[0] == c.shape[0] > 0 and c.min() >= 1
        else:
            off, t, c = host.read_edge_npz(fx.brkpt)
            assert off > 0 and t.shape == (c.shape[0], 4) and c.min() >= 1
        seen.add(fx.flag)
    assert seen == {"-r", "-R"}


def test_merge_edges_order():
    """Resumed Dict: loaded items, known edges updated in place, new ones
    appended, whole Dict reversed at a checkpoint (kmer_numba.py:1859-1887)."""
    from pangenome_amd import host
    lt = np.array([[1, 1, 2, 2], [3, 3, 4, 4]], np.uint64)
    lc = np.array([5, 6], np.int64)
    t = np.array([[3, 3, 4, 4], [7, 7, 8, 8], [9, 9, 9, 9]], np.uint64)
    c = np.array([1, 1, 2], np.int64)
    walk_first = np.array([0, 0, 2], np.int64)          # records 0, 0, 1
    ot, oc = host.merge_edges(lt, lc, t, c, walk_first, np.array([0, 0], np.int64), 0)
    assert ot[:, 0].tolist() == [1, 3, 7, 9] and oc.tolist() == [5, 7, 1, 2]
    ot, oc = host.merge_edges(lt, lc, t, c, walk_first, np.array([0, 1], np.int64), 1)
    assert ot[:, 0].tolist() == [7, 3, 1, 9] and oc.tolist() == [1, 7, 5, 2]


def test_label_table_matches_label_dict():
    """The array form of the label dictionary equals the text-parsing one
    (which test_label_dict_matches_oracle pins to the oracle), with and
    without a non-empty .mcl (repeated tokens: a later line wins)."""
    from pangenome_amd import host
    rng = np.random.default_rng(5)
    nodes = rng.integers(0, 40, (300, 2)).astype(np.uint64)
    nodes[:, 0] = nodes[:, 0] * np.uint64(1_000_003) + np.uint64(2 ** 62)
    e = rng.integers(0, 300, (500, 2))
    tuples = np.concatenate([nodes[e[:, 0]], nodes[e[:, 1]]], axis=1)
    counts = rng.integers(1, 9, 500)
    xyz = host.xyz_text(tuples, counts)
    toks = ["%d_%d" % tuple(nodes[i]) for i in rng.integers(0, 300, 40)]
    for mcl in ("", "\t".join(toks[:10]) + "\n" + "\t".join(toks[5:25]) + "\n" + toks[30] + "\n"):
        lab = host.label_dict(mcl, xyz.splitlines(keepends=True))
        k, v, i = host.label_table(mcl, tuples)
        got = dict(zip(zip(k.view(np.uint64).tolist(), v.tolist()), i.tolist()))
        assert got == lab
        assert list(got) == list(lab)                  # same insertion order


def test_native_text_formatters():
    """pg_format_xyz / pg_format_rows produce the reference's text
    (kmer_numba.py:1901 and :1949), including unsigned 64-bit keys and
    negative or large fields."""
    from pangenome_amd import _lib, host
    t = np.array([[2 ** 64 - 1, 32, 0, 1], [123456789012345678, 5, 7, 40]], np.uint64)
    c = np.array([1, 987654321], np.int64)
    assert _lib.format_xyz(t, c).decode() == host.xyz_text(t, c)
    rows = np.array([[0, 0, 27, 1, 3], [1, 5, 2 ** 31 - 1, 0, 0], [0, 10, 12, 0, 2 ** 40]], np.int64)
    names = [b"g0 desc", "quéry".encode()]
    want = "".join("%s\t%d\t%d\t%s\t%d\n" % (names[r].decode(), s, e, "+" if st == 1 else "-", lab)
                   for r, s, e, st, lab in rows.tolist())
    assert _lib.format_rows(rows, names).decode() == want
    assert _lib.format_xyz(np.zeros((0, 4), np.uint64), np.zeros(0, np.int64)) == b""

"""The host side of the npz side files (CPU): host.savez_stored writes the zip
np.savez writes (stored .npy members, ZIP64 records), in parallel pieces,
and np.load / zipfile read it back bit for bit with valid CRCs; the lazy
label table refuses to read labels a later label pass replaced."""
import zipfile

import numpy as np
import pytest


@pytest.mark.parametrize("piece", [1 << 10, 1 << 16, 32 << 20])
def test_savez_stored_roundtrip(tmp_path, piece, monkeypatch):
    from pangenome_amd import host
    monkeypatch.setattr(host, "NPZ_PIECE", piece)
    rng = np.random.default_rng(piece)
    arrs = {"parameters": np.array([5, 750000000, 3, 1, 1, 0], np.uint64),
            "keys": rng.integers(0, 2 ** 63, size=200_003, dtype=np.uint64),
            "values": rng.integers(0, 4096, size=200_003).astype(np.uint16),
            "counts": rng.integers(0, 256, size=200_003).astype(np.uint8),
            "empty": np.zeros(0, np.int64), "matrix": rng.integers(0, 9, size=(7, 4)).astype(np.int64)}
    fn = str(tmp_path / "x")
    host.savez_stored(fn, **arrs)
    assert zipfile.ZipFile(fn + ".npz").testzip() is None          # every member's CRC
    with np.load(fn + ".npz", allow_pickle=False) as z:
        assert sorted(z.files) == sorted(arrs)
        for k, v in arrs.items():
            assert z[k].dtype == v.dtype and z[k].shape == v.shape and np.array_equal(z[k], v), k


def test_savez_stored_deferred_members_match_savez(tmp_path):
    """Members written by a fill callback (what pg_dbg_dump_fd does from the
    device) give the same file as the arrays themselves: same bytes."""
    import os
    import zlib
    from pangenome_amd import host
    rng = np.random.default_rng(5)
    keys = rng.integers(0, 2 ** 63, size=70_001, dtype=np.uint64)
    vals = rng.integers(0, 4096, size=70_001).astype(np.uint16)
    cnts = rng.integers(0, 256, size=70_001).astype(np.uint8)
    host.write_db_npz(str(tmp_path / "a_db"), 70_001, 123, keys, vals, cnts, offset=9)

    def fill(fd, offs):
        out = []
        for a, o in zip((keys, vals, cnts), offs):
            b = a.view(np.uint8).tobytes()
            assert os.pwrite(fd, b, o) == len(b)
            out.append(zlib.crc32(b))
        return out
    host.write_db_npz_from(str(tmp_path / "b_db"), 70_001, 123, fill, offset=9)
    a = open(tmp_path / "a_db.npz", "rb").read()
    b = open(tmp_path / "b_db.npz", "rb").read()
    assert a == b
    assert zipfile.ZipFile(str(tmp_path / "b_db.npz")).testzip() is None


def test_write_db_npz_reads_back(tmp_path):
    from pangenome_amd import host
    keys = np.array([0, 11, 0, 42], np.uint64)
    vals = np.array([0, 3, 0, 64], np.uint16)
    cnts = np.array([0, 1, 0, 255], np.uint8)
    host.write_db_npz(str(tmp_path / "d_db"), 4, 2, keys, vals, cnts, offset=77)
    off, k, v, c = host.read_db_npz(str(tmp_path / "d_db.npz"))
    assert off == 77 and k.tolist() == [11, 42] and v.tolist() == [3, 64] and c.tolist() == [1, 255]
    with np.load(str(tmp_path / "d_db.npz")) as z:
        assert z["parameters"].tolist() == [4, host.DB_LOAD, 2, 1, 1, 77]


def test_label_table_invalidated_by_later_pass():
    from pangenome_amd._lib import Context
    from pangenome_amd.kmer import LabelTable

    class FakeCtx:                                  # the label part of a Context, no device
        labels = Context.labels

        def __init__(self):
            self.n_labels, self.label_gen = 0, 1
    ctx = FakeCtx()
    gen = ctx.label_gen
    table = LabelTable(loader=lambda: ctx.labels(gen))
    ctx.label_gen += 1                              # a later set_labels / labels_from_edges
    with pytest.raises(RuntimeError, match="replaced by a later label pass"):
        len(table)

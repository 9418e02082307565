"""The CPU oracle (oracle/pg_oracle.c) against the reference's own outputs.

Every fixture under tests/golden/ was produced by running
/root/reference/kmer_numba.py (tests/golden/make_goldens.py).  This pins the
oracle before anything is compared with it.
"""
import numpy as np
import pytest

from golden_util import Fixture, fixture_names


@pytest.mark.parametrize("name", fixture_names())
def test_oracle_matches_reference(oracle_mod, name):
    fx = Fixture(name)
    out = oracle_mod.run_pipeline(fx.fasta, fx.k, fx.c, fx.ns, fx.mcl, edge_chunk=fx.edge_chunk)
    assert np.array_equal(out["dbg_keys"], fx.dbg_keys)
    assert np.array_equal(out["dbg_masks"], fx.dbg_masks)
    assert np.array_equal(out["rdbg_keys"], fx.rdbg_keys)
    assert out["xyz"] == fx.xyz
    assert out["rows"] == fx.rows


@pytest.mark.parametrize("name", fixture_names())
def test_oracle_counts_match_reference_dump(oracle_mod, name):
    """The oakht occurrence counts and capacity the reference wrote to
    `<in>_db.npz` (:243-261)."""
    fx = Fixture(name)
    run = oracle_mod.OracleRun(fx.fasta, fx.k, fx.c, fx.ns)
    keys, masks, counts = run.dbg_counts()
    assert np.array_equal(keys, fx.dbg_keys)
    assert np.array_equal(counts, fx.dbg_counts)
    assert run.dbg_capacity() == int(fx.db_params[0])
    assert int(fx.db_params[2]) == keys.shape[0]


def test_label_table_order(oracle_mod):
    # .mcl line index first, then unseen .xyz nodes (kmer_numba.py:1918-1944)
    xyz = "1_2\t3_4\t1\n3_4\t5_6\t2\n7_8\t1_2\t1\n"
    mcl = "3_4\t9_9\n"
    keys, vals, ids = oracle_mod.label_table(xyz, mcl)
    got = {(int(a), int(b)): int(c) for a, b, c in zip(keys, vals, ids)}
    assert got == {(3, 4): 0, (9, 9): 0, (1, 2): 1, (5, 6): 2, (7, 8): 3}


def test_k_plus_one_record_numba_semantics(oracle_mod):
    """n == k+1: numba binds the never-entered loop variable to 0.

    Hand-derived (not reference-pinned: pure-Python raises UnboundLocalError
    there, so no golden exists): window 2 has key digits s[1..k-1], s[1];
    predecessor s[-k mod n] = s[1]; successor '$'.
    """
    k = 5
    s = b"ACGTAC"                       # n = 6 = k + 1
    run = oracle_mod.OracleRun(b">r\n" + s + b"\n", k, c=0)
    keys, masks = run.dbg()
    alpha = {ord("A"): 0, ord("G"): 1, ord("C"): 2, ord("T"): 3}
    lastc = {ord("A"): 1, ord("T"): 2, ord("G"): 4, ord("C"): 8}
    key0 = sum(alpha[c] * 5 ** j for j, c in enumerate(s[:k]))
    key1 = key0 // 5 + alpha[s[1]] * 5 ** (k - 1)
    expect = {key0: (0 << 6) | lastc[s[k]], key1: (lastc[s[1]] << 6) | 32}
    assert dict(zip(keys.tolist(), masks.tolist())) == expect


def test_sentinel_and_empty(oracle_mod):
    # n < k -> one sentinel occurrence, key 2^64-1, mask '$' (32); in the rdBG
    run = oracle_mod.OracleRun(b">a\nACG\n>b\n", 27, c=2)
    keys, masks = run.dbg()
    assert keys.tolist() == [2 ** 64 - 1] and masks.tolist() == [32]
    assert run.rdbg().tolist() == [2 ** 64 - 1]


@pytest.mark.parametrize("name", fixture_names())
def test_oracle_key_ranges_match_reference(oracle_mod, name):
    """pgo_dbg_range (the sorted form the benchmark-scale digests use for
    inputs too big for one oakht) gives the reference's dBG and rdBG range by
    range, at the fixture's -c, -n and checkpoint settings."""
    fx = Fixture(name)
    ks, ms = [], []
    for lo, hi in oracle_mod.key_ranges(fx.k, 7):
        k_, m_ = oracle_mod.dbg_range(fx.fasta, fx.k, fx.c, lo, hi, ns=fx.ns)
        assert np.all(np.diff(k_.astype(np.float64)) >= 0) and np.all((k_ >= lo) & ((k_ < hi) | (k_ == hi)))
        ks.append(k_)
        ms.append(m_)
    keys, masks = np.concatenate(ks), np.concatenate(ms)
    assert np.array_equal(keys, fx.dbg_keys)
    assert np.array_equal(masks, fx.dbg_masks)
    assert np.array_equal(keys[oracle_mod.rdbg_member(masks)], fx.rdbg_keys)

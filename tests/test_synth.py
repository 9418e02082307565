"""The synthetic workload generators (pangenome_amd/synth.py): deterministic
per (seed, genome, record), the shapes SURVEY.md §8(d) names."""
import numpy as np

from dist_util import seqio_records


def test_c5_record_is_deterministic_and_independent():
    from pangenome_amd import synth
    a = synth.c5_record(3, 5, record_len=200_000)
    assert a == synth.c5_record(3, 5, record_len=200_000)
    assert a != synth.c5_record(4, 5, record_len=200_000)            # another genome
    assert a != synth.c5_record(3, 6, record_len=200_000)            # another base segment
    (sl, hs, hl, _), = seqio_records(a)
    assert a[hs:hs + hl] == b">g3_c5" and abs(sl - 200_000) < 2_000   # 0.1 % indels
    seq = a[hl + 1:].replace(b"\n", b"")
    assert set(seq) <= set(b"ACGT") and len(seq) == sl
    # 1 % SNP against the genome-0 copy of the same segment
    b = synth.c5_record(0, 5, record_len=200_000)
    assert 0.5 < sum(x != y for x, y in zip(a[hl + 1:hl + 20001], b[hl + 1:hl + 20001])) / 20000 * 100


def test_write_c5_streams_records(tmp_path):
    from pangenome_amd import synth
    n = synth.write_c5(str(tmp_path / "c5.fa"), n_genomes=2, records=3, record_len=50_000)
    buf = (tmp_path / "c5.fa").read_bytes()
    assert len(buf) == n
    recs = seqio_records(buf)
    assert len(recs) == 6
    assert [buf[h + 1:h + l] for _, h, l, _ in recs] == [b"g%d_c%d" % (g, r) for g in range(2) for r in range(3)]
    assert synth.CONFIGS["c5"]["records"] * synth.CONFIGS["c5"]["n_genomes"] == 240

"""INTEGRATION.md's ctypes stub (the binding a maintainer of kmer_numba.py would
add), executed as written with the library path filled in: the rdBG and the
`_db.npz` dump of a golden input against what the reference produced."""
import os
import re
import types

import numpy as np
import pytest

from golden_util import Fixture

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def stub_source():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    blocks = re.findall(r"```python\n(.*?)```", text, re.S)
    src = next(b for b in blocks if b.startswith("# pangenome_gpu.py"))
    return src.replace("/path/to/pangenome_amd/libpangenome_hip.so",
                       os.path.join(ROOT, "pangenome_amd", "libpangenome_hip.so"))


def test_stub_binds_every_symbol_it_uses():
    """CPU: every pg_* name the stub calls is declared in include/pangenome.h."""
    src = stub_source()
    header = open(os.path.join(ROOT, "include", "pangenome.h")).read()
    used = set(re.findall(r"_L\.(pg_\w+)", src))
    assert used and all(re.search(r"\b%s\(" % n, header) for n in used), used


@pytest.mark.gpu
def test_stub_matches_reference(tmp_path):
    fx = Fixture("pan8_k27_c2")
    q = tmp_path / "input.fsa"
    q.write_bytes(fx.fasta)
    G = types.ModuleType("pangenome_gpu")
    exec(compile(stub_source(), "INTEGRATION.md:pangenome_gpu.py", "exec"), G.__dict__)
    h = G.dbg2rdbg(G.seq2rdbg(str(q), kmer=27, rc=True))
    assert np.array_equal(G.rdbg_keys(h), fx.rdbg_keys)
    G.dump(h, str(tmp_path / "db"))
    G.free(h)
    z = np.load(str(tmp_path / "db.npz"))
    sel = z["counts"] > 0
    o = np.argsort(z["keys"][sel], kind="stable")
    assert np.array_equal(z["keys"][sel][o], fx.dbg_keys)
    assert np.array_equal(z["values"][sel][o], fx.dbg_masks)
    assert np.array_equal(z["counts"][sel][o], fx.dbg_counts)
    assert z["parameters"].tolist() == fx.db_params.tolist()

#!/usr/bin/env python3
"""Development trace (not part of the product): 6 host-window builds of C3
batch A (pg_build_host from a populated mmap), for rocprofv3 --kernel-trace
--memory-copy-trace; tools/trace_step.py-style analysis reads the db."""
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    from pangenome_amd import kmer, synth
    from pangenome_amd._lib import Context
    d = tempfile.mkdtemp()
    q = os.path.join(d, "c3.fa")
    synth.write_pangenome(q, 100, 5_000_000, workers=8)
    mm = kmer.seq2bytes(q)
    ctx = Context(27)
    for _ in range(6):
        st = ctx.build_host(mm, True)
    print(st.n_dbg, st.n_rdbg, flush=True)


if __name__ == "__main__":
    main()

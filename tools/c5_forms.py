#!/usr/bin/env python3
"""Development check (not part of the product): the 3.75 Gbp C5 shard of
test_c5_shard_full_size_properties streamed at world 1 over RCCL, per
coverage form (PG_TUNE_K3_COVER 0 packed / 1 LDS-staged / 2 quad) and chunk
size, twice each, to tell a form's error from a nondeterministic one."""
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _diag_rank(rank, world, port, q, path, chunk_bases):
    """_c5_rank with every chunk build's and every merge's statistics printed."""
    import test_gpu_c5
    from pangenome_amd import dist as D

    def wrap(name):
        f = getattr(D.GpuShard, name)

        def g(self, *a, **kw):
            t0 = time.time()
            r = f(self, *a, **kw)
            st = self.ctx.stats()
            n = a[1] if name == "merge" and len(a) > 1 else -1
            print("  %s n=%s -> n_dbg %d n_canon? recA %d flags %#x bb? %.0f ms" %
                  (name, n, st.n_dbg, st.n_records_a, st.build_flags, 1e3 * (time.time() - t0)), flush=True)
            return r
        setattr(D.GpuShard, name, g)
    wrap("build")
    wrap("merge")
    test_gpu_c5._c5_rank(rank, world, port, q, path, "nccl", chunk_bases, None, False, None)


def main():
    from pangenome_amd import synth
    import test_gpu_c5
    from dist_util import spawn_ranks
    runs = [a.split(":") for a in (sys.argv[1:] or ["0:30", "0:30", "2:30", "1:30", "0:29"])]
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as d:
        p = os.path.join(d, "c5_shard0.fa")
        t0 = time.time()
        synth.write_c5(p, pairs=[(0, r) for r in range(24)] + [(1, r) for r in range(6)], workers=10)
        print("generated in %.0f s" % (time.time() - t0), flush=True)
        for form, cb in runs:
            os.environ["PG_TEST_K3_COVER"] = form
            if os.environ.get("C5_DIAG"):
                r = spawn_ranks(1, _diag_rank, (p, 1 << int(cb)), timeout=500)[0]
            else:
                r = spawn_ranks(1, test_gpu_c5._c5_rank, (p, "nccl", 1 << int(cb), None, False, None), timeout=500)[0]
            print("form %s chunk 2^%s: %s" % (form, cb, r["stream"]), flush=True)


if __name__ == "__main__":
    main()

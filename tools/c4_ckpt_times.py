#!/usr/bin/env python3
"""Development timing (not part of the product): kmer.seq2rdbg's checkpoint
route on C4 (5.08 GB, 10 Gbp of strand bases > 2^33: the prefix build, the
<in>_db_brkpt npz, the whole pass) phase by phase, twice (the second run has
warm mappings and buffers).  Prints one JSON line per run."""
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    from pangenome_amd import host, kmer
    d = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
    path = os.path.join(d, "c4.fa")
    t0 = time.time()
    subprocess.run([sys.executable, "-m", "pangenome_amd.synth", "c4", path, "16"], cwd=ROOT, check=True, timeout=600)
    print("generated in %.0f s" % (time.time() - t0), flush=True)
    for run in range(2):
        tm = {}
        t = time.perf_counter()
        g = kmer.DeviceGraph(path, 27, 0)
        tm["map_parse"] = time.perf_counter() - t
        t = time.perf_counter()
        flags, extra, ckpt = host.plan_dbg(g.seq_len, g.shape, True, 2 ** 63, 2 ** 33, resume=None, checkpoint=True)
        tm["plan"] = time.perf_counter() - t
        cf, ce, last = ckpt
        t = time.perf_counter()
        g.ctx.build_dbg(cf, ce, True)
        tm["prefix_build"] = time.perf_counter() - t
        t = time.perf_counter()
        cap, size = g.ctx.dbg_dump_size()
        tm["dump_counts"] = time.perf_counter() - t
        t = time.perf_counter()
        host.write_db_npz_from(path + "_db_brkpt", cap, size, lambda fd, offs: g.ctx.dbg_dump_fd(fd, offs, cap),
                               offset=int(g.rec_ptr[last]))
        tm["dump_write"] = time.perf_counter() - t
        t = time.perf_counter()
        st = g.ctx.build_dbg(flags, extra, True)
        tm["full_build"] = time.perf_counter() - t
        out = {k: round(1e3 * v, 1) for k, v in tm.items()}
        out.update(run=run, n_dbg=int(st.n_dbg), ckpt_bytes=os.path.getsize(path + "_db_brkpt.npz"))
        print(json.dumps(out), flush=True)
        g.ctx.close()
        del g


if __name__ == "__main__":
    main()

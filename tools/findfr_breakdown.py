#!/usr/bin/env python3
"""Development timing (not part of the product): where `# find fr` (seq2graph,
kmer_numba.py:1853-1951) goes on C3 batch A at -c 2 - the edge pass, the
.xyz text and its file, the labels, the row pass and the row text, each step
of kmer.seq2graph timed on its own (three repeats).  Prints one JSON line;
writes only into a temp directory."""
import io
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    from scale_util import make_input
    from pangenome_amd import host, kmer
    fasta = make_input("c3a")
    d = tempfile.mkdtemp()
    q = os.path.join(d, "c3.fa")
    open(q, "wb").write(fasta)
    del fasta
    g = kmer.seq2rdbg(q, 27, 5, 2 ** 63, brkpt="", chunk=2 ** 33, rc=True, device=0)
    kmer.dbg2rdbg(g)
    oname = q + "_rdbg_weight.xyz"
    open(oname + ".mcl", "w").close()
    res = {}

    def tick(name, t0):
        t = time.perf_counter()
        res.setdefault(name, []).append(round(1e3 * (t - t0), 1))
        return t

    for rep in range(3):
        t = time.perf_counter()
        kmer.rdbg_edges(g, 2 ** 63, 2 ** 33, False, brkpt="", keep_on_device=True)
        t = tick("edges_ms", t)
        xyz = g.ctx.edges_text()
        t = tick("edges_text_ms", t)
        with open(oname, "wb") as f:
            f.write(xyz)
        t = tick("xyz_write_ms", t)
        with open(oname + ".mcl", "r") as f:
            mk, mv, mi, nxt = host.mcl_labels(f.read())
        g.ctx.labels_from_edges(None, mk, mv, mi, nxt)
        t = tick("labels_ms", t)
        flags = host.plan_rows(g.seq_len, g.shape, g.buf, 2 ** 63)
        t = tick("plan_rows_ms", t)
        n_rows = g.ctx.rows_count(flags, False)
        t = tick("rows_ms", t)
        names = [bytes(g.buf[int(hs) + 1:int(hs) + int(hl)]) for hs, hl in zip(g.hdr_start, g.hdr_len)]
        text = g.ctx.rows_text(names)
        t = tick("rows_text_ms", t)
        out = io.BytesIO()
        out.write(text)
        t = tick("rows_sink_ms", t)
        with open(oname, "wb") as f:
            g.ctx.edges_write(f.fileno())
        t = tick("xyz_fd_ms", t)
        with open(os.path.join(d, "rows.txt"), "wb") as f:
            g.ctx.rows_write(names, f.fileno())
        t = tick("rows_fd_ms", t)
        r, w = os.pipe()
        import threading
        th = threading.Thread(target=lambda: [None for _ in iter(lambda: os.read(r, 1 << 20), b"")])
        th.start()
        g.ctx.rows_write(names, w)
        os.close(w)
        th.join()
        os.close(r)
        t = tick("rows_pipe_ms", t)
        res.update(n_rows=int(n_rows), rows_bytes=len(text), xyz_bytes=len(xyz))
        del text, out, xyz
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

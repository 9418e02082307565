#!/usr/bin/env python3
"""Development timing (not part of the product): where `# save dBG to disk`
goes on C3 batch A - pg_dbg_dump (device placement + the copy of the slot
arrays to the host) against the stored-npz writer, and the writer's CRC and
pwrite halves alone.  Prints one JSON line; writes nothing but a temp file."""
import json
import os
import sys
import tempfile
import time
import zlib
from concurrent.futures import ThreadPoolExecutor

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
    res = {}
    for rep in range(3):
        t0 = time.perf_counter()
        cap, size, keys, values, counts = g.ctx.dbg_dump()
        t1 = time.perf_counter()
        host.write_db_npz(os.path.join(d, "db%d" % rep), cap, size, keys, values, counts)
        t2 = time.perf_counter()
        res.setdefault("dump_ms", []).append(round(1e3 * (t1 - t0), 1))
        res.setdefault("write_ms", []).append(round(1e3 * (t2 - t1), 1))
    for rep in range(3):
        fn = os.path.join(d, "nat%d_db" % rep)
        t0 = time.perf_counter()
        kmer.dump(g, fn)
        res.setdefault("native_dump_ms", []).append(round(1e3 * (time.perf_counter() - t0), 1))
        os.unlink(fn + ".npz")
    nbytes = keys.nbytes + values.nbytes + counts.nbytes
    pieces = [a.reshape(-1).view(np.uint8)[p:p + host.NPZ_PIECE] for a in (keys, values, counts)
              for p in range(0, a.nbytes, host.NPZ_PIECE)]
    with ThreadPoolExecutor(16) as ex:
        t0 = time.perf_counter()
        list(ex.map(lambda x: zlib.crc32(memoryview(x)), pieces))
        t1 = time.perf_counter()
        fd = os.open(os.path.join(d, "raw"), os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
        offs = np.cumsum([0] + [x.shape[0] for x in pieces])
        list(ex.map(lambda i: os.pwrite(fd, memoryview(pieces[i]), int(offs[i])), range(len(pieces))))
        os.close(fd)
        t2 = time.perf_counter()
    res.update(crc_only_ms=round(1e3 * (t1 - t0), 1), pwrite_only_ms=round(1e3 * (t2 - t1), 1),
               capacity=int(cap), size=int(size), bytes=int(nbytes), tmp=d, cpus=os.cpu_count())
    t0 = time.perf_counter()
    z = np.empty(cap, np.uint64)
    z[:] = 1
    res["touch_keys_ms"] = round(1e3 * (time.perf_counter() - t0), 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

"""Drop-in for kmer_numba.py's k-mer -> dBG -> rdBG -> region-table path.

Same names, arguments and side files as the reference; every per-base step
runs in libpangenome_hip.so on an MI355X (pangenome_amd/csrc).  Mirrors:

  seq_chk      kmer_numba.py:873-885     file type sniffing
  seq2bytes    :117-119                  memory-map the input
  seq2rdbg     :1234-1268                dBG build (K1 parse + K3 insert)
  dbg2rdbg     :1313-1321                rdBG (K5 degree scan + compaction)
  seq2graph    :1853-1951                edges -> .xyz -> mcl -> labels -> rows
  dump / load_on_disk  :243-335         `<in>_db.npz` (oakht slot layout)
  entry_point  :1971-2146                CLI (-i -k -n -c -r -d -R -D)

Usage:  python -m pangenome_amd -i genomes.fa -k 27 > result.tab
"""
from __future__ import annotations

import mmap
import os
import sys
from time import time

import numpy as np

from collections.abc import Mapping

from . import host
from ._lib import Context, format_xyz


class LabelTable(Mapping):
    """seq2graph's label dictionary {(key, value): label} (:1918-1944), kept as
    arrays (or on the device, fetched by `loader` when first needed); the
    Python dict is built only if it is looked into."""

    def __init__(self, keys=None, vals=None, ids=None, loader=None):
        self._arrays = None if loader is not None else (keys, vals, ids)
        self._loader = loader
        self._d = None

    @property
    def keys_(self):
        return self._get()[0]

    @property
    def vals_(self):
        return self._get()[1]

    @property
    def ids_(self):
        return self._get()[2]

    def _get(self):
        if self._arrays is None:
            self._arrays = self._loader()
            self._loader = None
        return self._arrays

    def _dict(self):
        if self._d is None:
            k = self.keys_.view(np.uint64).tolist()
            self._d = dict(zip(zip(k, self.vals_.tolist()), self.ids_.tolist()))
        return self._d

    def __getitem__(self, key):
        return self._dict()[key]

    def __iter__(self):
        return iter(self._dict())

    def __len__(self):
        return int(self.ids_.shape[0])


# --------------------------------------------------------------- input files
def seq_chk(qry):
    """:873-885 — 'fasta' if a header starts the first 40 characters."""
    with open(qry, "r") as f:
        seq = f.read(2 * 20)
    if seq[0].startswith(">") or "\n>" in seq:
        return "fasta"
    if seq[0].startswith("@") or "\n@" in seq:
        return "fastq"
    return None


def seq2bytes(fn, populate=True):
    """:117-119 (read-only here: nothing is written back to the input).  The
    mapping's page tables are filled when it is made (MAP_POPULATE: one pass
    in the kernel, ~8 ms per GB of page-cache-warm file), so the staging
    threads that copy it to the GPU never stop on a page fault (demand faults
    from 8 threads at once took 3.7 s for C4's 5 GB)."""
    if not os.path.getsize(fn):
        return np.zeros(0, np.uint8)
    flags = mmap.MAP_SHARED | (getattr(mmap, "MAP_POPULATE", 0) if populate else 0)
    with open(fn, "rb") as f:
        mm = mmap.mmap(f.fileno(), 0, flags=flags, prot=mmap.PROT_READ)
    return np.frombuffer(mm, dtype=np.uint8)


def populate(buf, start: int, end: int):
    """Fill the page tables of bytes [start, end) of a seq2bytes(...,
    populate=False) mapping (madvise MADV_POPULATE_READ, Linux 5.14+;
    silently nothing elsewhere)."""
    mm = getattr(buf, "base", None)
    if not isinstance(mm, mmap.mmap) or end <= start:
        return
    a = start - start % mmap.PAGESIZE
    try:
        mm.madvise(22, a, end - a)                       # MADV_POPULATE_READ
    except (OSError, ValueError, AttributeError):
        pass


class DeviceGraph:
    """The device-resident dBG/rdBG of one input (what the reference keeps in
    its `oakht` tables), plus the parsed record table the later passes reuse.
    With `build_rc` set, the input is parsed and its dBG built in one call
    (pg_build_host: the build's first stage streamed under the upload), for a
    pass that inserts every record; otherwise it is only parsed."""

    def __init__(self, qry, kmer, device=0, data=None, build_rc=None, ctx=None):
        self.qry = qry
        self.k = min(max(1, int(kmer)), 27)                    # :1236
        self.buf = seq2bytes(qry) if data is None else data
        self.ctx = ctx if ctx is not None else Context(self.k, device)
        self.stats = None
        if build_rc is None:
            self.ctx.parse_host(self.buf)        # H2D in chunks, pipelined with K1
        else:
            self.stats = self.ctx.build_host(self.buf, bool(build_rc))
        rec = self.ctx.records()
        self.seq_len, self.hdr_start, self.hdr_len = rec["seq_len"], rec["hdr_start"], rec["hdr_len"]
        self.rec_ptr = rec["ptr"]
        self.shape = host.FileShape.from_bytes(self.buf, self.hdr_start, self.hdr_len)
        self.reduced = False

    @property
    def size(self):
        return self.stats.n_dbg if self.stats else 0

    def dbg_items(self):
        """(keys, masks) sorted by key — dump()'s content (:243-261)."""
        return self.ctx.dbg()

    def rdbg_keys(self):
        return self.ctx.rdbg()


# ------------------------------------------------------------------- passes
def seq2rdbg(qry, kmer=13, bits=5, Ns=1e6, chunk=2 ** 32, brkpt="./breakpoint", saved="dBG_disk",
             hashfunc=None, jit=True, rc=True, device=0, ctx=None):
    """:1234-1268.  Returns the device dBG.  An existing `brkpt` npz (-r) is
    the table so far plus the offset to resume at (:1239-1241).  When a pass
    crosses `chunk` bases the reference dumps the table so far to
    `<in>_db_brkpt.npz` (:1255-1259, each dump replacing the last); here the
    last such state is built, dumped and written once, then the whole build
    runs.  `ctx`: a Context to build in (the CLI creates it before its
    stage timer starts, so the timer excludes HIP runtime start-up)."""
    if seq_chk(qry) != "fasta":
        raise ValueError("%s: only FASTA input is supported (the reference's FASTQ branch is "
                         "broken, kmer_numba.py:174-186)" % qry)
    mult = 2 if rc else 1
    nbytes = os.path.getsize(qry)
    if not (brkpt and os.path.isfile(brkpt)) and nbytes * mult <= int(chunk) and not host.ns_hit(nbytes * mult, int(Ns)):
        # no -r resume, and no -n limit or 2^33-base checkpoint can touch a
        # file this size (bases <= bytes): every record is in the pass, so
        # parse and build in one call with the build streamed under the upload
        g = DeviceGraph(qry, kmer, device, build_rc=bool(rc), ctx=ctx)
        flags, extra = host.plan_dbg(g.seq_len, g.shape, bool(rc), int(Ns), int(chunk))
        if extra or not flags.all():                      # (cannot happen: bases <= bytes)
            g.stats = g.ctx.build_dbg(flags, extra, bool(rc))
        return g
    g = DeviceGraph(qry, kmer, device, ctx=ctx)
    resume = None
    if brkpt and os.path.isfile(brkpt):
        offset, keys, values, counts = host.read_db_npz(brkpt)
        g.ctx.dbg_load(keys, values, counts)
        resume = host.resume_position(offset, g.rec_ptr)
    flags, extra, ckpt = host.plan_dbg(g.seq_len, g.shape, bool(rc), int(Ns), int(chunk), resume=resume,
                                       checkpoint=True)
    if ckpt is not None:
        cf, ce, last = ckpt
        g.ctx.build_dbg(cf, ce, bool(rc))
        # the checkpoint file streamed from the device (pg_dbg_dump_fd: no
        # host copy of the slot arrays; C4: ~2.7 GB of them), then the pass
        cap, size = g.ctx.dbg_dump_size()
        host.write_db_npz_from(qry + "_db_brkpt", cap, size, lambda fd, offs: g.ctx.dbg_dump_fd(fd, offs, cap),
                               offset=int(g.rec_ptr[last]))
    g.stats = g.ctx.build_dbg(flags, extra, bool(rc))
    return g


def dump(g: DeviceGraph, fn="./tmp"):
    """:243-261 — `fn`.npz as an oakht the reference's load_on_disk accepts."""
    cap, size = g.ctx.dbg_dump_size()
    host.write_db_npz_from(fn, cap, size, lambda fd, offs: g.ctx.dbg_dump_fd(fd, offs, cap))
    return 0


def load_graph(qry, kmer, fn, device=0, rdbg=False, rc=True):
    """load_on_disk (:289-335) into a device graph over `qry`: -d (a dBG,
    reduced next) or -D (rdBG keys: staged with mask 0, so every key passes
    the rdBG rule and membership is exactly the file's key set)."""
    _, keys, values, counts = host.read_db_npz(fn)
    g = DeviceGraph(qry, kmer, device)
    g.ctx.dbg_load(keys, None if rdbg else values, counts)
    g.stats = g.ctx.build_dbg(np.zeros(g.seq_len.shape[0], np.uint8), 0, bool(rc))
    return g


def dbg2rdbg(kmer_dict):
    """:1313-1321.  Reduces in place on the device and returns the same graph."""
    kmer_dict.stats = kmer_dict.ctx.build_rdbg()
    kmer_dict.reduced = True
    return kmer_dict


def rdbg_edges(g: DeviceGraph, Ns, chunk, rc, brkpt="", keep_on_device=False):
    """Edge Dict of rdbg_edge_weight_jit_ (:1808-1827) in its iteration order;
    an existing `brkpt` (-R) is the Dict so far and the offset to resume at.
    With keep_on_device and neither a -R resume nor a checkpoint (the order is
    then the device's first-occurrence order), the edges stay on the device
    and None is returned."""
    loaded, resume = None, None
    if brkpt and os.path.isfile(brkpt):
        offset, lt, lc = host.read_edge_npz(brkpt)
        loaded, resume = (lt, lc), host.resume_position(offset, g.rec_ptr)
    flags, segment, ncp, ckpt = host.plan_edges(g.seq_len, g.shape, int(Ns), int(chunk), resume=resume,
                                                checkpoint=True)
    if keep_on_device and loaded is None and ncp == 0:
        g.ctx.edges_count(flags, bool(rc))
        return None

    def state(fl, upto):                          # the Dict after segments 0..upto, in iteration order
        tuples, counts, walk_first = g.ctx.edges(fl, bool(rc))
        if loaded is not None:
            return host.merge_edges(loaded[0], loaded[1], tuples, counts, walk_first, segment, upto)
        order = host.edge_order(walk_first, segment, upto)
        return tuples[order], counts[order]
    if ckpt is not None:
        # the last `<in>_rdb_brkpt.npz` dump (:1880-1887): the Dict after the
        # segments before the last checkpoint, each dump replacing the last
        last_seg = ncp - 1
        t, c = state((flags.astype(bool) & (segment <= last_seg)).astype(np.uint8), last_seg)
        host.write_edge_npz(g.qry + "_rdb_brkpt", t, c, int(g.rec_ptr[ckpt]))
    return state(flags, ncp)


def seq2graph(qry, kmer=13, bits=5, Ns=1e6, brkpt="./breakpoint_rdbg.npz", rdbg_dict=None, saved=None,
              hashfunc=None, jit=True, chunk=2 ** 33, rc=False, cluster=True, out=None):
    """:1853-1951: edge weights -> `<qry>_rdbg_weight.xyz` -> mcl (or reuse)
    -> label dictionary -> print the region rows.  The edges, the label
    table, the rows and both texts are made on the device; the host writes
    the files and runs (or reuses) mcl."""
    out = out or sys.stdout
    g = rdbg_dict
    res = rdbg_edges(g, Ns, chunk, rc, brkpt=brkpt, keep_on_device=True)
    oname = qry + "_rdbg_weight.xyz"
    with open(oname, "wb") as f:                      # "%d_%d\t%d_%d\t%d\n" (:1893-1904)
        if res is None:
            f.flush()
            g.ctx.edges_write(f.fileno())             # formatted on the device, streamed into the file
        else:
            f.write(format_xyz(*res))
    if cluster:
        if os.path.isfile("%s.mcl" % oname):
            print("# the mcl has been ran", file=out)
        else:
            out.flush()
            os.system("mcl %s --abc -I 1.5 -te 8 -o %s.mcl -q x -V all" % (oname, oname))
    with open(oname + ".mcl", "r") as f:
        mcl_text = f.read()
    mk, mv, mi, nxt = host.mcl_labels(mcl_text)              # :1918-1929
    g.ctx.labels_from_edges(None if res is None else res[0], mk, mv, mi, nxt)     # :1932-1944
    flags = host.plan_rows(g.seq_len, g.shape, g.buf, int(Ns))
    g.ctx.rows_count(flags, bool(rc))
    names = [bytes(g.buf[int(hs) + 1:int(hs) + int(hl)]) for hs, hl in zip(g.hdr_start, g.hdr_len)]
    fd = _fileno(out)                                 # print('%s\t%d\t%d\t%s\t%d') (:1946-1949)
    if fd is not None:
        out.flush()
        out.buffer.flush()
        g.ctx.rows_write(names, fd)                   # formatted on the device, streamed to the descriptor
    else:
        text = g.ctx.rows_text(names)
        if text:
            if hasattr(out, "buffer"):
                out.flush()
                out.buffer.write(text)
                out.buffer.flush()
            else:
                out.write(text.decode())
    gen = g.ctx.label_gen
    return LabelTable(loader=lambda: g.ctx.labels(gen))           # (raises once a later label pass replaced it)


def _fileno(out):
    """The descriptor under a text stream's binary buffer (stdout, a file),
    or None (a stand-in with no descriptor)."""
    try:
        return out.buffer.fileno()
    except (AttributeError, OSError, ValueError):   # (io.UnsupportedOperation is an OSError)
        return None


# ---------------------------------------------------------------------- CLI
def manual_print(out=None):
    out = out or sys.stdout
    for line in ("Usage:", "  pyhton this.py -i qry.fsa -k 10 -n 1000000", "Parameters:",
                 "  -i: query sequences in fasta format", "  -k: kmer length",
                 "  -d: the de bruijn graph", "  -r: break point of de bruijn graph",
                 "  -D: the reduced de bruijn graph", "  -R: break point of reduced de bruijn graph",
                 "  -n: length of query sequences for pan-genomic analysis",
                 "  -c: complementary reverse sequence. 00,01,10,11"):
        print(line, file=out)


def parse_args(argv):
    """:1983-1997 — same flag handling, including `-k27` and skipped unknowns."""
    args = {"-i": "", "-k": "50", "-n": "2**63", "-r": "", "-d": "", "-R": "", "-D": "", "-c": "2"}
    N = len(argv)
    for i in range(1, N):
        k = argv[i]
        if k in args:
            args[k] = argv[i + 1]
        elif k[:2] in args and len(k) > 2:
            args[k[:2]] = k[2:]
    return args


def entry_point(argv, out=None, device=0):
    out = out or sys.stdout
    args = parse_args(argv)
    qry, kmer, Ns = args["-i"], int(args["-k"]), host.eval_number(args["-n"])
    bkt, dbs, rbk, rc, rdb = args["-r"], args["-d"], args["-R"], int(args["-c"]), args["-D"]
    if not qry:
        manual_print(out)
        raise SystemExit()
    chunk = 2 ** 33
    rc0, rc1 = (rc >> 1) == 1, (rc & 1) == 1
    if dbs or rdb:                                    # :2073-2101
        if not rdb:
            print("load dBG from disk", file=out)
            kmer_dict = load_graph(qry, kmer, dbs, device, rdbg=False, rc=rc0)
            print("# build the reduced dBG", file=out)
            rdbg_dict = dbg2rdbg(kmer_dict)
        else:
            rdbg_dict = dbg2rdbg(load_graph(qry, kmer, rdb, device, rdbg=True, rc=rc0))
        print("# find fr", file=out)
        seq2graph(qry, kmer=kmer, bits=5, Ns=Ns, rdbg_dict=rdbg_dict, chunk=chunk, brkpt=rbk, rc=rc1, out=out)
        return 0
    ctx = Context(min(max(1, kmer), 27), device)     # HIP runtime start-up before the stage timer
    print("# build the dBG", file=out)
    st = time()
    kmer_dict = seq2rdbg(qry, kmer, 5, Ns, brkpt=bkt, chunk=chunk, rc=rc0, device=device, ctx=ctx)
    print("# finished in", time() - st, "seconds", file=out)
    print("# save dBG to disk", file=out)
    st = time()
    dump(kmer_dict, qry + "_db")
    print("# finished in", time() - st, "seconds", file=out)
    # the reference reloads the file it just wrote (:2120-2126); the device
    # table is that same dBG, so nothing is read back
    print("# load dBG from disk", file=out)
    st = time()
    print("# finished in", time() - st, "seconds", file=out)
    print("# build the reduced dBG", file=out)
    st = time()
    rdbg_dict = dbg2rdbg(kmer_dict)
    print("# finished in", time() - st, "seconds", file=out)
    print("# find fr", file=out)
    st = time()
    seq2graph(qry, kmer=kmer, bits=5, Ns=Ns, rdbg_dict=rdbg_dict, chunk=chunk, brkpt=rbk, rc=rc1, out=out)
    print("# finished in", time() - st, "seconds", file=out)
    return 0


def main():
    return entry_point(sys.argv)

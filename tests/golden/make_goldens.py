#!/usr/bin/env python3
"""Generate golden fixtures by running the reference ``kmer_numba.py`` itself.

Run ONLY in the build container (it needs ``/root/reference``; it refuses to run
elsewhere).  numba is not importable here, so the reference is
imported in pure-Python mode through a throwaway ``numba``/``Bio`` shim created
in a temp dir, plus the numba-typing emulations SURVEY.md §8c lists:

1. ``alpha``/``lastc`` widened int8 -> int64 (numba promotes int8 arithmetic);
2. ``nbit`` argument widened (uint16 ``>>`` under NEP 50);
3. negative ints stored into uint64 arrays wrap (the n<k sentinel, :1038);
4. the uint8 ``counts`` array widened so 255+1 does not wrap to 0 (numpy 2);
5. ``np.empty`` returns zero-filled memory, as numba's fresh-mmap allocations
   of the multi-MB ``oakht`` arrays do (NRT only poisons the first 256 B, and
   key 0's home slot is >= 213275 for every capacity of the 1.62x growth
   chain).  Without this, recycled heap bytes in never-written slots make
   ``has_key`` (:599-603, no ``counts`` check) report stale keys as members.

Records of length exactly k+1 raise ``UnboundLocalError`` in pure Python
(numba instead binds the loop variable to 0), so fixture inputs avoid them.

Each fixture directory gets: ``input.fsa``, ``meta.json``, ``rows.tsv`` (the
5-field region rows, in order), ``rdbg_weight.xyz`` (the edge file),
``dbg_keys.npy``/``dbg_masks.npy`` (the dBG, sorted by key) and
``rdbg_keys.npy`` (sorted).  Nothing here is imported by the tests.
"""
from __future__ import annotations

import contextlib
import gzip
import io
import json
import os
import shutil
import sys
import tempfile
import warnings

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"

SHIM_NUMBA = r'''
import numpy as _np
class _T:
    def __init__(self, name, dt, bits, signed):
        self.name, self.dtype, self.bits, self.signed = name, _np.dtype(dt), bits, signed
    def __call__(self, x):
        v = int(x) & ((1 << self.bits) - 1)
        if self.signed and v >= (1 << (self.bits - 1)):
            v -= (1 << self.bits)
        return v
    def __getitem__(self, k):
        return self
uint64 = _T('uint64', 'uint64', 64, False); uint32 = _T('uint32', 'uint32', 32, False)
uint16 = _T('uint16', 'uint16', 16, False); uint8 = _T('uint8', 'uint8', 8, False)
int64 = _T('int64', 'int64', 64, True); int32 = _T('int32', 'int32', 32, True)
int16 = _T('int16', 'int16', 16, True); int8 = _T('int8', 'int8', 8, True)
longlong = int64; ulonglong = uint64; float32 = 'float32'; float64 = 'float64'
def njit(*a, **kw):
    if len(a) == 1 and callable(a[0]) and not kw:
        return a[0]
    return lambda f: f
jit = njit
prange = range
def jitclass(spec):
    return lambda cls: cls
'''
SHIM_TYPED = r'''
Dict = dict
class List(list):
    @staticmethod
    def empty_list(t):
        return List()
'''


def load_reference():
    if not os.path.isfile(os.path.join(REF, "kmer_numba.py")):
        raise SystemExit("make_goldens.py needs /root/reference (build container only)")
    shim = tempfile.mkdtemp(prefix="pg_shim_")
    os.makedirs(os.path.join(shim, "numba"))
    os.makedirs(os.path.join(shim, "Bio"))
    with open(os.path.join(shim, "numba", "__init__.py"), "w") as f:
        f.write(SHIM_NUMBA)
    with open(os.path.join(shim, "numba", "typed.py"), "w") as f:
        f.write(SHIM_TYPED)
    with open(os.path.join(shim, "numba", "experimental.py"), "w") as f:
        f.write("from numba import jitclass\n")
    with open(os.path.join(shim, "Bio", "__init__.py"), "w") as f:
        f.write("SeqIO = None\n")
    sys.dont_write_bytecode = True
    warnings.simplefilter("ignore")
    sys.path.insert(0, shim)
    sys.path.insert(1, REF)
    import kmer_numba as K  # noqa: E402  (pure-Python mode)

    a64, l64 = K.alpha.astype(np.int64), K.lastc.astype(np.int64)
    for name in list(vars(K)):
        fn = getattr(K, name)
        if callable(fn) and getattr(fn, "__defaults__", None):
            fn.__defaults__ = tuple(a64 if d is K.alpha else l64 if d is K.lastc else d
                                    for d in fn.__defaults__)
    K.alpha, K.lastc = a64, l64
    nbit = K.nbit
    K.nbit_jit_ = lambda n: nbit(int(n))

    class Wrap64(np.ndarray):
        def __setitem__(self, i, v):
            if isinstance(v, (int, np.integer)) and self.dtype == np.uint64:
                v = int(v) & 0xFFFFFFFFFFFFFFFF
            super().__setitem__(i, v)

    class NP:
        def __getattr__(self, a):
            return getattr(np, a)

        def empty(self, *a, **kw):
            r = np.zeros(*a, **kw)              # emulation 5: fresh zeroed pages
            return r.view(Wrap64) if r.dtype == np.uint64 else r

        def zeros(self, *a, **kw):
            dt = kw.get("dtype", a[1] if len(a) > 1 else None)
            if dt is not None and np.dtype(getattr(dt, "dtype", dt)) == np.uint8:
                kw["dtype"] = np.int64          # emulation 4: counts never wrap
                a = a[:1]
            return np.zeros(*a, **kw)

    K.np = NP()
    return K, shim


def run_fixture(K, name, input_name, fasta: bytes, k, c=2, n=None, mcl=None, chunk=None):
    """Run the reference CLI (or its stage functions when ``chunk`` is given)."""
    out_dir = os.path.join(HERE, name)
    if os.path.isdir(out_dir):
        shutil.rmtree(out_dir)
    os.makedirs(out_dir)
    os.makedirs(os.path.join(HERE, "inputs"), exist_ok=True)
    os.makedirs(os.path.join(HERE, "graphs"), exist_ok=True)
    inp = os.path.join(HERE, "inputs", input_name + ".fsa")
    with open(inp, "wb") as f:
        f.write(fasta)
    work = tempfile.mkdtemp(prefix="pg_gold_")
    qry = os.path.join(work, "input.fsa")
    with open(qry, "wb") as f:
        f.write(fasta)
    with open(qry + "_rdbg_weight.xyz.mcl", "w") as f:
        f.write(mcl or "")

    captured = {}
    orig = K.dbg2rdbg

    def dbg2rdbg(d):
        r = orig(d)
        captured["rdbg"] = np.asarray(r.keys)[np.asarray(r.counts) > 0].astype(np.uint64)
        return r

    K.dbg2rdbg = dbg2rdbg
    buf = io.StringIO()
    try:
        with contextlib.redirect_stdout(buf):
            if chunk is None:
                argv = ["kmer_numba.py", "-i", qry, "-k", str(k), "-c", str(c)]
                if n is not None:
                    argv += ["-n", str(n)]
                K.entry_point(argv)
            else:
                # same stage order as entry_point :2104-2144 with a small edge-pass chunk
                # so the checkpoint dump/reload order reversal (:1881-1887) is exercised
                Ns = int(eval(str(n))) if n is not None else 2 ** 63
                kd = K.seq2rdbg(qry, k, 5, Ns, brkpt="", chunk=2 ** 33, rc=(c >> 1) == 1)
                K.dump(kd, qry + "_db")
                _, kd = K.load_on_disk(qry + "_db.npz")
                rd = K.dbg2rdbg(kd)
                K.seq2graph(qry, kmer=k, bits=5, Ns=Ns, rdbg_dict=rd, chunk=chunk, brkpt="",
                            rc=(c & 1) == 1)
    finally:
        K.dbg2rdbg = orig
    stdout = buf.getvalue()
    rows = [ln for ln in stdout.split("\n")
            if len(ln.split("\t")) == 5 and ln.split("\t")[3] in ("+", "-")]

    db = np.load(qry + "_db.npz")
    cnt = db["counts"]
    keys = db["keys"][cnt > 0].astype(np.uint64)
    masks = db["values"][cnt > 0].astype(np.uint16)
    counts = cnt[cnt > 0].astype(np.uint8)          # the reference's own dump (:243-261)
    params = db["parameters"].astype(np.uint64)
    o = np.argsort(keys, kind="stable")
    rdbg = np.sort(captured["rdbg"])

    # the dBG/rdBG depend only on (input, k, dBG strand bit, -n): share them
    graph = "%s_k%d_rc%d%s" % (input_name, k, c >> 1, "" if n is None else "_n%s" % n)
    gpath = os.path.join(HERE, "graphs", graph + ".npz")
    if os.path.isfile(gpath):
        g = np.load(gpath)
        assert np.array_equal(g["dbg_keys"], keys[o]) and np.array_equal(g["dbg_masks"], masks[o])
        assert np.array_equal(g["rdbg_keys"], rdbg)
        assert np.array_equal(g["dbg_counts"], counts[o]) and np.array_equal(g["db_params"], params)
    else:
        np.savez_compressed(gpath, dbg_keys=keys[o], dbg_masks=masks[o], rdbg_keys=rdbg,
                            dbg_counts=counts[o], db_params=params)
    with open(qry + "_rdbg_weight.xyz", "rb") as f, \
            gzip.GzipFile(os.path.join(out_dir, "rdbg_weight.xyz.gz"), "wb", mtime=0) as g:
        g.write(f.read())
    with gzip.GzipFile(os.path.join(out_dir, "rows.tsv.gz"), "wb", mtime=0) as g:
        g.write("".join(r + "\n" for r in rows).encode())
    if mcl:
        with open(os.path.join(out_dir, "input.mcl"), "w") as f:
            f.write(mcl)
    meta = dict(input=input_name + ".fsa", graph=graph + ".npz", k=k, c=c, n=n,
                mcl="fixture" if mcl else "empty", chunk=chunk,
                n_dbg=int(keys.shape[0]), n_rdbg=int(rdbg.shape[0]), n_rows=len(rows),
                n_edges=sum(1 for _ in open(qry + "_rdbg_weight.xyz")),
                generator="tests/golden/make_goldens.py (reference kmer_numba.py, pure-Python mode)")
    with open(os.path.join(out_dir, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    shutil.rmtree(work)
    print("%-18s k=%-2d c=%d dbg=%-7d rdbg=%-6d edges=%-6d rows=%d" % (
        name, k, c, meta["n_dbg"], meta["n_rdbg"], meta["n_edges"], meta["n_rows"]), file=sys.stderr)
    return meta


def run_resume_fixture(K, name, input_name, fasta: bytes, k, c, flag, chunk):
    """A checkpoint written by the reference itself, then its CLI resuming from
    it: flag "-r" (seq2rdbg's `<in>_db_brkpt.npz`, :1255-1259) or "-R"
    (seq2graph's `<in>_rdb_brkpt.npz`, :1880-1887).  Stored under resume/."""
    out_dir = os.path.join(HERE, "resume", name)
    os.makedirs(out_dir)
    work = tempfile.mkdtemp(prefix="pg_gold_")
    qry = os.path.join(work, "input.fsa")
    with open(qry, "wb") as f:
        f.write(fasta)
    with open(qry + "_rdbg_weight.xyz.mcl", "w") as f:
        f.write("")
    with contextlib.redirect_stdout(io.StringIO()):
        if flag == "-r":
            K.seq2rdbg(qry, k, 5, 2 ** 63, brkpt="", chunk=chunk, rc=(c >> 1) == 1)
            brk = qry + "_db_brkpt.npz"
        else:
            kd = K.seq2rdbg(qry, k, 5, 2 ** 63, brkpt="", chunk=2 ** 33, rc=(c >> 1) == 1)
            rd = K.dbg2rdbg(kd)
            K.seq2graph(qry, kmer=k, bits=5, Ns=2 ** 63, rdbg_dict=rd, chunk=chunk, brkpt="", rc=(c & 1) == 1)
            brk = qry + "_rdb_brkpt.npz"
            os.remove(qry + "_rdbg_weight.xyz")
    saved = os.path.join(out_dir, "brkpt.npz")
    with np.load(brk) as z:                            # counts as numba writes them (uint8); the
        arrs = {a: z[a] for a in z.files}              # shim widened them (emulation 4)
    if "counts" in arrs:
        assert arrs["counts"].max() <= 255
        arrs["counts"] = arrs["counts"].astype(np.uint8)
    np.savez_compressed(saved, **arrs)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        K.entry_point(["kmer_numba.py", "-i", qry, "-k", str(k), "-c", str(c), flag, saved])
    rows = [ln for ln in buf.getvalue().split("\n")
            if len(ln.split("\t")) == 5 and ln.split("\t")[3] in ("+", "-")]
    with open(qry + "_rdbg_weight.xyz", "rb") as f, \
            gzip.GzipFile(os.path.join(out_dir, "rdbg_weight.xyz.gz"), "wb", mtime=0) as g:
        g.write(f.read())
    with gzip.GzipFile(os.path.join(out_dir, "rows.tsv.gz"), "wb", mtime=0) as g:
        g.write("".join(r + "\n" for r in rows).encode())
    meta = dict(input=input_name + ".fsa", k=k, c=c, flag=flag, chunk=chunk, n_rows=len(rows),
                generator="tests/golden/make_goldens.py (reference kmer_numba.py, pure-Python mode)")
    if flag == "-r":                                   # the dBG the resumed run dumped: a graph file
        db = np.load(qry + "_db.npz")
        cnt = db["counts"]
        keys = db["keys"][cnt > 0].astype(np.uint64)
        o = np.argsort(keys, kind="stable")
        graph = "%s_k%d_rc%d" % (input_name, k, c >> 1)
        g = np.load(os.path.join(HERE, "graphs", graph + ".npz"))
        assert np.array_equal(g["dbg_keys"], keys[o])
        assert np.array_equal(g["dbg_masks"], db["values"][cnt > 0].astype(np.uint16)[o])
        assert np.array_equal(g["dbg_counts"], cnt[cnt > 0].astype(np.uint8)[o])
        meta["graph"] = graph + ".npz"
    with open(os.path.join(out_dir, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    shutil.rmtree(work)
    print("%-18s resume %s k=%d c=%d rows=%d" % (name, flag, k, c, len(rows)), file=sys.stderr)


def edge_case_fasta() -> bytes:
    """Hand-built edge cases (no record of length k+1)."""
    from pangenome_amd import synth
    rnd = lambda n, s: bytes(synth.ACGT[synth.base_genome(n, s)])
    lines = [b"junkline_before_header\n"]
    # lowercase + N + IUPAC + '$' / '#' bytes inside a record, multi-line
    r0 = bytearray(rnd(700, 11))
    r0[50:80] = r0[50:80].lower()
    r0[200] = ord("N"); r0[201] = ord("n"); r0[300] = ord("R"); r0[420] = ord("Y")
    r0[500] = ord("$"); r0[560] = ord("#"); r0[610:640] = b"N" * 30
    lines.append(b">rec0 lower/N/IUPAC/$/#\n")
    lines += [bytes(r0[i:i + 70]) + b"\n" for i in range(0, len(r0), 70)]
    lines.append(b">short_lt_k\n" + rnd(10, 12) + b"\n")            # n < k27
    lines.append(b">exact_k27\n" + rnd(27, 13) + b"\n")             # n == 27
    lines.append(b">empty_record\n")                                 # n == 0
    lines.append(b">k_plus_2\n" + rnd(29, 14) + b"\n")              # n == k+2
    # CRLF record: '\r' stays in the sequence (each line loses only '\n')
    r5 = rnd(400, 15)
    lines.append(b">crlf record\r\n")
    lines += [r5[i:i + 60] + b"\r\n" for i in range(0, 400, 60)]
    # repeats shared between records so the rdBG and edges are non-trivial
    rep = rnd(300, 16)
    for j in range(4):
        body = bytearray(rnd(200, 20 + j) + rep + rnd(150, 30 + j))
        body[100 + 3 * j] = ord("ACGT"[j])
        lines.append(b">rep%d\n" % j + bytes(body) + b"\n")
    rc_rep = bytes(synth.ACGT[3 - synth.base_genome(300, 16)][::-1])
    lines.append(b">rev_rep\n" + rnd(90, 40) + rc_rep + rnd(90, 41) + b"\n")
    # final record without trailing newline: its last byte is dropped (:131-132, :167)
    lines.append(b">no_trailing_newline\n" + rnd(200, 42) + rep[:120])
    return b"".join(lines)


def polya_fasta() -> bytes:
    """Records with poly-A runs so key 0 (all-A) is a real k-mer (Q6)."""
    from pangenome_amd import synth
    rnd = lambda n, s: bytes(synth.ACGT[synth.base_genome(n, s)])
    out = []
    for j in range(4):
        body = rnd(900 + 37 * j, 60 + j) + b"A" * (40 + 5 * j) + rnd(1000, 70 + j)
        out.append(b">pa%d\n" % j + b"\n".join(body[i:i + 60] for i in range(0, len(body), 60)) + b"\n")
    return b"".join(out)


def components_mcl(xyz_path: str) -> str:
    """A non-empty .mcl stand-in: connected components of the .xyz graph,
    largest first (pins the label-line logic, Q11; not micans mcl output)."""
    parent = {}

    def find(x):
        while parent.setdefault(x, x) != x:
            parent[x] = parent[parent[x]]
            x = parent[x]
        return x

    order = []
    for ln in open(xyz_path):
        a, b = ln.rstrip("\n").split("\t")[:2]
        for t in (a, b):
            if t not in parent:
                order.append(t)
        ra, rb = find(a), find(b)
        if ra != rb:
            parent[ra] = rb
    comps = {}
    for t in order:
        comps.setdefault(find(t), []).append(t)
    cc = sorted(comps.values(), key=lambda c: -len(c))
    # keep only every other component so the unseen-node path (:1932-1944) runs too
    return "".join("\t".join(c) + "\n" for c in cc[::2])


def main():
    from pangenome_amd import synth
    K, shim = load_reference()
    for d in os.listdir(HERE):
        if os.path.isdir(os.path.join(HERE, d)) and d != "__pycache__":
            shutil.rmtree(os.path.join(HERE, d))
    try:
        test_fsa = open(os.path.join(REF, "test", "test.fsa"), "rb").read()
        run_fixture(K, "test_k5", "test", test_fsa, 5)
        run_fixture(K, "test_k5_c3", "test", test_fsa, 5, c=3)
        run_fixture(K, "test_k27", "test", test_fsa, 27)
        run_fixture(K, "test_k3_c1", "test", test_fsa, 3, c=1)
        run_fixture(K, "test_k1", "test", test_fsa, 1)
        edge = edge_case_fasta()
        run_fixture(K, "edge_k27", "edge", edge, 27)
        run_fixture(K, "edge_k27_c3", "edge", edge, 27, c=3)
        run_fixture(K, "edge_k11", "edge", edge, 11, c=3)
        run_fixture(K, "edge_k5", "edge", edge, 5)
        run_fixture(K, "polya_k27", "polya", polya_fasta(), 27, c=3)
        pan = synth.pangenome(8, 20000, snp=0.01, indel=0.001, seed=0xBEEF)
        for c in (0, 1, 2, 3):
            run_fixture(K, "pan8_k27_c%d" % c, "pan8", pan, 27, c=c)
        run_fixture(K, "pan8_k15", "pan8", pan, 15, c=3)
        run_fixture(K, "pan8_k27_n", "pan8", pan, 27, c=3, n=70000)
        run_fixture(K, "pan8_k27_chunk", "pan8", pan, 27, c=3, chunk=30000)
        mcl = components_mcl_from(os.path.join(HERE, "pan8_k27_c3", "rdbg_weight.xyz.gz"))
        run_fixture(K, "pan8_k27_mcl", "pan8", pan, 27, c=3, mcl=mcl)
        run_resume_fixture(K, "pan8_k27_r", "pan8", pan, 27, 3, "-r", 100000)
        run_resume_fixture(K, "pan8_k27_R", "pan8", pan, 27, 3, "-R", 30000)
    finally:
        shutil.rmtree(shim, ignore_errors=True)


def components_mcl_from(xyz_gz):
    tmp = tempfile.mktemp()
    with gzip.open(xyz_gz, "rb") as f, open(tmp, "wb") as g:
        g.write(f.read())
    try:
        return components_mcl(tmp)
    finally:
        os.unlink(tmp)


if __name__ == "__main__":
    sys.path.insert(0, REPO)
    main()

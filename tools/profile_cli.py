#!/usr/bin/env python3
"""Development profile (not part of the product): the CLI's stages on C3 batch
A (kmer.entry_point, empty .mcl) under cProfile, to see where `# find fr`
goes.  Writes the top functions by cumulative time to gpurun_out/."""
import cProfile
import io
import os
import pstats
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


class Out:
    def __init__(self):
        self.buffer = io.BytesIO()

    def write(self, s):
        self.buffer.write(s.encode())

    def flush(self):
        pass


def main():
    from scale_util import make_input
    from pangenome_amd import kmer
    c = sys.argv[1] if len(sys.argv) > 1 else "2"
    fasta = make_input("c3a")
    d = tempfile.mkdtemp()
    q = os.path.join(d, "c3.fa")
    open(q, "wb").write(fasta)
    open(q + "_rdbg_weight.xyz.mcl", "w").close()
    del fasta
    kmer.entry_point(["x", "-i", q, "-k", "27", "-c", c], out=Out())      # warm (first touches)
    out = Out()
    pr = cProfile.Profile()
    pr.enable()
    kmer.entry_point(["x", "-i", q, "-k", "27", "-c", c], out=out)
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(45)
    lines = [ln for ln in out.buffer.getvalue().split(b"\n") if ln.startswith(b"#")]
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/profile_cli_c%s.txt" % c, "w") as f:
        f.write("\n".join(x.decode() for x in lines) + "\n\n" + s.getvalue())
    print("\n".join(x.decode() for x in lines))


if __name__ == "__main__":
    main()

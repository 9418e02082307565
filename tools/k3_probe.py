"""Development probe: K3 phase costs on a bench workload (GPU).

Times build_dbg under the PG_K3 (tile | group) and PG_K3_DBG knobs
(1 = windows only, 2 = HBM loads without updates, 4 = group form without its
HBM phase) at a fixed table size.  Not part of the product path or the tests.

    python tools/k3_probe.py [--config c3] [--reps 3]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--variants", default="tile:0,tile:1,tile:2,group:0,group:1,group:4,group:2")
    a = ap.parse_args()
    import torch
    import bench
    from pangenome_amd._lib import Context
    fasta, desc = bench.workload(a.config, 0, 1)
    d = torch.frombuffer(bytearray(fasta), dtype=torch.uint8).to("cuda:0")
    torch.cuda.synchronize()
    ctx = Context(27)
    ctx.set_fasta_device(d.data_ptr(), d.numel(), keepalive=d)
    ctx.parse()
    st = ctx.build_dbg(None, 0, True)                 # real build: learns the table size
    keys = int(st.n_slots * 1.25)
    print("workload:", desc, "canonical keys:", st.n_slots, flush=True)
    os.environ["PG_K3_KEYS"] = str(keys)
    for v in a.variants.split(","):
        mode, dbg = v.split(":")
        os.environ["PG_K3"] = mode
        res = []
        for _ in range(a.reps):
            if dbg == "0":
                os.environ.pop("PG_K3_DBG", None)
            else:
                os.environ["PG_K3_DBG"] = dbg
            s = ctx.build_dbg(None, 0, True)
            res.append(s.ms_insert)
        os.environ.pop("PG_K3_DBG", None)
        print("%-6s dbg=%s insert ms: %s" % (mode, dbg, " ".join("%.3f" % x for x in res)), flush=True)


if __name__ == "__main__":
    main()

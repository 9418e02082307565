#!/usr/bin/env python3
"""C5-form timing probe on one GPU (development tool, not the bench).

* c5m (1.25 Gbp, 10 x 125 Mbp records at 1 % SNP): whole HBM-resident builds
  (pg_build_device) with per-stage HIP-event spans, counts against the
  oracle digest.
* c5shard (3.75 Gbp: the rank-0 shard at N = 8): the streamed exchange at
  world 1 (dist.exchange_stream, 2^30-base chunks) with per-phase seconds.

    python tools/c5_probe.py [whole] [stream] [reps=N]
"""
import json
import os
import sys
import tempfile
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def beat(t0, done):
    while not done.wait(20):
        print("c5_probe: %.0f s" % (time.time() - t0), flush=True)


def gen(name, d):
    from pangenome_amd import synth
    from scale_util import INPUTS, load_digest
    dg = load_digest(name)
    p = os.path.join(d, name + ".fa")
    t0 = time.time()
    n = synth.write_c5(p, pairs=INPUTS[name]["pairs"], workers=10)
    assert n == dg["fasta_bytes"], (n, dg["fasta_bytes"])
    print("%s: %d bytes generated in %.1f s" % (name, n, time.time() - t0), flush=True)
    return p, dg


def main():
    args = sys.argv[1:] or ["whole", "stream"]
    reps = 3
    for a in args:
        if a.startswith("reps="):
            reps = int(a[5:])
    import torch
    from pangenome_amd import kmer
    from pangenome_amd._lib import Context
    t00 = time.time()
    done = threading.Event()
    threading.Thread(target=beat, args=(t00, done), daemon=True).start()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    out = {}
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as d:
        if "whole" in args:
            p, dg = gen("c5m", d)
            mm = kmer.seq2bytes(p)
            dbuf = torch.from_numpy(np.array(mm)).to(dev)
            ctx = Context(27, 0)
            runs = []
            for i in range(reps + 1):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                st = ctx.build_device(dbuf.data_ptr(), dbuf.numel(), True, keepalive=dbuf)
                torch.cuda.synchronize()
                ms = 1e3 * (time.perf_counter() - t0)
                r = dict(wall_ms=round(ms, 3), parse=st.ms_parse, stage_a=st.ms_insert, split=st.ms_split,
                         range=st.ms_range, recs_a=st.n_records_a, work=st.n_work_items, cap=st.table_capacity,
                         n_dbg=st.n_dbg, n_rdbg=st.n_rdbg, flags=st.build_flags,
                         ok=(st.n_dbg, st.n_rdbg) == (dg["n_dbg"], dg["n_rdbg"]),
                         gbps=round(st.n_bases / ms / 1e6, 3))
                print("c5m whole %d: %s" % (i, json.dumps(r)), flush=True)
                runs.append(r)
            out["c5m_whole"] = runs
            ctx.close()
            del ctx, dbuf, mm
            torch.cuda.empty_cache()
            os.unlink(p)
        if "stream" in args:
            import torch.distributed as dist
            from pangenome_amd.dist import GpuShard, exchange_stream, stream_chunks
            from bench import _free_port
            p, dg = gen("c5shard", d)
            dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % _free_port(), rank=0,
                                    world_size=1, device_id=dev)
            sh = GpuShard(27, 0)
            mm = kmer.seq2bytes(p)
            t0 = time.time()
            meta = sh.load(mm)
            print("c5shard parsed in %.2f s" % (time.time() - t0), flush=True)
            R = int(meta["seq_len"].shape[0])
            runs = []
            forms = [a for a in args if a in ("routed", "local")] or ["routed"]
            for i, form in [(i, f) for f in forms for i in range(max(1, reps - 1))]:
                tm = {}
                chunks = stream_chunks(np.ones(R, np.uint8), meta["seq_len"], 1 << 30)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                lib = {}
                res = exchange_stream(sh, 1, 0, dev, chunks, R, True, tm=tm, routed=(form == "routed"),
                                      lib_stats=lib, keys=(i == 0))
                el = time.perf_counter() - t0
                tm.pop("start", None)
                r = {k: round(1e3 * v, 2) for k, v in tm.items()}
                r["form"] = form
                if lib:
                    r["lib"] = lib
                r.update(total_ms=round(1e3 * el, 2), n_dbg=int(res[0]), n_rdbg=int(res[1]), rounds=res[4],
                         ok=(int(res[0]), int(res[1])) == (dg["n_dbg"], dg["n_rdbg"]),
                         gbps=round(dg["n_bases"] / el / 1e9, 3))
                print("c5shard stream %d: %s" % (i, json.dumps(r)), flush=True)
                runs.append(r)
            out["c5shard_stream"] = runs
            dist.destroy_process_group()
    done.set()
    print("C5PROBE " + json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

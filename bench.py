#!/usr/bin/env python3
"""Gbp/s of the k-mer -> rdBG build at k=27 on MI355X (BASELINE.json metric).

One step = the window SURVEY.md §8(d) times, over this rank's synthetic
pangenome shard: FASTA bytes in a page-cache-warm np.memmap of the file
(kmer.seq2bytes, what the CLI passes; the reference's seq2bytes,
kmer_numba.py:117-119) -> H2D through the pinned staging ring -> K1 parse ->
K3 dBG build (both strands, the reference's default -c 2) -> [N>1: owner
all-to-all over RCCL and OR-merge] -> rdBG rule, ending with the rdBG key
count on the host (pg_build_host).  Weak scaling: every rank owns 100 x 5 Mbp
genomes (C3 per GPU; 8 GPUs = 800 genomes).

The same build from HBM-resident input (pg_build_device) is timed too
(`path.device_resident_gbps`); its per-kernel HIP-event spans give the
roofline of the dominant kernel.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c4]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK = 8.0e12         # MI355X HBM3E, B/s (MI355X_MICROARCH.md)
K = 27


def workload(config: str, rank: int, world: int):
    """[(genome spec, digest name or None), ...] batches of this rank, the
    digest of the global population (N>1), and the description.

    N=1, C3: two batches of the same population alternate (genomes 0-99 =
    c3a, 100-199 = c3b), so no step rebuilds the input the step before it
    built.  N>1: the population is genomes 0 .. 100N-1; rank r holds block r
    on even steps and block (r+1) mod N on odd ones, so every step builds the
    same global population (one oracle digest per N, tests/golden/scale/popN)
    from a different shard than the step before."""
    if config == "c2":
        return [("c2", "c2" if world == 1 else None)], None, "C2: synthetic E. coli K-12 stand-in, 4,641,652 bp, 1 record"
    if config in ("c3", "c4"):
        n = 100 if config == "c3" else 1000 // world
        if world == 1:
            if config == "c3":
                return ([(("pan", n, 0), "c3a"), (("pan", n, 100), "c3b")], None,
                        "C3: 100 x 5 Mbp variants (0.1% SNP, 0.01% indel), two alternating batches of the "
                        "same population (genomes 0-99, 100-199)")
            return [(("pan", n, 0), "c4")], None, "C4: 1000 x 5 Mbp variants (5 Gbp, 5.08 GB of FASTA) on one GPU"
        blocks = [rank, (rank + 1) % world]
        pop = ("pop%d" % world) if config == "c3" else "c4"
        return ([(("pan", n, b * n), None) for b in blocks], pop,
                "%s: %d x 5 Mbp variants per GPU and step (genomes 0..%d in total, each rank's block rotating "
                "between steps)" % (config.upper(), n, n * world - 1))
    if config == "small":
        return [(("pan_small", 10, rank * 10), None)], None, "small: 10 x 1 Mbp per GPU"
    raise SystemExit("unknown --config %s" % config)


def make_fasta(spec) -> bytes:
    from pangenome_amd import synth
    if spec == "c2":
        return synth.ecoli_like()
    kind, n, first = spec
    if kind == "pan_small":
        return synth.pangenome(n, 1_000_000, first_index=first)
    return synth.pangenome(n, 5_000_000, snp=1e-3, indel=1e-4, first_index=first)


def cpu_baseline(config: str, sample: bool = False):
    """The oracle's faithful single-core restatement (same oakht hash, probe
    sequence, growth and 3 probes per occurrence as kmer_numba.py) on the
    whole workload batch (C3 in full, ~2 min on one core), or
    on its first 12 genomes with --cpu-sample (~12 s).  A heartbeat goes to
    stderr every 30 s while it runs.  Peak RSS is the process's (it includes
    the torch/HIP runtime); table_bytes is the oracle's oakht at 11 B/slot."""
    import resource
    import threading
    from oracle import oracle
    from pangenome_amd import synth
    if config == "c2":
        fa, desc = synth.ecoli_like(), "whole C2 genome (4.64 Mbp)"
    else:
        g = 12 if sample else 100
        fa = synth.pangenome(g, 5_000_000, snp=1e-3, indel=1e-4)
        desc = ("all 100 C3 genomes (500 Mbp, batch c3a)" if not sample else
                "first %d of the C3 genomes (%.0f Mbp)" % (g, g * 5.0)) + ", dBG + rdBG, k=27, -c 2"
    done = threading.Event()

    def beat():
        t0 = time.time()
        while not done.wait(30):
            print("cpu_baseline: %.0f s" % (time.time() - t0), file=sys.stderr, flush=True)
    th = threading.Thread(target=beat, daemon=True)
    th.start()
    try:
        r = oracle.OracleRun(fa, K, 2)
    finally:
        done.set()
    t_dbg, t_rdbg = r.timings()
    rss = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024.0
    lib = oracle.lib()
    return {"value": r.n_bases() / (t_dbg + t_rdbg) / 1e9, "unit": "Gbp/s", "cores": 1, "kind": "port",
            "sample": desc, "t_dbg_s": round(t_dbg, 3), "t_rdbg_s": round(t_rdbg, 3),
            "n_dbg": int(lib.pgo_n_dbg(r.h)), "n_rdbg": int(lib.pgo_n_rdbg(r.h)),
            "table_bytes": int(lib.pgo_dbg_capacity(r.h)) * 11, "peak_rss_mb": round(rss, 1),
            "cpu": _cpu_model(), "nproc": os.cpu_count()}


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _digest(name):
    if not name:
        return None
    p = os.path.join(ROOT, "tests", "golden", "scale", name + ".json")
    return json.load(open(p)) if os.path.isfile(p) else None


def _sha_dbg(keys, masks):
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(keys, dtype="<u8").tobytes())
    h.update(np.ascontiguousarray(masks, dtype="<u2").tobytes())
    return h.hexdigest()


def _sha_rdbg(keys):
    return hashlib.sha256(np.ascontiguousarray(np.sort(keys), dtype="<u8").tobytes()).hexdigest()


def _gather_rdbg_sha(ctx, world, rank, device, rehearse):
    """SHA-256 of the sorted union of the owners' rdBG keys (all-gathered)."""
    import torch
    import torch.distributed as dist
    comm = torch.device("cpu") if rehearse else device
    keys = torch.from_numpy(ctx.rdbg().view(np.int64)).to(comm)
    n = torch.tensor([keys.shape[0]], dtype=torch.int64, device=comm)
    ns = [torch.empty_like(n) for _ in range(world)]
    dist.all_gather(ns, n)
    m = max(int(x.item()) for x in ns)
    pad = torch.zeros(max(m, 1), dtype=torch.int64, device=comm)
    pad[:keys.shape[0]] = keys
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad)
    if rank != 0:
        return None
    allk = np.concatenate([p[:int(c.item())].cpu().numpy() for p, c in zip(parts, ns)]).view(np.uint64)
    return _sha_rdbg(allk)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", action="store_true", help="CPU baseline on 12 of the 100 C3 genomes (~12 s)")
    ap.add_argument("--no-host-window", action="store_true",
                    help="profiler runs: time only the HBM-resident build (no chunked host-window launches "
                         "mixed into the per-kernel averages); `value` is then the device-resident rate")
    ap.add_argument("--tmpdir", default=None, help="where the FASTA files go (default: a fresh dir in $TMPDIR)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE=%d (launch N>1 with torch.distributed.run)" % (args.gpus, world))
    # PG_BENCH_REHEARSE=1 (development only): every rank on cuda:0 with gloo,
    # to exercise the N>1 orchestration on a one-GPU box; never a bench number
    rehearse = os.environ.get("PG_BENCH_REHEARSE") == "1"
    dev_index = 0 if rehearse else local
    torch.cuda.set_device(dev_index)
    device = torch.device("cuda", dev_index)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=device)

    from pangenome_amd import kmer
    from pangenome_amd._lib import Context
    from pangenome_amd.dist import exchange_and_reduce

    batches, pop_name, desc = workload(args.config, rank, world)
    tmp = tempfile.mkdtemp(prefix="pgbench_r%d_" % rank, dir=args.tmpdir)
    try:
        run(args, torch, dist, kmer, Context, exchange_and_reduce, batches, pop_name, desc, world, rank,
            dev_index, device, rehearse, tmp)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def run(args, torch, dist, kmer, Context, exchange_and_reduce, batches, pop_name, desc, world, rank, dev_index,
        device, rehearse, tmp):
    # ---- inputs: FASTA files, read once (page cache warm), memory-mapped
    # read-only exactly as the CLI maps them; and HBM copies for the
    # device-resident loop
    paths, mms, d_in, digests = [], [], [], []
    for i, (spec, dname) in enumerate(batches):
        p = os.path.join(tmp, "batch%d.fa" % i)
        fasta = make_fasta(spec)
        with open(p, "wb") as f:
            f.write(fasta)
        d_in.append(torch.frombuffer(bytearray(fasta), dtype=torch.uint8).to(device))
        del fasta
        with open(p, "rb") as f:                            # page-cache warm
            while f.read(1 << 26):
                pass
        paths.append(p)
        mms.append(kmer.seq2bytes(p))
        digests.append(_digest(dname))
    pop = _digest(pop_name)
    nbytes = [int(m.shape[0]) for m in mms]
    torch.cuda.synchronize()

    def exchange(ctx, st):
        return exchange_and_reduce(ctx, world, rank, device, bool(st.sentinel))

    def step_host(ctx, i):
        """mmap -> H2D (pinned staging ring) -> parse -> build -> rdBG count."""
        st = ctx.build_host(mms[i % len(mms)], True)
        if world == 1:
            return st, st, st.n_dbg, st.n_rdbg, 0
        n_dbg, n_rdbg, _, sent = exchange(ctx, st)
        return st, ctx.stats(), n_dbg, n_rdbg, sent

    def step_device(ctx, i):
        """the same build from the HBM-resident copy (pg_build_device)."""
        d = d_in[i % len(d_in)]
        st = ctx.build_device(d.data_ptr(), d.numel(), True, keepalive=d)
        if world == 1:
            return st, st, st.n_dbg, st.n_rdbg, 0
        n_dbg, n_rdbg, _, sent = exchange(ctx, st)
        return st, ctx.stats(), n_dbg, n_rdbg, sent

    def timed(ctx, step):
        for i in range(args.warmup):
            step(ctx, i)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        recs = []
        for i in range(args.steps):
            r = step(ctx, args.warmup + i)
            recs.append(((args.warmup + i) % len(mms), r))
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        return time.perf_counter() - t0, recs

    # cold first build: a fresh context (no working memory, no learned sizes,
    # no staging threads) from the mmap
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    cold = Context(K, dev_index)
    cst = step_host(cold, 0)
    cold_ms = 1e3 * (time.perf_counter() - t0)
    cold.close()
    del cold

    ctx = Context(K, dev_index)
    host_window = not args.no_host_window
    if host_window:
        el_host, recs_host = timed(ctx, step_host)
        # SHA-256 of the last host-window build (N=1: the whole dBG and rdBG;
        # N>1: the union of the owners' rdBG)
        last_host_batch = recs_host[-1][0]
        if world == 1:
            keys, masks = ctx.dbg()
            host_sha = (_sha_dbg(keys, masks), _sha_rdbg(ctx.rdbg()))
            del keys, masks
        else:
            host_sha = (None, _gather_rdbg_sha(ctx, world, rank, device, rehearse))
    el_dev, recs_dev = timed(ctx, step_device)
    if world > 1 and not host_window:
        host_sha = (None, _gather_rdbg_sha(ctx, world, rank, device, rehearse))

    el, recs = (el_host, recs_host) if host_window else (el_dev, recs_dev)
    if world > 1:
        comm = torch.device("cpu") if rehearse else device
        t = torch.tensor([el, el_dev], dtype=torch.float64, device=comm)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el, el_dev = t.tolist()
        tot = torch.tensor([sum(r[0].n_bases for _, r in recs), sum(r[0].n_bases for _, r in recs_dev),
                            sum(r[0].n_windows // 2 for _, r in recs[-1:]), nbytes[0]], dtype=torch.int64,
                           device=comm)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        total_bases, total_bases_dev, wfw_all, bytes_all = [int(x) for x in tot.tolist()]
    else:
        total_bases = sum(r[0].n_bases for _, r in recs)
        total_bases_dev = sum(r[0].n_bases for _, r in recs_dev)
        wfw_all, bytes_all = recs[-1][1][0].n_windows // 2, nbytes[recs[-1][0]]

    # ---- parity, after the timed regions: every timed step's counts (both
    # loops) and the cold build's against the oracle digest of its batch (N>1:
    # of the global population), SHA-256 of one host-window build
    parity = None
    if world == 1 and all(digests):
        def cnt_ok(rr):
            return all((r[2], r[3]) == (digests[b]["n_dbg"], digests[b]["n_rdbg"]) for b, r in rr)
        ok_host = cnt_ok(recs_host) if host_window else True
        ok_dev = cnt_ok(recs_dev)
        ok_cold = (cst[2], cst[3]) == (digests[0]["n_dbg"], digests[0]["n_rdbg"])
        if host_window:
            dg = digests[last_host_batch]
            sha_ok = host_sha == (dg["dbg_sha256"], dg["rdbg_sha256"])
        else:
            ctx.build_device(d_in[0].data_ptr(), d_in[0].numel(), True, keepalive=d_in[0])
            keys, masks = ctx.dbg()
            sha_ok = (_sha_dbg(keys, masks), _sha_rdbg(ctx.rdbg())) == (digests[0]["dbg_sha256"],
                                                                        digests[0]["rdbg_sha256"])
        parity = {"ok": bool(ok_host and ok_dev and ok_cold and sha_ok),
                  "checked": "n_dbg/n_rdbg of every timed step (host window and HBM-resident loops) and of the "
                             "cold build vs the oracle digests (tests/golden/scale); SHA-256 of the sorted dBG and "
                             "rdBG of the last host-window build",
                  "host_steps_ok": bool(ok_host), "device_steps_ok": bool(ok_dev), "cold_ok": bool(ok_cold),
                  "sha256_ok": bool(sha_ok)}
    elif world > 1 and pop is not None:
        def cnt_ok(rr):
            return all((r[2], r[3]) == (pop["n_dbg"], pop["n_rdbg"]) for _, r in rr)
        ok = cnt_ok(recs_dev) and (cnt_ok(recs_host) if host_window else True) and \
            (cst[2], cst[3]) == (pop["n_dbg"], pop["n_rdbg"])
        sha_ok = host_sha[1] == pop["rdbg_sha256"] if rank == 0 else None
        parity = {"ok": bool(ok and sha_ok) if rank == 0 else bool(ok),
                  "checked": "global n_dbg/n_rdbg of every timed step and of the cold build vs the oracle digest "
                             "of the whole population (tests/golden/scale/%s.json); SHA-256 of the all-gathered "
                             "owner rdBG keys of the last %s build" % (pop_name, "host-window" if host_window
                                                                     else "HBM-resident"),
                  "counts_ok": bool(ok), "rdbg_sha256_ok": sha_ok}

    # ---- the bounds of the window: a bare staged upload of the mmap (the
    # pinned ring alone, pg_set_fasta) and a bare pinned H2D; and the same
    # build from a pinned host buffer (pg_build_host with plain DMA)
    extra = {}
    if host_window:
        jb = 0
        m = mms[jb]
        def best(fn, reps=3):
            ts = []
            for _ in range(reps):
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t1)
            return min(ts)
        t_stage = best(lambda: ctx.set_fasta(m))
        pin = torch.empty(nbytes[jb], dtype=torch.uint8, pin_memory=True)
        pin.numpy()[:] = m
        dst = torch.empty_like(d_in[jb])
        t_pin = best(lambda: dst.copy_(pin, non_blocking=True))
        t_pin_build = best(lambda: ctx.build_host_ptr(pin.data_ptr(), pin.numel(), True))
        pin_counts = (ctx.stats().n_dbg, ctx.stats().n_rdbg)
        del pin, dst
        ms_step = 1e3 * el / args.steps
        extra = {"h2d_staged_mmap_gbs": round(nbytes[jb] / t_stage / 1e9, 2),
                 "h2d_pinned_gbs": round(nbytes[jb] / t_pin / 1e9, 2),
                 "window_frac_of_staged_h2d": round(t_stage * 1e3 / ms_step, 4),
                 "window_frac_of_pinned_h2d": round(t_pin * 1e3 / ms_step, 4),
                 "pinned_host_ms": round(1e3 * t_pin_build, 3),
                 "pinned_host_gbps": round(recs_host[0][1][0].n_bases / t_pin_build / 1e9, 3)}
        if parity is not None and world == 1:
            ok_pin = pin_counts == (digests[jb]["n_dbg"], digests[jb]["n_rdbg"])
            parity["pinned_ok"] = bool(ok_pin)
            parity["ok"] = bool(parity["ok"] and ok_pin)
        if world == 1:
            # the CLI's own dBG pass (kmer.seq2rdbg: a fresh context, build
            # from the mmap), as `# build the dBG` times it
            t1 = time.perf_counter()
            g = kmer.seq2rdbg(paths[jb], K, 5, 2 ** 63, brkpt="", chunk=2 ** 33, rc=True, device=dev_index)
            extra["cli_seq2rdbg_ms"] = round(1e3 * (time.perf_counter() - t1), 3)
            if parity is not None:
                ok_cli = (g.stats.n_dbg, g.stats.n_rdbg) == (digests[jb]["n_dbg"], digests[jb]["n_rdbg"])
                parity["cli_ok"] = bool(ok_cli)
                parity["ok"] = bool(parity["ok"] and ok_cli)
            g.ctx.close()
            del g

    last = recs[-1][1]
    st_b, st_c, n_dbg, n_rdbg, sent = last
    ms_step = 1e3 * el / args.steps
    value = total_bases / el / 1e9

    # ---- roofline, from the HBM-resident loop.  Per kernel, ALGORITHMIC
    # bytes = what the kernel must read and write by its own definition
    # (DESIGN.md §4), over its HIP-event time on the context's stream,
    # averaged over the timed steps:
    #   K1 parse    F FASTA bytes read + B class codes written
    #   K3 stage A  B class codes read + 12 B per emitted record (8 B h + 4 B mask word)
    #   K3 stage B  24 B per record (read + write; one split pass at C3)
    #   K3 stage C  12 B per record read + 16 B per table bucket + 8 B per rdBG key written
    # The dominant kernel (the longest span) is `roofline`; `traffic` is its
    # PMC-measured HBM bytes per build (profiles/traffic_<config>.json, from
    # a separate rocprofv3 run).  SURVEY.md §8(d)'s path model, F + 20 W +
    # 10 D + 8 R, is `path.alg_bytes_s8d`: it charges every window 20 B that
    # the coverage pass never moves, so it is an "equivalent" figure.
    dst_b = recs_dev[-1][1][0]
    dst_c = recs_dev[-1][1][1]
    nrec_a = dst_b.n_records_a
    mean = lambda f: float(np.mean([f(r) for _, r in recs_dev]))   # noqa: E731
    spans = {
        "k1_parse": (mean(lambda r: r[0].ms_parse), nbytes[recs_dev[-1][0]] + dst_b.n_bases,
                     "F FASTA bytes read + B class codes written"),
        "k3a_cover_emit": (mean(lambda r: r[0].ms_insert), dst_b.n_bases + 12 * nrec_a,
                           "B class codes read + 12 B per emitted record"),
        "k3b_split": (mean(lambda r: r[1].ms_split), 24 * dst_c.n_records_a, "24 B per record (read + write)"),
        "k3c_range": (mean(lambda r: r[1].ms_range), 12 * dst_c.n_records_a + 16 * dst_c.table_capacity +
                      8 * dst_c.n_rdbg, "12 B per record + 16 B per bucket + 8 B per rdBG key"),
    }
    pmc = {}
    tp = os.path.join(ROOT, "profiles", "traffic_%s.json" % args.config)
    if os.path.isfile(tp):
        pmc = json.load(open(tp)).get("hbm_bytes_per_build", {})
    kernels = {}
    for name, (ms, ab, model) in spans.items():
        kernels[name] = {"ms": round(ms, 4), "alg_bytes": int(ab), "alg_model": model,
                         "frac": round(ab / (ms * 1e-3) / HBM_PEAK, 4) if ms > 0 else None,
                         "pmc_bytes": pmc.get(name), "pmc_frac": round(pmc[name] / (ms * 1e-3) / HBM_PEAK, 4)
                         if pmc.get(name) and ms > 0 else None}
    dom = max(kernels, key=lambda n: kernels[n]["ms"])
    kd = kernels[dom]
    # whole-path algorithmic fraction, SURVEY.md §8(d): F + 20 W + 10 D + 8 R
    path_bytes = bytes_all + 20 * wfw_all + 10 * n_dbg + 8 * n_rdbg

    out = {
        "metric": "Gbp/s k-mer->rdBG build at k=27; bit-exact region table vs numba ref",
        "value": round(value, 4),
        "unit": "Gbp/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (splitmix64 pangenome generator, pangenome_amd/synth.py)",
        "config": {"workload": desc, "k": K, "strands": "-c 2 (dBG both strands)",
                   "bases_per_gpu": st_b.n_bases, "fasta_bytes_per_gpu": nbytes[0],
                   "input": ("page-cache-warm mmap of the FASTA file (kmer.seq2bytes); H2D, parse, build and the "
                             "rdBG count on the host inside the timed region (SURVEY 8(d) window)")
                   if host_window else "FASTA resident in HBM when the timed region starts (--no-host-window)",
                   "parallelism": "record-sharded, owner all-to-all" if world > 1 else "single GPU"},
        "roofline": {"kernel": dom, "bound": "hbm", "achieved": round(kd["alg_bytes"] / (kd["ms"] * 1e-3) / 1e9, 2),
                     "peak": HBM_PEAK / 1e9, "unit": "GB/s", "frac": kd["frac"],
                     "traffic": kd["pmc_bytes"], "traffic_frac": kd["pmc_frac"],
                     "traffic_source": "PMC FETCH_SIZE x2 + WRITE_SIZE per build, profiles/traffic_%s.json" % args.config,
                     "alg_bytes_per_launch": kd["alg_bytes"], "alg_model": kd["alg_model"],
                     "avg_launch_ms": kd["ms"], "measured_in": "the HBM-resident loop (pg_build_device)"},
        "kernels": kernels,
        "path": {"device_resident_gbps": round(total_bases_dev / el_dev / 1e9, 4),
                 "device_resident_ms": round(1e3 * el_dev / args.steps, 3),
                 "alg_bytes_s8d": path_bytes, "frac_of_hbm_s8d_device_resident":
                     round(path_bytes / (el_dev / args.steps) / (world * HBM_PEAK), 5),
                 "n_records_a": nrec_a, "n_dbg": n_dbg, "n_rdbg": n_rdbg,
                 "table_slots": dst_b.table_capacity, "exchange_bytes_sent_rank0": sent,
                 "cold_first_build_ms": round(cold_ms, 3),
                 "cold_first_build_gbps": round(cst[0].n_bases / cold_ms / 1e6, 3)},
    }
    out["path"].update(extra)
    if parity is not None:
        out["parity"] = parity
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.config, args.cpu_sample)
    if rehearse:
        out["data"] += "; REHEARSAL: all ranks on cuda:0 over gloo, not a measurement"
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if parity is not None and not parity["ok"]:
        raise SystemExit("parity check FAILED: %s" % json.dumps(parity))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Gbp/s of the k-mer -> rdBG build at k=27 on MI355X (BASELINE.json metric).

One step = one pass of the hot path over this rank's synthetic pangenome
shard, FASTA already resident in HBM: K1 parse -> K3 dBG insert (both
strands, the reference's default -c 2) -> [N>1: owner all-to-all over RCCL
and OR-merge] -> K5 degree scan + rdBG compaction, ending with the rdBG key
count on the host.  Weak scaling: every rank owns the same number of genomes
(C3 = 100 x 5 Mbp per GPU; 8 GPUs = 800 genomes, C4-scale).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c4]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK = 8.0e12         # MI355X HBM3E, B/s (MI355X_MICROARCH.md)
K = 27


def workload(config: str, rank: int, world: int):
    """[(fasta, digest name or None), ...] batches of this rank, and the description.
    C3 alternates two distinct batches of the same population (genomes
    r*100.. and (world+r)*100..), so that no step rebuilds the input the step
    before it built."""
    from pangenome_amd import synth
    if config == "c2":
        return [(synth.ecoli_like(), "c2")], "C2: synthetic E. coli K-12 stand-in, 4,641,652 bp, 1 record"
    if config == "c3":
        n = 100
        b = [(synth.pangenome(n, 5_000_000, snp=1e-3, indel=1e-4, first_index=(i * world + rank) * n),
              ("c3a", "c3b")[i] if world == 1 else None) for i in range(2)]
        return b, ("C3: 100 x 5 Mbp variants (0.1%% SNP, 0.01%% indel) per GPU and step, two alternating "
                   "batches of the same population; %d genomes per step in total" % (n * world))
    if config == "c4":
        n = 1000 // world
        return ([(synth.pangenome(n, 5_000_000, snp=1e-3, indel=1e-4, first_index=rank * n), None)],
                "C4: 1000 x 5 Mbp variants sharded %d per GPU" % n)
    if config == "small":
        return [(synth.pangenome(10, 1_000_000, first_index=rank * 10), None)], "small: 10 x 1 Mbp per GPU"
    raise SystemExit("unknown --config %s" % config)


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


def _full_check(ctx, dg):
    """SHA-256 of the sorted dBG and rdBG against the oracle's digest."""
    import hashlib
    keys, masks = ctx.dbg()
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(keys, dtype="<u8").tobytes())
    h.update(np.ascontiguousarray(masks, dtype="<u2").tobytes())
    ok_dbg = h.hexdigest() == dg["dbg_sha256"]
    ok_rdbg = hashlib.sha256(np.ascontiguousarray(ctx.rdbg(), dtype="<u8").tobytes()).hexdigest() == dg["rdbg_sha256"]
    return ok_dbg and ok_rdbg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", action="store_true", help="CPU baseline on 12 of the 100 C3 genomes (~12 s)")
    ap.add_argument("--no-host-window", action="store_true",
                    help="skip the host-resident window (profiler runs: its chunked K1 dispatches)")
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

    from pangenome_amd._lib import Context
    from pangenome_amd.dist import exchange_and_reduce

    batches, desc = workload(args.config, rank, world)
    d_in, digests, host0 = [], [], None
    for i, (fasta, dname) in enumerate(batches):
        d_in.append(torch.frombuffer(bytearray(fasta), dtype=torch.uint8).to(device))
        digests.append(_digest(dname))
        if i == 0:
            host0 = torch.empty(len(fasta), dtype=torch.uint8, pin_memory=True)
            host0.numpy()[:] = np.frombuffer(fasta, np.uint8)
    nbytes = [d.numel() for d in d_in]
    del batches, fasta
    torch.cuda.synchronize()

    def step(ctx, i):
        d = d_in[i % len(d_in)]
        if world == 1:                      # parse + seq2rdbg + dbg2rdbg in one call (pg_build_device)
            st = ctx.build_device(d.data_ptr(), d.numel(), True, keepalive=d)
            return st, st, st.n_dbg, st.n_rdbg, 0
        ctx.set_fasta_device(d.data_ptr(), d.numel(), keepalive=d)
        ctx.parse()
        st_b = ctx.build_dbg(None, 0, True)
        n_dbg, n_rdbg, _, sent = exchange_and_reduce(ctx, world, rank, device, bool(st_b.sentinel))
        return st_b, ctx.stats(), n_dbg, n_rdbg, sent

    # cold first build: a fresh context (no working memory, no learned sizes, no cached tiles)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    cold = Context(K, dev_index)
    cst = step(cold, 0)
    cold_ms = 1e3 * (time.perf_counter() - t0)
    cold.close()
    del cold

    ctx = Context(K, dev_index)
    for i in range(args.warmup):
        step(ctx, i)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ins_ms, split_ms, range_ms, parse_ms, counts = [], [], [], [], []
    last = None
    for i in range(args.steps):
        last = step(ctx, args.warmup + i)
        ins_ms.append(last[0].ms_insert)
        split_ms.append(last[1].ms_split)
        range_ms.append(last[1].ms_range)
        parse_ms.append(last[0].ms_parse)
        counts.append(((args.warmup + i) % len(d_in), last[2], last[3]))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        comm = torch.device("cpu") if rehearse else device
        t = torch.tensor([elapsed], dtype=torch.float64, device=comm)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        tot = torch.tensor([last[0].n_bases, last[0].n_windows // 2, nbytes[0]], dtype=torch.int64, device=comm)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        bases_all, wfw_all, bytes_all = [int(x) for x in tot.tolist()]
        total_bases = bases_all * args.steps
    else:
        bases_all, wfw_all, bytes_all = last[0].n_bases, last[0].n_windows // 2, nbytes[-1]
        # bases of every timed step (the batches differ by a few indels)
        per_batch = {}
        for j in range(len(d_in)):
            ctx.set_fasta_device(d_in[j].data_ptr(), d_in[j].numel(), keepalive=d_in[j])
            per_batch[j] = ctx.parse()[1]
        total_bases = sum(per_batch[b] for b, _, _ in counts)

    # ---- parity after the timed region: every timed step's counts against the
    # oracle digest of its batch, and the full dBG / rdBG digests of one build
    parity = None
    if world == 1 and all(digests):
        ok = all((n_dbg, n_rdbg) == (digests[b]["n_dbg"], digests[b]["n_rdbg"]) for b, n_dbg, n_rdbg in counts)
        jb = (args.warmup + args.steps - 1) % len(d_in)
        d = d_in[jb]
        ctx.set_fasta_device(d.data_ptr(), d.numel(), keepalive=d)
        ctx.parse()
        ctx.build(None, 0, True)
        full = _full_check(ctx, digests[jb])
        ok_cold = (cst[2], cst[3]) == (digests[0]["n_dbg"], digests[0]["n_rdbg"])
        parity = {"ok": bool(ok and full and ok_cold),
                  "checked": "n_dbg/n_rdbg of every timed step and of the cold build vs the oracle digests "
                             "(tests/golden/scale); SHA-256 of one more build's sorted dBG and rdBG",
                  "steps_ok": bool(ok), "sha256_ok": bool(full), "cold_ok": bool(ok_cold)}

    # ---- host-resident input (BASELINE.md §3 window): pinned host FASTA ->
    # H2D -> parse -> build -> rdBG count on the host; and the bare H2D rate
    host_ms, h2d_gbs = None, None
    if world == 1 and not args.no_host_window:
        # pg_build_host: chunked H2D, K1 per chunk, stage A over each chunk's
        # completed records under the copy, then stages B/C
        ts, host_counts = [], []
        for _ in range(3):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            sth = ctx.build_host_ptr(host0.data_ptr(), host0.numel(), True)
            ts.append(time.perf_counter() - t1)
            host_counts.append((sth.n_dbg, sth.n_rdbg))
        host_ms = 1e3 * min(ts)
        if parity is not None and digests[0]:
            ok_host = all(hc == (digests[0]["n_dbg"], digests[0]["n_rdbg"]) for hc in host_counts)
            parity["host_window_ok"] = bool(ok_host)
            parity["ok"] = bool(parity["ok"] and ok_host)
        tmp = torch.empty_like(d_in[0])
        hs = []
        for _ in range(3):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            tmp.copy_(host0, non_blocking=True)
            torch.cuda.synchronize()
            hs.append(time.perf_counter() - t1)
        h2d_gbs = host0.numel() / min(hs) / 1e9
        del tmp

    st_b, st_r, n_dbg, n_rdbg, sent = last
    ms_step = 1e3 * elapsed / args.steps
    value = total_bases / elapsed / 1e9

    # ---- roofline.  Per kernel, ALGORITHMIC bytes = what the kernel must read
    # and write by its own definition, over its HIP-event time
    # on the context's stream, averaged over the timed steps:
    #   K1 parse    F FASTA bytes read + B class codes written
    #   K3 stage A  B class codes read + 12 B per emitted record (8 B h + 4 B mask word)
    #   K3 stage B  24 B per record (read + write; one split pass at C3)
    #   K3 stage C  12 B per record read + 16 B per table bucket + 8 B per rdBG key written
    # The dominant kernel (the longest span) is `roofline`; `traffic` is its
    # PMC-measured HBM bytes per build (profiles/traffic_<config>.json, from
    # a separate rocprofv3 run).  SURVEY.md §8(d)'s path model, F + 20 W +
    # 10 D + 8 R, is `path.alg_bytes_s8d`: it charges every window 20 B that
    # the coverage pass never moves, so it is an "equivalent" figure.
    st_b, st_c = last[0], last[1]             # stage A stats; stage B/C (N>1: the owner merge's)
    nrec_a = st_b.n_records_a
    spans = {
        "k1_parse": (float(np.mean(parse_ms)), nbytes[-1] + st_b.n_bases,
                     "F FASTA bytes read + B class codes written"),
        "k3a_cover_emit": (float(np.mean(ins_ms)), st_b.n_bases + 12 * nrec_a,
                           "B class codes read + 12 B per emitted record"),
        "k3b_split": (float(np.mean(split_ms)), 24 * st_c.n_records_a, "24 B per record (read + write)"),
        "k3c_range": (float(np.mean(range_ms)), 12 * st_c.n_records_a + 16 * st_c.table_capacity + 8 * st_c.n_rdbg,
                      "12 B per record + 16 B per bucket + 8 B per rdBG key"),
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
                   "input": "FASTA resident in HBM when the timed region starts",
                   "parallelism": "record-sharded, owner all-to-all" if world > 1 else "single GPU"},
        "roofline": {"kernel": dom, "bound": "hbm", "achieved": round(kd["alg_bytes"] / (kd["ms"] * 1e-3) / 1e9, 2),
                     "peak": HBM_PEAK / 1e9, "unit": "GB/s", "frac": kd["frac"],
                     "traffic": kd["pmc_bytes"], "traffic_frac": kd["pmc_frac"],
                     "traffic_source": "PMC FETCH_SIZE x2 + WRITE_SIZE per build, profiles/traffic_%s.json" % args.config,
                     "alg_bytes_per_launch": kd["alg_bytes"], "alg_model": kd["alg_model"],
                     "avg_launch_ms": kd["ms"]},
        "kernels": kernels,
        "path": {"alg_bytes_s8d": path_bytes, "frac_of_hbm_s8d": round(path_bytes / (elapsed / args.steps) /
                                                                         (world * HBM_PEAK), 5),
                 "n_records_a": nrec_a, "n_dbg": n_dbg, "n_rdbg": n_rdbg,
                 "table_slots": st_b.table_capacity, "exchange_bytes_sent_rank0": sent,
                 "cold_first_build_ms": round(cold_ms, 3),
                 "cold_first_build_gbps": round(cst[0].n_bases / cold_ms / 1e6, 3)},
    }
    if host_ms is not None:
        out["path"]["host_to_rdbg_ms"] = round(host_ms, 3)
        out["path"]["host_to_rdbg_gbps"] = round(per_batch[0] / host_ms / 1e6, 3)
        out["path"]["h2d_pinned_gbs"] = round(h2d_gbs, 2)
        # the PCIe bound of that window: the FASTA's bare pinned H2D time
        out["path"]["host_to_rdbg_frac_of_pcie_bound"] = round(nbytes[0] / (h2d_gbs * 1e9) / (host_ms * 1e-3), 4)
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

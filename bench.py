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


def cpu_baseline(config: str, full: bool = False):
    """The oracle's faithful single-core restatement (same oakht hash, probe
    sequence, growth and 3 probes per occurrence as kmer_numba.py) on a bounded
    prefix of the same workload (~10-30 s of CPU work), or the whole batch
    with --cpu-full (C3: a few minutes).  Peak RSS is the process's."""
    import resource
    from oracle import oracle
    from pangenome_amd import synth
    if config == "c2":
        fa, sample = synth.ecoli_like(), "whole C2 genome (4.64 Mbp)"
    else:
        g = 100 if full else 12
        fa = synth.pangenome(g, 5_000_000, snp=1e-3, indel=1e-4)
        sample = ("all 100 C3 genomes (500 Mbp)" if full else "first %d of the C3 genomes (%.0f Mbp)" % (g, g * 5.0)) \
            + ", dBG + rdBG, k=27, -c 2"
    r = oracle.OracleRun(fa, K, 2)
    t_dbg, t_rdbg = r.timings()
    rss = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024.0
    return {"value": r.n_bases() / (t_dbg + t_rdbg) / 1e9, "unit": "Gbp/s", "cores": 1, "kind": "port",
            "sample": sample, "t_dbg_s": round(t_dbg, 3), "t_rdbg_s": round(t_rdbg, 3),
            "n_dbg": int(lib_n(r)), "peak_rss_mb": round(rss, 1),
            "cpu": _cpu_model(), "nproc": os.cpu_count()}


def lib_n(r):
    from oracle import oracle
    return oracle.lib().pgo_n_dbg(r.h)


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
    ap.add_argument("--cpu-full", action="store_true", help="CPU baseline on the whole batch (minutes)")
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
        ctx.set_fasta_device(d.data_ptr(), d.numel(), keepalive=d)
        ctx.parse()
        if world == 1:                      # seq2rdbg + dbg2rdbg in one call (pg_build)
            st = ctx.build(None, 0, True)
            return st, st, st.n_dbg, st.n_rdbg, 0
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
    ins_ms, scan_ms, parse_ms, counts = [], [], [], []
    last = None
    for i in range(args.steps):
        last = step(ctx, args.warmup + i)
        ins_ms.append(last[0].ms_insert)
        scan_ms.append(last[1].ms_scan)
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
    if world == 1:
        ts = []
        for _ in range(3):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            ctx.set_fasta_host_ptr(host0.data_ptr(), host0.numel())
            ctx.parse()
            ctx.build(None, 0, True)
            ts.append(time.perf_counter() - t1)
        host_ms = 1e3 * min(ts)
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

    # roofline of the dominant kernel group, K3 (this rank): the coverage and
    # work passes of all chunks, bracketed by one HIP-event pair on the
    # context's stream (the side stream joins it before the stop event);
    # algorithmic bytes = 1 B class code per base + 20 B per forward window
    # (8 B key + 2 B mask on each strand); averaged over the
    # timed steps
    ins_avg = float(np.mean(ins_ms))
    ins_bytes = st_b.n_bases + 20 * (st_b.n_windows // 2)
    achieved = ins_bytes / (ins_avg * 1e-3)
    traffic = None
    tp = os.path.join(ROOT, "profiles", "traffic_%s.json" % args.config)
    if os.path.isfile(tp):
        traffic = json.load(open(tp)).get("k_insert_hbm_bytes_per_launch")
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
        "roofline": {"kernel": "K3 = k_cover + k_insert_work in 4 chunks on 2 streams (one HIP-event span)", "bound": "hbm",
                     "achieved": round(achieved / 1e9, 2),
                     "peak": HBM_PEAK / 1e9, "unit": "GB/s", "frac": round(achieved / HBM_PEAK, 4),
                     "traffic": traffic, "traffic_source": "profile-derived (profiles/traffic_%s.json)" % args.config,
                     "alg_bytes_per_launch": ins_bytes,
                     "avg_launch_ms": round(ins_avg, 4)},
        "path": {"alg_bytes": path_bytes, "frac_of_hbm": round(path_bytes / (elapsed / args.steps) /
                                                             (world * HBM_PEAK), 5),
                 "ms_parse": round(float(np.mean(parse_ms)), 3), "ms_insert": round(ins_avg, 3),
                 "ms_scan": round(float(np.mean(scan_ms)), 3), "n_dbg": n_dbg, "n_rdbg": n_rdbg,
                 "table_slots": st_b.table_capacity, "exchange_bytes_sent_rank0": sent,
                 "cold_first_build_ms": round(cold_ms, 3),
                 "cold_first_build_gbps": round(cst[0].n_bases / cold_ms / 1e6, 3)},
    }
    if host_ms is not None:
        out["path"]["host_to_rdbg_ms"] = round(host_ms, 3)
        out["path"]["host_to_rdbg_gbps"] = round(per_batch[0] / host_ms / 1e6, 3)
        out["path"]["h2d_pinned_gbs"] = round(h2d_gbs, 2)
    if parity is not None:
        out["parity"] = parity
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.config, args.cpu_full)
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

"""Multi-GPU k-mer -> dBG -> rdBG -> region table: one process per GPU.

SURVEY.md §8(e).  The reference runs seq2rdbg / dbg2rdbg / seq2graph
(kmer_numba.py:1234-1268, :1313-1321, :1853-1951) in one process; here the
input FASTA is sharded by bases across ranks at record boundaries, and the
per-base work of every pass runs on each rank's own GPU over its own records:

1. shard     every rank memory-maps the file and takes the byte range
             [bounds[r], bounds[r+1]) (split just before a header line, so
             each shard parses exactly as those records do in the whole file);
             the record tables are all-gathered, and the pass plans (-n
             limits, 2**33-base checkpoints, -r/-R resume) are computed over
             the global record list exactly as host.plan_* does on one GPU.
2. dBG       each rank builds the OR-table of its records (K1 + K3).
3. dump      `<in>_db.npz` needs the occurrence counts of the whole input:
             every rank counts its own records' occurrences per oriented key
             (saturating at 255, so summing saturated counts and saturating
             again is exact), rank 0 gathers them and places the union in the
             reference's oakht slot layout (pg_dbg_load + pg_dbg_dump).
4. rdBG      owner exchange: the pass's stage A records are held for their
             owners (the top bits of the table hash) and moved with one
             all-to-all (RCCL over xGMI); owners build their partition once
             from them, rdBG rule included (exchange_routed, the same step
             the N>1 bench times).  After -d / -r, whose staged npz slots no
             stage A rebuilds, and at a world that is not a power of two,
             the local table's entries are exchanged instead
             (exchange_and_reduce).
             The owners' rdBG keys are all-gathered (C3: 1.9 M keys, 15 MB),
             and every rank loads them as its walk membership table (the
             `-D` path, :2093).
5. edges     every rank walks its records (rdbg_edge_weight :1446-1518);
             rank 0 gathers the edge lists in rank order — records are
             contiguous per rank, so first-occurrence order across ranks is
             rank order — and reduces them by edge (walk counts add, the first
             occurrence wins), then applies the checkpoint reversals
             (host.edge_order / host.merge_edges for -R).
6. labels    rank 0 writes `.xyz`, runs `mcl` (or reuses `.mcl`) and builds
             the label table (:1893-1944); it is broadcast to every rank.
7. rows      every rank computes and formats its records' region rows
             (seqs2path_jit_ :1830-1849); rank 0 gathers the text in rank
             (= record) order and prints it.

Collectives: one all-to-all (the only data-path exchange), all-gathers of the
record tables and of the rdBG keys, point-to-point gathers to rank 0 of the
dump counts, edges and row text, one broadcast of the label table.  RCCL has
no bitwise-OR reduction and slot layouts differ per GPU, so an all-reduce of
"the count table" would not be exact — the owner all-to-all is.

The orchestration talks to a per-rank *shard backend* (GpuShard here; the CPU
tests use an oracle-backed stand-in with the same methods):
  load(data) -> records dict (seq_len, hdr_start, hdr_len, ptr), shard-relative
  stage(keys, masks, counts)        stage npz slots into the next build (-r/-d/-D)
  build(flags, extra, rc0) -> bool  the local dBG; returns the n<k sentinel flag
  counts() -> (keys, masks, counts) oriented entries of the local build with
                                    their occurrence counts
  partition / merge / build_rdbg    the exchange (exchange_and_reduce)
  owner_rdbg() -> keys              the owner partition's rdBG keys
  members(keys, n_records, rc0)     the global rdBG as walk membership
  edges(flags, rc1) -> (tuples, counts, walk)   first-occurrence order
  rows_text(labels, flags, rc1, names) -> bytes
  dump_global(keys, masks, counts) -> (capacity, size, keys, values, counts)
"""
from __future__ import annotations

import os
import sys
from time import perf_counter, time

import numpy as np

from . import host

SENTINEL = 2 ** 64 - 1
# A shard whose planned dBG pass holds more forward bases than this streams
# its exchange in chunks of this size (exchange_stream; C5: 3.75 Gbp per GPU
# in 4 chunks).  C3 / C4 shards (0.5-0.63 Gbp) exchange whole.
STREAM_BASES = 1 << 30
# The `<in>_db.npz` dump is built on rank 0 from every rank's (key, mask,
# count) entries: at most this many of them (_grab_counts).
DUMP_MAX_ENTRIES = 1 << 31


def _is_cuda(device) -> bool:
    return getattr(device, "type", str(device)).startswith("cuda")


def _comm_device(device, group):
    """(stage through host memory?, the device collectives run on): gloo moves
    host tensors only."""
    import torch
    import torch.distributed as dist
    stage = _is_cuda(device) and dist.get_backend(group) == "gloo"
    return stage, (torch.device("cpu") if stage else device)


M64 = (1 << 64) - 1
# env PG_EXCHANGE_SELF_RCCL=1: a rank's own run goes through the collective
# like every other (at world 1: through RCCL) instead of a device copy
SELF_COPY = os.environ.get("PG_EXCHANGE_SELF_RCCL") != "1"
# env PG_DEBUG_POISON=<byte>: the exchange's torch buffers are filled with it
# before use (pg_tune PG_TUNE_POISON does the same for the library's own)
_POISON = os.environ.get("PG_DEBUG_POISON")
_NO_FENCE = os.environ.get("PG_DEBUG_NO_FENCE") == "1"


class ExchangeIntegrityError(RuntimeError):
    """Records of the owner exchange changed between the sender's partition
    and the owner's merge (the message names the round, the peer, the piece
    and the stage where the sums first disagree)."""


def _fence(device, table=None):
    """The library runs on its own non-blocking streams, which do not wait on
    torch's: before native code reads or writes memory the torch allocator
    handed out, everything torch's current stream queued (a clone, the wait
    on an RCCL collective) must be done - a block freed behind queued work is
    handed out again at once to the next torch.empty on the same stream.
    With a `table` that can (stream_wait: pg_stream_wait), the library's
    streams wait on an event of torch's current stream, on the device (the
    host does not block); otherwise the device is synchronised.  (Every
    library call returns with its device work done, so torch needs no fence
    after it.)  PG_DEBUG_NO_FENCE=1, diagnostics only: round 4's unfenced
    behaviour."""
    if _is_cuda(device) and not _NO_FENCE:
        import torch
        wait = getattr(table, "stream_wait", None)
        if wait is not None:
            wait(torch.cuda.current_stream(device).cuda_stream)
        else:
            torch.cuda.synchronize(device)


def _fmix64(k):
    k = k ^ (k >> np.uint64(33))
    k = k * np.uint64(0xFF51AFD7ED558CCD)
    k = k ^ (k >> np.uint64(33))
    k = k * np.uint64(0xC4CEB9FE1A85EC53)
    return k ^ (k >> np.uint64(33))


def row_check_sum(rows) -> int:
    """Sum mod 2^64 of row_check (pg_common.h) over records on the host: the
    CPU form of pg_rows_checksum.  `rows`: 16-byte records as (n, 2) 64-bit
    or (n, 4) 32-bit words, or 12-byte routed rows as (n, 3) 32-bit words
    ({h low, h high, mask word}: the hash of {h, mask word, 0})."""
    a = np.ascontiguousarray(np.asarray(rows))
    if a.ndim == 2 and a.shape[1] == 3 and a.dtype.itemsize == 4:
        u = a.view(np.uint32).astype(np.uint64)
        w0, w1 = u[:, 0] | (u[:, 1] << np.uint64(32)), u[:, 2]
    else:
        w = a.reshape(-1).view(np.uint64).reshape(-1, 2)
        w0, w1 = w[:, 0], w[:, 1]
    if w0.shape[0] == 0:
        return 0
    with np.errstate(over="ignore"):
        h = _fmix64(w0 ^ _fmix64(w1 ^ np.uint64(0x9E3779B97F4A7C15)))
        return int(h.sum(dtype=np.uint64))


def _seg_sums(shard, buf, offsets, device) -> list:
    """row_check sums of segments [offsets[i], offsets[i+1]) of the rows of
    buf ((n, 4) int32 16-byte records, or (n, 3) int32 routed rows): on the
    device through the library, on the host with numpy."""
    if len(offsets) < 2:
        return []
    if getattr(buf, "is_cuda", False):
        _fence(device, shard)
        return [int(x) for x in shard.rows_checksum(buf.data_ptr(), np.asarray(offsets, np.uint64))]
    a = buf.numpy() if hasattr(buf, "numpy") else np.asarray(buf)
    return [row_check_sum(a[offsets[i]:offsets[i + 1]]) for i in range(len(offsets) - 1)]


def _poisoned(t):
    if _POISON is not None:
        t.view(-1).view(__import__("torch").uint8).fill_(int(_POISON, 0) & 255)
    return t


def _route(table, world: int, device, group=None, sentinel_local: bool = False, subparts: int = 1, tm=None,
           where: str = "", fail=None, defer=None):
    """This rank's table -> owner runs of records (pg_dbg_partition's 16-byte
    records, or a _Routed table's 12-byte rows: table.row_words 32-bit words
    per row) -> one all-to-all.  Every rank's run lengths and their integrity sums,
    with its n<k sentinel flag, go to every rank in one small all-gather: the
    whole (source, owner) matrix gives this rank's receive sizes, the largest
    peer message (the piece count of _all_to_all_rows), the global sentinel
    and the sums each received run must have; it is the only host read.  With
    `subparts` = P > 1 the table is cut into world x P parts (part q: owner
    q // P, the owner's sub-log q % P; world x P <= 64), so an owner's run
    from each rank arrives already split into its P sub-logs.
    Integrity (always on): the partition must hold every entry of the table
    (record conservation), and every received (source, sub-log) run must
    carry the sum its sender computed while scattering it; a mismatch on any
    rank raises ExchangeIntegrityError on every rank (one MAX all-reduce of a
    flag), naming `where`, the peer, the sub-log and the A2A_ROWS piece.
    `fail`: a failed check of this rank since the last collective (a
    message): it travels in the count matrix and every rank raises.
    `defer` (a dict): the received-run check skips its own all-reduce and
    leaves `bad` (this rank's mismatching runs) and `diagnose` (the
    collective that raises) for the caller's next all-reduce to carry.
    Returns (the records this rank owns as an (n, row_words) int32 tensor on
    `device`, the received counts per (source rank, sub-log) as a (world, P)
    array, their expected sums as a (world, P) array of Python ints, bytes
    sent to other ranks, whether any rank saw the sentinel).  `tm` (a dict)
    accumulates the seconds of the partition and of the all-to-all (the
    collectives are synchronised for it)."""
    import torch
    import torch.distributed as dist
    P = subparts
    W = getattr(table, "row_words", 4)
    stage, comm = _comm_device(device, group)
    rank = dist.get_rank(group)
    t0 = perf_counter()
    counts = table.partition(world * P).astype(np.int64).reshape(world, P)
    total = int(counts.sum())
    n_ent = table.entries() if hasattr(table, "entries") else None
    if n_ent is not None and total != n_ent and not fail:
        fail = ("%s: rank %d's partition holds %d records for a table of %d entries (stage: partition)"
                % (where or "exchange", rank, total, n_ent))
    send = _poisoned(torch.empty((max(total, 1), W), dtype=torch.int32, device=device))
    sums = np.zeros(world * P, np.uint64)
    if total:
        _fence(device, table)
        table.partition(world * P, send.data_ptr(), total)   # (returns after the scatter)
        sums = np.asarray(table.partition_sums(world * P), np.uint64)
    t1 = perf_counter()
    head = np.zeros((world, 2 * P + 2), np.int64)
    head[:, :P] = counts
    head[:, P] = 1 if sentinel_local else 0
    head[:, P + 1:2 * P + 1] = sums.reshape(world, P).view(np.int64)
    head[:, 2 * P + 1] = 1 if fail else 0
    if world == 1:
        H = head.reshape(1, 1, 2 * P + 2)            # (a one-rank all-gather is the identity)
    else:
        send_head = torch.from_numpy(head.reshape(-1)).to(comm)
        heads = [torch.empty_like(send_head) for _ in range(world)]
        dist.all_gather(heads, send_head, group=group)
        H = torch.stack(heads).cpu().numpy().reshape(world, world, 2 * P + 2)  # [source, owner, counts|flag|sums|fail]
    _raise_if_any(fail, H[:, 0, 2 * P + 1].tolist(), rank)
    rh = H[:, rank, :P]
    want = H[:, rank, P + 1:2 * P + 1].copy().view(np.uint64)
    rsplit = rh.sum(axis=1).tolist()
    nrecv = int(sum(rsplit))
    ssplit = counts.sum(axis=1).tolist()
    alias = world == 1 and SELF_COPY and not stage
    # world 1: the rank's only run is its own, and the send buffer already
    # holds it where the receive would put it (no copy, no second buffer)
    recv = send if alias else _poisoned(torch.empty((max(nrecv, 1), W), dtype=torch.int32, device=comm))
    if alias:
        pass
    elif stage:
        dist.all_to_all_single(recv[:nrecv], send.cpu()[:total], output_split_sizes=rsplit,
                               input_split_sizes=ssplit, group=group)
        recv = recv.to(device)
    else:
        _all_to_all_rows(recv, send, rsplit, ssplit, comm, group, big=int(H[:, :, :P].sum(axis=2).max()),
                         self_copy=SELF_COPY)
    # every received (source, sub-log) run against its sender's sum (world 1:
    # nothing moved - the scatter's buffer is the receive - and the owner's
    # merge checks the same sums over what it reads)
    off = np.concatenate([[0], np.cumsum(rh.reshape(-1))]).astype(np.int64).tolist()
    got = [int(x) for x in want.reshape(-1)] if alias else _seg_sums(table, recv, off, device)
    bad = [(s, p) for s in range(world) for p in range(P) if got[s * P + p] != int(want[s, p])]
    if defer is not None:
        # the caller's next all-reduce carries the check.  (The closure keeps
        # the send buffer until the caller returns - one more buffer of 12 B
        # per sent record at the owner merge's peak, <= ~1 GB for C4-sized
        # shards - rather than summing its pieces up front on every exchange:
        # a pass over the whole buffer, ~0.1 ms on C3, for a failure path.)
        defer["bad"] = bad
        defer["diagnose"] = lambda: _diagnose(table, send, recv, counts, sums, rh, bad, world, P, rank, device, comm,
                                              group, where)
    elif world == 1:
        if bad:
            _diagnose(table, send, recv, counts, sums, rh, bad, world, P, rank, device, comm, group, where)
    else:
        flag = torch.tensor([1 if bad else 0], dtype=torch.int64, device=comm)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
        if int(flag.item()):
            _diagnose(table, send, recv, counts, sums, rh, bad, world, P, rank, device, comm, group, where)
    if tm is not None:
        if _is_cuda(device):
            torch.cuda.synchronize(device)
        t2 = perf_counter()
        tm["partition"] = tm.get("partition", 0.0) + (t1 - t0)
        tm["all_to_all"] = tm.get("all_to_all", 0.0) + (t2 - t1)
        tm["rows"] = tm.get("rows", 0) + total
    want_l = [[int(want[s, p]) for p in range(P)] for s in range(world)]
    return recv[:nrecv], rh, want_l, 4 * W * (total - int(counts[rank].sum())), bool(H[:, :, P].any())


def _piece_count(ssplit, rsplit) -> int:
    return max(1, int(-(-max(int(np.max(ssplit)), int(np.max(rsplit)), 1) // A2A_ROWS)))


def _piece_offsets(split, world: int, npc: int):
    base = np.concatenate([[0], np.cumsum(split)]).astype(np.int64)
    return [[int(min(base[o] + j * A2A_ROWS, base[o + 1])) for j in range(npc + 1)] for o in range(world)]


def _piece_sums(table, send, ssplit, rsplit, world: int, device, npc=None):
    """(npc, this rank's send buffer summed per owner and A2A_ROWS piece as a
    (world, npc) uint64 array)."""
    npc = npc or _piece_count(ssplit, rsplit)
    so = _piece_offsets(ssplit, world, npc)
    return npc, np.array([_seg_sums(table, send, so[o], device) for o in range(world)], np.uint64).reshape(world, npc)


def _diagnose(table, send, recv, counts, sums, rh, bad, world, P, rank, device, comm, group, where, pieces=None):
    """A received run's sum disagreed somewhere: every rank sums its send and
    receive messages per A2A_ROWS piece, the senders' piece sums go to every
    rank, and every rank raises, the receivers naming the pieces that
    differ.  The piece count is the largest over the ranks (one MAX
    all-reduce before any rank diverges), a rank with fewer pieces padding
    with empty ones, so every rank reaches the all-gather.  `pieces`: this
    rank's send piece sums computed before its send buffer was released
    (then `send` is None)."""
    import torch
    import torch.distributed as dist
    ssplit, rsplit = counts.sum(axis=1), rh.sum(axis=1)
    npc_t = torch.tensor([pieces[0] if pieces else _piece_count(ssplit, rsplit)], dtype=torch.int64, device=comm)
    dist.all_reduce(npc_t, op=dist.ReduceOp.MAX, group=group)
    npc = int(npc_t.item())
    if pieces is not None:
        mine = np.zeros((world, npc), np.uint64)
        mine[:, :pieces[0]] = pieces[1]                 # (pieces past a rank's own count are empty: sum 0)
    else:
        mine = _piece_sums(table, send, ssplit, rsplit, world, device, npc)[1]
    ro = _piece_offsets(rsplit, world, npc)
    psum = sums.reshape(world, P)
    with np.errstate(over="ignore"):
        changed = [o for o in range(world) if int(mine[o].sum(dtype=np.uint64)) != int(psum[o].sum(dtype=np.uint64))]
    t = torch.from_numpy(mine.view(np.int64).reshape(-1)).to(comm)
    allp = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(allp, t, group=group)
    sent = torch.stack(allp).cpu().numpy().view(np.uint64).reshape(world, world, npc)   # [source, owner, piece]
    msgs = ["this rank's send buffer for owners %s no longer matches its partition sums (stage: send buffer, between "
            "the scatter and the all_to_all)" % changed] if changed else []
    for s in sorted({b[0] for b in bad}):
        got = _seg_sums(table, recv, ro[s], device)
        pcs = [j for j in range(npc) if got[j] != int(sent[s, rank, j])]
        msgs.append("from rank %d: sub-logs %s, %s (stage: all_to_all, %s)"
                    % (s, [p for (s2, p) in bad if s2 == s],
                       "pieces %s of %d rows each differ on the wire" % (pcs, A2A_ROWS) if pcs else
                       "no piece differs on the wire: the sender's buffer changed after its partition sums",
                       "self copy" if s == rank and SELF_COPY else "collective"))
    raise ExchangeIntegrityError("%s: rank %d: exchanged records changed between the partition and the receive: %s"
                                 % (where or "exchange", rank, "; ".join(msgs) or "(another rank's records)"))


# Records per peer and collective on device backends: RCCL 2.26 (ROCm 7)
# all_to_all returns wrong data for a peer message past 1 GiB (half of a
# 1.6 GB message lost at world 1, tools/rccl_a2a_check.py); a C5 round moves
# ~2 GB per peer at N = 8.
A2A_ROWS = 1 << 25


def _all_to_all_rows(recv, send, rsplit, ssplit, comm, group=None, big=None, self_copy=True):
    """all_to_all of rows (a 2-D tensor, any row width) in pieces of at most A2A_ROWS rows per
    peer (every rank runs the same number of pieces: the largest message of
    any rank decides; `big`, when the caller knows it, else one MAX
    all-reduce finds it).  Views of contiguous runs; the rank's own run is a
    device copy and never goes through the collective (`self_copy=False`:
    it does, as every other run; at world 1 that drives RCCL)."""
    import torch
    import torch.distributed as dist
    world = len(ssplit)
    me = dist.get_rank(group) if world > 1 else 0
    if not self_copy:
        me = -1
    if me >= 0 and ssplit[me]:
        so_me = int(np.sum(ssplit[:me])) if me else 0
        ro_me = int(np.sum(rsplit[:me])) if me else 0
        recv[ro_me:ro_me + rsplit[me]].copy_(send[so_me:so_me + ssplit[me]])
    if world == 1 and me == 0:
        return
    ssplit, rsplit = list(ssplit), list(rsplit)
    ssplit_me, rsplit_me = (ssplit[me], rsplit[me]) if me >= 0 else (0, 0)
    if me >= 0:
        ssplit[me] = rsplit[me] = 0
    if big is None:
        b = torch.tensor([max(max(ssplit), max(rsplit)) if world else 0], dtype=torch.int64, device=comm)
        dist.all_reduce(b, op=dist.ReduceOp.MAX, group=group)
        big = int(b.item())
    # (offsets from the real run lengths: the own run keeps its place)
    so = np.concatenate([[0], np.cumsum([x if i != me else ssplit_me for i, x in enumerate(ssplit)])]).astype(np.int64)
    ro = np.concatenate([[0], np.cumsum([x if i != me else rsplit_me for i, x in enumerate(rsplit)])]).astype(np.int64)
    npieces = max(1, -(-int(big) // A2A_ROWS))
    lists = dist.get_backend(group) != "gloo"             # (gloo has no list all_to_all: pieces copied)
    for j in range(npieces):
        lo = j * A2A_ROWS
        ins = [send[so[o] + min(lo, ssplit[o]):so[o] + min(lo + A2A_ROWS, ssplit[o])] for o in range(world)]
        outs = [recv[ro[o] + min(lo, rsplit[o]):ro[o] + min(lo + A2A_ROWS, rsplit[o])] for o in range(world)]
        if lists:
            dist.all_to_all(outs, ins, group=group)
        else:
            tmp = torch.empty((max(1, sum(x.shape[0] for x in outs)),) + tuple(recv.shape[1:]), dtype=recv.dtype,
                              device=recv.device)
            n = sum(x.shape[0] for x in outs)
            dist.all_to_all_single(tmp[:n], torch.cat(ins), output_split_sizes=[x.shape[0] for x in outs],
                                   input_split_sizes=[x.shape[0] for x in ins], group=group)
            at = 0
            for x in outs:
                x.copy_(tmp[at:at + x.shape[0]])
                at += x.shape[0]


def _merge_checked(table, buf, n: int, sentinel: bool, want_sum: int, device, what: str):
    """table.merge of the first n records of buf, then what the merge read
    against (n, want_sum): record conservation and integrity of the log
    between the all-to-all and the merge.  Returns None, or the mismatch as a
    message for the caller to raise on every rank at its next collective
    (raising here alone would leave the other ranks waiting in it)."""
    _fence(device, table)
    table.merge(buf.data_ptr() if n else 0, n, sentinel=sentinel)
    if hasattr(table, "merge_check"):
        rows, s = table.merge_check()
        if rows != n or (s & M64) != (want_sum & M64):
            return ("%s: the merge read %d records with sum %#x, the log holds %d with sum %#x (stage: merge)"
                    % (what, rows, s, n, want_sum & M64))
    return None


def _raise_if_any(fail, flags, rank: int):
    """every rank raises when any rank's check failed (flags: one per rank)"""
    bad = [r for r, f in enumerate(flags) if f]
    if bad:
        raise ExchangeIntegrityError(fail if fail else "exchange: rank(s) %s failed an integrity check (rank %d's "
                                     "records are fine)" % (bad, rank))


def _owner_reduce(table, recv, rank: int, device, sentinel_local: bool, group=None, sentinel_global=None, tm=None,
                  want_sum=None, route=None):
    """OR-merge the owned records into a fresh owner table, rdBG rule on it;
    global (n_dbg, n_rdbg) by one sum all-reduce.  `sentinel_global`: whether
    any rank saw the n<k sentinel, when the caller already knows (else one MAX
    all-reduce of `sentinel_local` finds out); `want_sum`: the integrity sum
    the received records must have; `route`: _route's deferred receive
    check, carried by the count all-reduce.  Returns (n_dbg_total, n_rdbg_total,
    n_rdbg_local); `tm["merge"]` accumulates the seconds of the merge, the
    rdBG rule and the count all-reduce."""
    import torch
    import torch.distributed as dist
    _, comm = _comm_device(device, group)
    world = dist.get_world_size(group)
    t0 = perf_counter()
    if sentinel_global is None:
        if world == 1:
            sentinel_global = bool(sentinel_local)
        else:
            flag = torch.tensor([1 if sentinel_local else 0], dtype=torch.int64, device=comm)
            dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
            sentinel_global = bool(flag.item())
    # the n<k sentinel key belongs to one owner: rank 0
    n = int(recv.shape[0])
    fail = None
    if want_sum is None:
        _fence(device, table)
        table.merge(recv.data_ptr(), n, sentinel=sentinel_global and rank == 0)
    else:
        fail = _merge_checked(table, recv, n, sentinel_global and rank == 0, want_sum, device,
                              "exchange: rank %d's owner merge" % rank)
    st = table.build_rdbg()
    rbad = 1 if route and route.get("bad") else 0
    if world == 1:                                    # (a one-rank all-reduce is the identity)
        n_dbg, n_rdbg, nfail, nrbad = int(st.n_dbg), int(st.n_rdbg), 1 if fail else 0, rbad
    else:
        sums = torch.tensor([st.n_dbg, st.n_rdbg, 1 if fail else 0, rbad], dtype=torch.int64, device=comm)
        dist.all_reduce(sums, op=dist.ReduceOp.SUM, group=group)
        n_dbg, n_rdbg, nfail, nrbad = sums.tolist()
    if nrbad:
        route["diagnose"]()                          # (collective; raises on every rank)
    if nfail:
        _raise_if_any(fail, [1], rank)
    if tm is not None:
        tm["merge"] = tm.get("merge", 0.0) + (perf_counter() - t0)
    return int(n_dbg), int(n_rdbg), int(st.n_rdbg)


def exchange_and_reduce(table, world: int, rank: int, device, sentinel_local: bool, group=None, tm=None):
    """Owner all-to-all + OR-merge + rdBG rule on the owner partition: two
    host reads (the count matrix, the global counts) besides the partition's
    own count read.  Returns (n_dbg_total, n_rdbg_total, n_rdbg_local,
    bytes_sent); `tm` accumulates partition / all_to_all / merge seconds."""
    chk = {}
    recv, _, want, sent, sentinel = _route(table, world, device, group, sentinel_local, tm=tm, where="exchange",
                                           defer=chk)
    want_sum = sum(x for row in want for x in row) & M64
    return _owner_reduce(table, recv, rank, device, sentinel_local, group, sentinel_global=sentinel, tm=tm,
                         want_sum=want_sum, route=chk) + (sent,)


class _Routed:
    """A shard whose last build held its stage A records for their owners
    (route_stage_a), seen by _route / _owner_reduce as a table: its
    "partition" is the held records grouped by owner (whole stage A regions:
    the owner is the top bits of the record's h), its "merge" the owner's
    build from the received records (stages A, B, C once)."""

    row_words = 3                                       # 12-byte rows {h, mask word} (pg_route_scatter)

    def __init__(self, shard, nparts: int, counts):
        self.sh, self.nparts, self.counts = shard, nparts, np.asarray(counts, np.uint64)

    def partition(self, nparts, ptr=None, cap=0):
        if nparts != self.nparts:
            raise ValueError("routed records are held for %d owners, not %d" % (self.nparts, nparts))
        if ptr is not None:
            self.sums = self.sh.route_scatter(nparts, ptr, cap)
        return self.counts

    def partition_sums(self, nparts):
        return self.sums

    def entries(self):
        return int(self.counts.sum())

    def rows_checksum(self, d_rows, seg_off):
        return self.sh.route_rows_checksum(d_rows, seg_off)

    @property
    def stream_wait(self):
        return getattr(self.sh, "stream_wait", None)

    def merge(self, ptr, n, sentinel=False):
        self.sh.route_merge(ptr, n, self.nparts, sentinel)

    def merge_check(self):
        return self.sh.merge_check()

    def build_rdbg(self):
        return self.sh.build_rdbg()


def exchange_routed(shard, world: int, rank: int, device, flags, extra: int, rc0: bool, group=None, tm=None,
                    force: bool = False):
    """The N>1 build-and-reduce step with the owners building once: stage A
    of this rank's records (held, not built: route_stage_a), the records to
    their owners in one all-to-all (the owner = the top log2(world) bits of
    h, so a rank's run for one owner is whole stage A regions: a segmented
    copy, pg_route_scatter), and each owner's stages A (re-binning), B and
    C over what it received (pg_route_merge) - no local table, no
    pg_dbg_partition, no second full build.  World 1: stages B and C on the
    held records where they lie (pg_route_finish; force: through the
    scatter, the own run's device copy and the owner merge as at N > 1, to
    price them).  The same integrity checks
    as exchange_and_reduce (per-run sums from the scatter to the merge, record
    conservation).  A world that is not a power of two builds locally and
    runs exchange_and_reduce instead (same result).  Returns (n_dbg_total,
    n_rdbg_total, n_rdbg_local, bytes_sent); `tm` accumulates partition /
    all_to_all / merge seconds (partition = the scatter of the held regions)."""
    if not _pow2(world):
        # (the routed owner is a top-bit range of h: 2^j owners only) any
        # other world size runs the local-table exchange on a local build
        st = shard.build(flags, extra, rc0)                 # (GpuShard: the flag; a Context: its stats)
        return exchange_and_reduce(shard, world, rank, device, bool(getattr(st, "sentinel", st)), group, tm)
    counts, sentinel = shard.route_stage_a(flags, extra, rc0, world)
    if world == 1 and not force:
        t0 = perf_counter()
        st = shard.route_finish()
        if tm is not None:
            tm["merge"] = tm.get("merge", 0.0) + (perf_counter() - t0)
        return int(st.n_dbg), int(st.n_rdbg), int(st.n_rdbg), 0
    return exchange_and_reduce(_Routed(shard, world, counts), world, rank, device, sentinel, group, tm)


def stream_chunks(flags, seq_len, limit: int) -> list:
    """A rank's flagged records as consecutive chunks of at most `limit`
    forward bases each (a longer record is a chunk of its own): record flag
    arrays, one per chunk."""
    flags = np.asarray(flags, np.uint8)
    out, cur, n = [], [], 0
    for r in np.flatnonzero(flags).tolist():
        L = int(seq_len[r])
        if cur and n + L > limit:
            out.append(cur)
            cur, n = [], 0
        cur.append(r)
        n += L
    if cur:
        out.append(cur)
    res = []
    for c in out:
        f = np.zeros(flags.shape[0], np.uint8)
        f[c] = 1
        res.append(f)
    return res


def sublog_count(world: int, rounds: int, subparts=None) -> int:
    """The owner's sub-log count P of exchange_stream: `subparts` or the round
    count, rounded up to a power of two, but never past the largest power of
    two with world x P <= 64 (pg_dbg_partition's part limit; world 3: 16)."""
    P, want, cap = 1, max(1, subparts or rounds), 64 // max(1, world)
    while P < want and P * 2 <= cap:
        P *= 2
    return P


def _free_device_bytes(device) -> int:
    import torch
    if _is_cuda(device):
        return int(torch.cuda.mem_get_info(device)[0])
    return 1 << 36


def _pow2(n: int) -> bool:
    return n >= 1 and not n & (n - 1)


def exchange_stream(shard, world: int, rank: int, device, chunks: list, n_records: int, rc0: bool, extra: int = 0,
                    staged=None, group=None, on_chunk=None, compact_at=None, subparts=None, tm=None, routed=None,
                    lib_stats=None, keys=True):
    """The streaming exchange of SURVEY §8(e) for shards whose whole local
    table does not fit beside the owner partition (C5: 3.75 Gbp per GPU).

    Two forms.  `routed` (the default whenever no local table is needed:
    no `on_chunk` count gathering, no `staged` checkpoint slots, no explicit
    `compact_at`, and a power-of-two world): _stream_routed - every chunk's
    stage A records go straight to their owners, which build each sub-log
    once at the end; nothing is built locally.  Otherwise the local-table
    form below.

    Per chunk of records (stream_chunks): the local OR-table of the chunk
    (`shard.build`, K1 already done for the whole shard), its entries to their
    owners with one all-to-all (`_route`).  The owner keeps what it receives
    in `subparts` sub-logs by a hash of the key (default: the round count,
    rounded up to a power of two, at most 64 / world: _route cuts the
    sender's table into world x P parts, so the sub-logs arrive split and
    no device-wide sort of a round's records is needed), so that no step ever handles the whole
    log at once: a compaction OR-merges ONE sub-log (pg_dbg_merge, 1/P of the
    owner's entries, within the stage A-C buffers the chunk builds already
    hold) and re-exports it in place (pg_dbg_partition into one run); it runs
    on a sub-log that has doubled since its last compaction once the whole log
    holds `compact_at` records (default: a quarter of the device memory free
    when the exchange starts, at 16 B per record).  After the last chunk each
    sub-log is merged once, the rdBG rule applied to it and its rdBG keys
    kept; the owner's counts are the sums.  Every rank runs the same number of
    rounds (the maximum chunk count; a rank out of records builds an empty
    chunk).  `staged` (rank 0's -r checkpoint slots) goes into the first chunk
    only; `extra` (the n<k empty records) too.  `on_chunk()` runs after each
    chunk's build (the dump gathers its occurrence counts there).  Returns
    (n_dbg_total, n_rdbg_total, n_rdbg_local, bytes_sent, rounds, the owner's
    rdBG keys - sorted within each sub-log, not across them: the callers
    sort what they gather; routed form with keys=False: counts only, the
    keys are not exported and the last item is None).  `lib_stats` (a dict, routed form): filled with the
    library's HIP-event spans and record counts of every round and sub-log
    merge.  `tm` (a dict) accumulates the seconds of each phase (build,
    route = partition + all-to-all + checks, compact, final = the sub-logs'
    merges, rdBG rules and key exports), the device synchronised at each
    phase boundary."""
    import torch
    import torch.distributed as dist
    _, comm = _comm_device(device, group)
    if routed is None:
        routed = on_chunk is None and staged is None and compact_at is None and _pow2(world)
    if routed and (on_chunk is not None or staged is not None or not _pow2(world)):
        raise ValueError("exchange_stream: the routed form needs a power-of-two world and no local table "
                         "(on_chunk / staged)")
    lap = _lapper(tm, device)
    t0 = perf_counter()
    nch = torch.tensor([len(chunks)], dtype=torch.int64, device=comm)
    dist.all_reduce(nch, op=dist.ReduceOp.MAX, group=group)
    rounds = max(1, int(nch.item()))
    P = sublog_count(world, rounds, subparts)
    lap("setup", t0)
    if routed:
        return _stream_routed(shard, world, rank, device, chunks, n_records, rc0, extra, group, rounds, P, lap,
                              lib_stats, keys)
    if compact_at is None:
        compact_at = max(1 << 20, _free_device_bytes(device) // 4 // 16)
    logs = [[] for _ in range(P)]
    logn, base = [0] * P, [0] * P
    logsum = [0] * P                                   # integrity sum of each sub-log's records (mod 2^64)
    sentinel, sent = False, 0
    fail = []                                          # failed checks, raised on every rank at the next collective

    def compact(p, i):
        cat = torch.cat(logs[p]) if len(logs[p]) > 1 else logs[p][0]
        logs[p] = []                                   # (the pieces go as soon as they are merged)
        f = _merge_checked(shard, cat, int(cat.shape[0]), False, logsum[p], device,
                           "exchange round %d: rank %d's compaction of sub-log %d" % (i, rank, p))
        if f:
            fail.append(f)
        del cat
        m = int(shard.partition(1)[0])
        out = _poisoned(torch.empty((max(m, 1), 4), dtype=torch.int32, device=device))
        if m:
            _fence(device, shard)
            shard.partition(1, out.data_ptr(), m)
        logs[p] = [out[:m]] if m else []
        logn[p] = base[p] = m
        logsum[p] = int(shard.partition_sums(1)[0]) if m else 0

    for i in range(rounds):
        if staged is not None and i < 2:
            if i == 0:
                shard.stage(*staged)
            else:
                shard.stage(np.zeros(0, np.uint64))
        f = chunks[i] if i < len(chunks) else np.zeros(n_records, np.uint8)
        t0 = lap("start", perf_counter())
        sentinel |= bool(shard.build(f, extra if i == 0 else 0, rc0))
        if on_chunk is not None:
            on_chunk()
        t0 = lap("build", t0)
        recv, sub, want, s, _ = _route(shard, world, device, group, subparts=P, where="exchange round %d" % i,
                                       fail=fail[0] if fail else None)
        t0 = lap("route", t0)
        sent += s
        # each source's run arrives as its P sub-log runs; with P > 1 each run
        # is copied out, so that compacting one sub-log frees its memory (a
        # view would keep the whole round's receive buffer alive)
        off = 0
        for src in range(sub.shape[0]):
            for p in range(P):
                m = int(sub[src, p])
                if m:
                    logs[p].append(recv[off:off + m].clone() if P > 1 else recv[off:off + m])
                    logn[p] += m
                    logsum[p] = (logsum[p] + want[src][p]) & M64
                off += m
        del recv
        t0 = lap("log", t0)
        total = sum(logn)
        if total >= compact_at:
            for p in sorted(range(P), key=lambda q: -logn[q]):
                if logn[p] >= 2 * base[p] and len(logs[p]) > 1:
                    compact(p, i)
        lap("compact", t0)
    # the n<k sentinel key belongs to one owner: rank 0 (sub-log 0)
    flag = torch.tensor([1 if sentinel else 0, 1 if fail else 0], dtype=torch.int64, device=comm)
    dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
    sent_global = bool(flag[0].item())
    if int(flag[1].item()):
        _raise_if_any(fail[0] if fail else None, [1], rank)
    n_dbg_loc = n_rdbg_loc = 0
    keys = []
    t0 = lap("start", perf_counter())
    for p in range(P):
        cat = (torch.cat(logs[p]) if len(logs[p]) > 1 else logs[p][0]) if logs[p] else None
        logs[p] = []
        n = 0 if cat is None else int(cat.shape[0])
        if n != logn[p]:
            fail.append("exchange: rank %d's sub-log %d holds %d records, %d were received (stage: log)"
                        % (rank, p, n, logn[p]))
        f = _merge_checked(shard, cat, n, sent_global and rank == 0 and p == 0, logsum[p], device,
                           "exchange: rank %d's final merge of sub-log %d" % (rank, p))
        if f:
            fail.append(f)
        del cat
        st = shard.build_rdbg()
        n_dbg_loc += int(st.n_dbg)
        n_rdbg_loc += int(st.n_rdbg)
        keys.append(np.ascontiguousarray(shard.owner_rdbg(), dtype=np.uint64))
    lap("final", t0)
    sums = torch.tensor([n_dbg_loc, n_rdbg_loc, 1 if fail else 0], dtype=torch.int64, device=comm)
    dist.all_reduce(sums, op=dist.ReduceOp.SUM, group=group)
    n_dbg, n_rdbg, nfail = sums.tolist()
    if nfail:
        _raise_if_any(fail[0] if fail else None, [1], rank)
    own = np.concatenate(keys) if keys else np.zeros(0, np.uint64)      # (each sub-log's keys sorted)
    return int(n_dbg), int(n_rdbg), n_rdbg_loc, sent, rounds, own


def _lapper(tm, device):
    """lap(name, t0): with a `tm` dict, synchronise the device and add the
    seconds since t0 to tm[name]; returns the new t0."""
    def lap(name, t0):
        if tm is None:
            return 0.0
        if _is_cuda(device):
            import torch
            torch.cuda.synchronize(device)
        t1 = perf_counter()
        tm[name] = tm.get(name, 0.0) + (t1 - t0)
        return t1
    return lap


def _stream_routed(shard, world: int, rank: int, device, chunks, n_records: int, rc0: bool, extra: int, group,
                   rounds: int, P: int, lap, lib_stats=None, want_keys=True):
    """exchange_stream's routed form.  Per round: stage A of the chunk held
    for its owners (pg_route_stage_a; every rank runs `rounds` rounds, an
    empty chunk when out of records), the held regions to their owners in
    world x P parts (the owner = the top log2(world) bits of h, its sub-log
    the next log2(P): _route over a _Routed view, with the same integrity
    sums from the scatter to the merge), and the received buffer kept as it
    arrived - its runs are the sub-logs' segments.  At the end each sub-log
    is one owner table built from all of its segments at once
    (pg_route_merge_segs: stages A (re-binning), B and C, no concatenation),
    its rdBG counted and its keys exported.  Owner memory: 12 B per received
    record (C5 at N = 8: ~3.75e9 records, 45 GB) plus one sub-log's build."""
    import torch
    import torch.distributed as dist
    _, comm = _comm_device(device, group)
    nparts = world * P
    # with `lib` (a dict): the library's own spans of every round and merge
    # (HIP events; the shard's stats()), for the bench's per-stage roofline
    lib = {"rounds": [], "merges": []} if lib_stats is not None and hasattr(shard, "stats") else None
    bufs, segs = [], [[] for _ in range(P)]             # received buffers; per sub-log (device pointer, rows)
    logn, logsum = [0] * P, [0] * P
    sentinel, sent = False, 0
    fail = []
    for i in range(rounds):
        f = chunks[i] if i < len(chunks) else np.zeros(n_records, np.uint8)
        t0 = lap("start", perf_counter())
        counts, s_flag = shard.route_stage_a(f, extra if i == 0 else 0, rc0, nparts)
        sentinel |= bool(s_flag)
        t0 = lap("build", t0)
        if lib is not None:
            st = shard.stats()
            lib["rounds"].append(dict(stage_a_ms=st.ms_insert, records=int(counts.sum()), work_items=st.n_work_items,
                                      windows=st.n_windows))
        recv, sub, want, s, _ = _route(_Routed(shard, nparts, counts), world, device, group, subparts=P,
                                       where="exchange round %d" % i, fail=fail[0] if fail else None)
        t0 = lap("route", t0)
        sent += s
        off = 0
        base = recv.data_ptr() if hasattr(recv, "data_ptr") else recv.ctypes.data
        for src in range(sub.shape[0]):
            for p in range(P):
                m = int(sub[src, p])
                if m:
                    segs[p].append((base + 12 * off, m))
                    logn[p] += m
                    logsum[p] = (logsum[p] + want[src][p]) & M64
                off += m
        bufs.append(recv)
        lap("log", t0)
    # the n<k sentinel key belongs to one owner: rank 0 (sub-log 0)
    t0 = perf_counter()
    flag = torch.tensor([1 if sentinel else 0, 1 if fail else 0], dtype=torch.int64, device=comm)
    dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
    sent_global = bool(flag[0].item())
    if int(flag[1].item()):
        _raise_if_any(fail[0] if fail else None, [1], rank)
    n_dbg_loc = n_rdbg_loc = 0
    keys = []
    t0 = lap("flag", t0)
    for p in range(P):
        _fence(device, shard)
        shard.route_merge_segs(segs[p], nparts, sentinel=sent_global and rank == 0 and p == 0)
        rows, sm = shard.merge_check()
        if rows != logn[p] or (sm & M64) != logsum[p]:
            fail.append("exchange: rank %d's final merge of sub-log %d read %d records with sum %#x, the log holds %d "
                        "with sum %#x (stage: merge)" % (rank, p, rows, sm & M64, logn[p], logsum[p]))
        st = shard.build_rdbg()
        n_dbg_loc += int(st.n_dbg)
        n_rdbg_loc += int(st.n_rdbg)
        if lib is not None:
            lib["merges"].append(dict(rebin_ms=st.ms_insert, split_ms=st.ms_split, range_ms=st.ms_range,
                                      records=int(logn[p]), buckets=int(st.table_capacity), n_rdbg=int(st.n_rdbg),
                                      split_passes=int(st.build_flags) >> 16 & 255))
        t0 = lap("merge", t0)
        if want_keys:
            keys.append(np.ascontiguousarray(shard.owner_rdbg(), dtype=np.uint64))
            t0 = lap("keys", t0)
    del bufs
    sums = torch.tensor([n_dbg_loc, n_rdbg_loc, 1 if fail else 0], dtype=torch.int64, device=comm)
    dist.all_reduce(sums, op=dist.ReduceOp.SUM, group=group)
    n_dbg, n_rdbg, nfail = sums.tolist()
    if nfail:
        _raise_if_any(fail[0] if fail else None, [1], rank)
    own = (np.concatenate(keys) if keys else np.zeros(0, np.uint64)) if want_keys else None   # (sorted per sub-log)
    lap("tail", t0)
    if lib is not None:
        lib_stats.update(lib, subparts=P)
    return int(n_dbg), int(n_rdbg), n_rdbg_loc, sent, rounds, own


# ------------------------------------------------------------------ sharding
def _find_header_after(buf, pos: int, step: int = 1 << 22) -> int:
    """Smallest p >= pos with buf[p] == '>' and buf[p-1] == '\\n' (a header
    line start other than byte 0), or len(buf)."""
    n = len(buf)
    p = max(pos, 1)
    while p < n:
        a = np.asarray(buf[p - 1:min(n, p + step)])
        hit = np.flatnonzero((a[:-1] == 10) & (a[1:] == 62))
        if hit.shape[0]:
            return p + int(hit[0])
        p += step
    return n


def shard_bounds(buf, world: int) -> list:
    """Byte bounds of the world shards of a FASTA: about len/world bytes each,
    split just before a header line, so a shard starts in the line state
    seqio_jit_ (:135-172) is in at that header in the whole file.  A split that
    would leave the last shard without any '\\n' is not taken: readline_jit_'s
    final unterminated line is yielded only when it does not start at byte 0
    (`end > start > 0`, :130), which differs between a shard and the file."""
    n = len(buf)
    b = [0]
    for r in range(1, world):
        p = _find_header_after(buf, max(b[-1], r * n // world))
        b.append(max(p, b[-1]))
    b.append(n)
    # the last non-empty shard must hold a newline unless it starts at byte 0
    # (the shard before it then ends with the '\n' before its header)
    s = max((x for x in b[1:world] if x < n), default=0)
    if s > 0 and not np.any(np.asarray(buf[s:n]) == 10):
        b = [x if j == 0 or x < s else n for j, x in enumerate(b)]
    return b


class Shards:
    """The global record table assembled from every rank's shard-relative one."""

    def __init__(self, metas: list, bounds: list, n_bytes: int):
        self.bounds = bounds
        self.R = [int(m["seq_len"].shape[0]) for m in metas]
        self.off = np.concatenate([[0], np.cumsum(self.R)]).astype(np.int64)
        cat = lambda k, add: np.concatenate([m[k].astype(np.int64) + (bounds[i] if add else 0)
                                             for i, m in enumerate(metas)]) if metas else np.zeros(0, np.int64)
        self.seq_len = cat("seq_len", False)
        self.hdr_start = cat("hdr_start", True)
        self.hdr_len = cat("hdr_len", False)
        ptr = cat("ptr", True)
        # a shard's last record is yielded, in the whole file, when seqio reads
        # the next shard's first header line: its ptr is that line's start
        for i in range(len(metas)):
            if self.R[i] and bounds[i + 1] < n_bytes:
                ptr[self.off[i + 1] - 1] = bounds[i + 1]
        self.ptr = ptr

    def local(self, arr, rank: int):
        return arr[self.off[rank]:self.off[rank + 1]]


# ------------------------------------------------------------- communication
class Comm:
    """The few collectives the pipeline needs, on torch.distributed (RCCL over
    xGMI when the backend is nccl; gloo moves host tensors)."""

    def __init__(self, device, group=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.group = torch, dist, group
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        self.dev = torch.device("cpu") if dist.get_backend(group) == "gloo" else device

    def allgather_obj(self, obj):
        out = [None] * self.world
        self.dist.all_gather_object(out, obj, group=self.group)
        return out

    def _sizes(self, n: int):
        t = self.torch.tensor([n], dtype=self.torch.int64, device=self.dev)
        out = [self.torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t, group=self.group)
        return [int(x.item()) for x in out]

    def gather_bytes(self, payload: np.ndarray, dst: int = 0):
        """Variable-size uint8 payloads to rank dst (point to point), in rank order."""
        torch = self.torch
        payload = np.ascontiguousarray(payload, dtype=np.uint8).reshape(-1)
        sizes = self._sizes(payload.shape[0])
        if self.rank != dst:
            if payload.shape[0]:
                self.dist.send(torch.from_numpy(payload).to(self.dev), dst, group=self.group)
            return None
        out = []
        for r in range(self.world):
            if r == dst:
                out.append(payload)
            elif sizes[r]:
                t = torch.empty(sizes[r], dtype=torch.uint8, device=self.dev)
                self.dist.recv(t, r, group=self.group)
                out.append(t.cpu().numpy())
            else:
                out.append(np.zeros(0, np.uint8))
        return out

    def allgather_bytes(self, payload: np.ndarray):
        torch = self.torch
        payload = np.ascontiguousarray(payload, dtype=np.uint8).reshape(-1)
        sizes = self._sizes(payload.shape[0])
        m = max(max(sizes), 1)
        t = torch.zeros(m, dtype=torch.uint8, device=self.dev)
        if payload.shape[0]:
            t[:payload.shape[0]] = torch.from_numpy(payload).to(self.dev)
        out = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t, group=self.group)
        return [o[:s].cpu().numpy() for o, s in zip(out, sizes)]

    def bcast_bytes(self, payload, src: int = 0) -> np.ndarray:
        torch = self.torch
        n = self.torch.tensor([payload.shape[0] if self.rank == src else 0], dtype=torch.int64, device=self.dev)
        self.dist.broadcast(n, src, group=self.group)
        t = torch.empty(int(n.item()), dtype=torch.uint8, device=self.dev)
        if self.rank == src and payload.shape[0]:
            t.copy_(torch.from_numpy(np.ascontiguousarray(payload, dtype=np.uint8)).to(self.dev))
        if t.numel():
            self.dist.broadcast(t, src, group=self.group)
        return t.cpu().numpy()

    def barrier(self):
        self.dist.barrier(group=self.group)


def _pack(*arrs) -> np.ndarray:
    """Arrays of 8-byte elements -> one uint8 payload (a header of lengths)."""
    hdr = np.array([len(arrs)] + [a.shape[0] if a.ndim == 1 else a.size for a in arrs], np.int64)
    return np.concatenate([hdr.view(np.uint8)] + [np.ascontiguousarray(a).reshape(-1).view(np.uint8)
                                                  for a in arrs])


def _unpack(buf: np.ndarray, dtypes):
    hdr = buf[:8].view(np.int64)
    k = int(hdr[0])
    lens = buf[8:8 * (k + 1)].view(np.int64)
    out, o = [], 8 * (k + 1)
    for n, dt in zip(lens.tolist(), dtypes):
        nb = n * np.dtype(dt).itemsize
        out.append(buf[o:o + nb].view(dt))
        o += nb
    return out


# ------------------------------------------------------------ shard backend
class GpuShard:
    """This rank's records on its GPU (a pg_ctx through the C ABI)."""

    def __init__(self, k: int, device: int):
        from ._lib import Context
        self.ctx = Context(k, device)

    def load(self, data):
        self.ctx.parse_host(data)
        return self.ctx.records()

    def stage(self, keys, masks=None, counts=None):
        self.ctx.dbg_load(keys, masks, counts)

    def build(self, flags, extra, rc0):
        st = self.ctx.build_dbg(flags, int(extra), bool(rc0))
        self.n_entries = int(st.n_slots)
        return bool(st.sentinel)

    def entries(self):
        """canonical entries of the last build or merge (what a partition must hold)"""
        return self.n_entries

    def counts(self):
        _, _, keys, values, counts = self.ctx.dbg_dump()
        sel = counts > 0
        return keys[sel], values[sel], counts[sel]

    # the exchange (exchange_and_reduce)
    def partition(self, nparts, ptr=None, cap=0):
        return self.ctx.partition(nparts, ptr, cap)

    def merge(self, ptr, n, sentinel=False):
        self.ctx.merge(ptr, n, 0, sentinel)
        self.n_entries = int(self.ctx.stats().n_slots)

    def merge_check(self):
        return self.ctx.merge_check()

    def partition_sums(self, nparts):
        return self.ctx.partition_sums(nparts)

    def rows_checksum(self, d_rows, seg_off):
        return self.ctx.rows_checksum(d_rows, seg_off)

    def route_rows_checksum(self, d_rows, seg_off):
        return self.ctx.route_rows_checksum(d_rows, seg_off)

    # the routed exchange (exchange_routed): stage A held for the owners
    def route_stage_a(self, flags, extra, rc0, nparts):
        return self.ctx.route_stage_a(flags, int(extra), bool(rc0), int(nparts))

    def route_scatter(self, nparts, ptr, cap):
        return self.ctx.route_scatter(nparts, ptr, cap)

    def route_finish(self):
        st = self.ctx.route_finish()
        self.n_entries = int(st.n_slots)
        return st

    def route_merge(self, ptr, n, nparts, sentinel=False):
        st = self.ctx.route_merge(ptr, n, nparts, sentinel)
        self.n_entries = int(st.n_slots)
        return st

    def stats(self):
        return self.ctx.stats()

    def stream_wait(self, stream_handle):
        self.ctx.stream_wait(stream_handle)

    def route_merge_segs(self, segs, nparts, sentinel=False):
        st = self.ctx.route_merge_segs(segs, nparts, sentinel)
        self.n_entries = int(st.n_slots)
        return st

    def build_rdbg(self):
        return self.ctx.build_rdbg()

    def owner_rdbg(self):
        return self.ctx.rdbg()

    def members(self, keys, n_records, rc0):
        self.ctx.dbg_load(keys, None, None)
        self.ctx.build_dbg(np.zeros(n_records, np.uint8), 0, bool(rc0))
        self.ctx.build_rdbg()

    def edges(self, flags, rc1):
        return self.ctx.edges(flags, bool(rc1))

    def rows_text(self, labels, flags, rc1, names):
        self.ctx.set_labels(*labels)
        self.ctx.rows_count(flags, bool(rc1))
        return self.ctx.rows_text(names)

    def dump_global(self, keys, masks, counts, k, device):
        from ._lib import Context
        d = Context(k, device)
        try:
            d.set_fasta(np.zeros(0, np.uint8))
            d.parse()
            d.dbg_load(keys, masks, counts)
            d.build_dbg(np.zeros(0, np.uint8), 0, True)
            return d.dbg_dump()
        finally:
            d.close()


# ------------------------------------------------------------------ pipeline
class DistRun:
    """The CLI stages of entry_point (:2073-2146) over world shards."""

    def __init__(self, qry: str, k: int, shard, comm: Comm, device=None, out=None, dev_index: int = 0,
                 edge_chunk: int = host.CHUNK, dbg_chunk: int = host.CHUNK, stream_bases: int = STREAM_BASES,
                 compact_at=None):
        self.qry, self.k, self.sh, self.comm = qry, min(max(1, int(k)), 27), shard, comm
        self.stream_bases = int(stream_bases)              # a shard above this streams its exchange
        self.compact_at = None if compact_at is None else int(compact_at)
        self.streamed = None
        self.edge_chunk = int(edge_chunk)                  # seq2graph's checkpoint size (:2073; tests vary it)
        self.dbg_chunk = int(dbg_chunk)                    # seq2rdbg's
        self.device, self.dev_index = device, dev_index
        self.rank, self.world = comm.rank, comm.world
        self.out = out or sys.stdout
        from .kmer import populate, seq2bytes
        self.buf = seq2bytes(qry, populate=False)        # (the shard's bytes are populated once it is known)
        self.bounds = shard_bounds(self.buf, self.world)
        lo, hi = self.bounds[self.rank], self.bounds[self.rank + 1]
        populate(self.buf, lo, hi)
        self.data = np.ascontiguousarray(self.buf[lo:hi])
        meta = self.sh.load(self.data)
        metas = comm.allgather_obj({k_: np.asarray(v, np.int64) for k_, v in meta.items()})
        self.S = Shards(metas, self.bounds, len(self.buf))
        self.R_local = self.S.R[self.rank]
        self.shape = host.FileShape.from_bytes(self.buf, self.S.hdr_start, self.S.hdr_len)

    def say(self, *a):
        if self.rank == 0:
            print(*a, file=self.out)

    def names(self):
        hs, hl = self.S.local(self.S.hdr_start, self.rank), self.S.local(self.S.hdr_len, self.rank)
        lo = self.bounds[self.rank]
        return [bytes(self.data[int(s) - lo + 1:int(s) - lo + int(n)]) for s, n in zip(hs, hl)]

    # ---------------------------------------------------------------- dBG
    def build_dbg(self, Ns, rc0, brkpt=""):
        """seq2rdbg (:1234-1268) over the shards; -r stages the checkpoint on rank 0."""
        resume, staged = None, None
        if brkpt and os.path.isfile(brkpt):
            offset, keys, values, counts = host.read_db_npz(brkpt)
            if self.rank == 0:
                staged = (keys, values, counts)
                self.sh.stage(*staged)
            resume = host.resume_position(offset, self.S.ptr)
        flags, extra, ckpt = host.plan_dbg(self.S.seq_len, self.shape, bool(rc0), int(Ns), self.dbg_chunk,
                                           resume=resume, checkpoint=True)
        # stream the exchange when the largest shard's planned bases exceed
        # stream_bases (the same decision on every rank: global record table)
        stream = self._max_local_bases(flags) > self.stream_bases
        if ckpt is not None:
            # <in>_db_brkpt.npz (:1255-1259): the last dump's state, built and dumped once
            cf, ce, last = ckpt
            if stream:
                parts = []
                chunks = stream_chunks(self.S.local(cf, self.rank), self.S.local(self.S.seq_len, self.rank),
                                       self.stream_bases)
                self._chunked_builds(chunks, ce if self.rank == 0 else 0, rc0, staged, parts)
                self.dump(self.qry + "_db_brkpt", offset=int(self.S.ptr[last]), parts=parts)
            else:
                self.sh.build(self.S.local(cf, self.rank), ce if self.rank == 0 else 0, rc0)
                self.dump(self.qry + "_db_brkpt", offset=int(self.S.ptr[last]))
        if stream:
            # C5 form: chunked local builds, one all-to-all per chunk into the
            # owner's record log; the counts of each chunk gathered for the dump
            self.stream_parts = []
            chunks = stream_chunks(self.S.local(flags, self.rank), self.S.local(self.S.seq_len, self.rank),
                                   self.stream_bases)
            grab = lambda: self._grab_counts(self.stream_parts)
            self.streamed = exchange_stream(self.sh, self.world, self.rank, self.device, chunks, self.R_local, rc0,
                                            extra if self.rank == 0 else 0, staged, self.comm.group, grab,
                                            self.compact_at)
            return
        self.sentinel = self.sh.build(self.S.local(flags, self.rank), extra if self.rank == 0 else 0, rc0)
        # the rdBG's exchange re-runs this pass's stage A held for its owners
        # (exchange_routed) - unless this is a -r resume, whose checkpoint
        # slots rank 0 staged into the build above only (the same decision
        # on every rank: `resume` is global, `staged` is rank 0's)
        self.route_plan = (self.S.local(flags, self.rank), extra if self.rank == 0 else 0, rc0) \
            if not (brkpt and os.path.isfile(brkpt)) else None

    def _max_local_bases(self, flags) -> int:
        sl = self.S.seq_len * np.asarray(flags, np.int64)
        return max(int(self.S.local(sl, r).sum()) for r in range(self.world)) if self.world else 0

    def _grab_counts(self, parts: list):
        """This build's occurrence counts, gathered to rank 0 (appended to
        parts) as 11 bytes per entry (key, 12-bit mask as uint16, saturated
        count as uint8).  rank 0 builds the `<in>_db.npz` table from all of
        them on its one GPU and in its host memory (the reference's own dump
        holds 11 B per oakht slot, :251-259), so the gathered entries are
        capped at DUMP_MAX_ENTRIES: past it the dump fails with a clear error
        instead of exhausting rank 0 (C5's ~2.2e10 keys would need ~320 GB of
        slot arrays)."""
        import torch
        keys, masks, counts = self.sh.counts()
        _, dev = _comm_device(self.device, self.comm.group)
        n = torch.tensor([keys.shape[0]], dtype=torch.int64, device=dev)
        self.comm.dist.all_reduce(n, op=self.comm.dist.ReduceOp.SUM, group=self.comm.group)
        self._dump_entries = getattr(self, "_dump_entries", 0) + int(n.item())
        if self._dump_entries > DUMP_MAX_ENTRIES:
            raise RuntimeError("<in>_db.npz: %d oakht entries gathered so far exceed the single-rank dump's budget "
                               "of %d (DUMP_MAX_ENTRIES): the dump of an input this size does not fit one rank"
                               % (self._dump_entries, DUMP_MAX_ENTRIES))
        got = self.comm.gather_bytes(_pack(keys.astype(np.uint64), masks.astype(np.uint16),
                                           np.minimum(counts, 255).astype(np.uint8)))
        if self.rank == 0:
            parts.extend(got)

    def _chunked_builds(self, chunks, extra, rc0, staged, parts):
        """Local builds of the chunks (same round count on every rank), counts
        gathered after each: the dump of a streamed checkpoint."""
        import torch
        _, dev = _comm_device(self.device, self.comm.group)
        n = torch.tensor([len(chunks)], dtype=torch.int64, device=dev)
        self.comm.dist.all_reduce(n, op=self.comm.dist.ReduceOp.MAX, group=self.comm.group)
        for i in range(max(1, int(n.item()))):
            if staged is not None and i < 2:
                self.sh.stage(*staged) if i == 0 else self.sh.stage(np.zeros(0, np.uint64))
            f = chunks[i] if i < len(chunks) else np.zeros(self.R_local, np.uint8)
            self.sh.build(f, extra if i == 0 else 0, rc0)
            self._grab_counts(parts)

    def load_dbg(self, fn, rdbg: bool, rc0):
        """load_on_disk (:289-335) of a -d / -D file: staged on rank 0 (-d: the
        exchange sends every entry to its owner) or, for -D, on every rank as
        the membership table itself."""
        _, keys, values, counts = host.read_db_npz(fn)
        zeros = np.zeros(self.R_local, np.uint8)
        if rdbg:
            self.sh.members(keys, self.R_local, rc0)
            self.reduced = True
            return
        if self.rank == 0:
            self.sh.stage(keys, values, counts)
        self.sentinel = self.sh.build(zeros, 0, rc0)

    def dump(self, fn, offset: int = 0, parts=None):
        """dump() (:243-261) of the global dBG, written by rank 0 (a streamed
        build: from the counts gathered chunk by chunk)."""
        if parts is None and self.streamed is not None:
            parts = self.stream_parts
        if parts is None:
            parts = []
            self._grab_counts(parts)
        if self.rank == 0:
            ks, ms, cs = [], [], []
            for p in parts:
                k_, m_, c_ = _unpack(p, (np.uint64, np.uint16, np.uint8))
                ks.append(k_); ms.append(m_); cs.append(c_)
            cap, size, K, V, C = self.sh.dump_global(np.concatenate(ks), np.concatenate(ms),
                                                     np.concatenate(cs), self.k, self.dev_index)
            host.write_db_npz(fn, cap, size, K, V, C, offset=offset)
        self.comm.barrier()

    # --------------------------------------------------------------- rdBG
    def reduce(self, rc0):
        """dbg2rdbg (:1313-1321): owner exchange, then every rank's walk
        membership = the union of the owners' rdBG keys."""
        if getattr(self, "reduced", False):
            return
        if self.streamed is not None:
            n_dbg, n_rdbg = self.streamed[:2]
            own = self.streamed[5]                          # (the sub-logs' rdBG keys)
        else:
            plan = getattr(self, "route_plan", None)
            if plan is not None:
                # the routed owner exchange (as the bench's N>1 step): the
                # local table above served the dump's occurrence counts only
                n_dbg, n_rdbg, _, _ = exchange_routed(self.sh, self.world, self.rank, self.device, plan[0], plan[1],
                                                      plan[2], self.comm.group)
            else:
                # -d (the npz slots staged on rank 0) or a -r resume: the
                # local table holds what no stage A can rebuild
                n_dbg, n_rdbg, _, _ = exchange_and_reduce(self.sh, self.world, self.rank, self.device, self.sentinel,
                                                          self.comm.group)
            own = np.ascontiguousarray(self.sh.owner_rdbg(), dtype=np.uint64)
        allk = np.sort(np.concatenate([p.view(np.uint64) for p in self.comm.allgather_bytes(own.view(np.uint8))]))
        if allk.shape[0] != n_rdbg:
            raise RuntimeError("rdBG all-gather: %d keys, owners reported %d" % (allk.shape[0], n_rdbg))
        self.n_dbg, self.n_rdbg = n_dbg, n_rdbg
        self.sh.members(allk, self.R_local, rc0)
        self.reduced = True

    # -------------------------------------------------------------- graph
    def graph(self, Ns, rc1, brkpt="", cluster=True):
        """seq2graph (:1853-1951) over the shards."""
        loaded, resume = None, None
        if brkpt and os.path.isfile(brkpt):
            offset, lt, lc = host.read_edge_npz(brkpt)
            loaded, resume = (lt, lc), host.resume_position(offset, self.S.ptr)
        eflags, segment, ncp, ckpt = host.plan_edges(self.S.seq_len, self.shape, int(Ns), self.edge_chunk,
                                                     resume=resume, checkpoint=True)

        def state(fl, upto):
            """the edge Dict after segments 0..upto on rank 0 (iteration order)"""
            t, c, w = self.sh.edges(self.S.local(fl, self.rank), rc1)
            w = np.asarray(w, np.int64) + 2 * int(self.S.off[self.rank])
            parts = self.comm.gather_bytes(_pack(np.ascontiguousarray(t, np.uint64), np.asarray(c, np.int64), w))
            if self.rank != 0:
                return None, None
            tuples, counts, walk = reduce_edges([_unpack(p, (np.uint64, np.int64, np.int64)) for p in parts])
            if loaded is not None:
                return host.merge_edges(loaded[0], loaded[1], tuples, counts, walk, segment, upto)
            o = host.edge_order(walk, segment, upto)
            return tuples[o], counts[o]
        if ckpt is not None:
            # <in>_rdb_brkpt.npz (:1880-1887): the Dict before the last checkpoint
            t_c, c_c = state((eflags.astype(bool) & (segment <= ncp - 1)).astype(np.uint8), ncp - 1)
            if self.rank == 0:
                host.write_edge_npz(self.qry + "_rdb_brkpt", t_c, c_c, int(self.S.ptr[ckpt]))
        tuples, counts = state(eflags, ncp)
        oname = self.qry + "_rdbg_weight.xyz"
        payload = np.zeros(0, np.uint8)
        if self.rank == 0:
            from ._lib import format_xyz
            with open(oname, "wb") as f:                       # :1893-1904
                f.write(format_xyz(tuples, counts))
            if cluster:
                if os.path.isfile("%s.mcl" % oname):
                    self.say("# the mcl has been ran")
                else:
                    self.out.flush()
                    os.system("mcl %s --abc -I 1.5 -te 8 -o %s.mcl -q x -V all" % (oname, oname))
            with open(oname + ".mcl", "r") as f:
                mcl_text = f.read()
            keys, vals, ids = host.label_table(mcl_text, tuples)      # :1918-1944
            payload = _pack(keys, vals, ids)
        keys, vals, ids = _unpack(self.comm.bcast_bytes(payload), (np.int64, np.int64, np.int64))
        rflags = host.plan_rows(self.S.seq_len, self.shape, self.buf, int(Ns))
        text = self.sh.rows_text((keys, vals, ids), self.S.local(rflags, self.rank), rc1, self.names())
        parts = self.comm.gather_bytes(np.frombuffer(text, np.uint8) if text else np.zeros(0, np.uint8))
        if self.rank == 0:
            body = b"".join(p.tobytes() for p in parts)
            if body:
                if hasattr(self.out, "buffer"):
                    self.out.flush()
                    self.out.buffer.write(body)
                    self.out.buffer.flush()
                else:
                    self.out.write(body.decode())
        self.comm.barrier()


def reduce_edges(parts):
    """Edge lists of the ranks (each in its own first-occurrence order, ranks
    in record order) -> one list in global first-occurrence order: walk counts
    add, the first occurrence's walk index is kept (rdbg_edge_weight :1476-1484
    per walk, the typed Dict's insertion order across walks)."""
    t = np.concatenate([p[0].reshape(-1, 4) for p in parts]) if parts else np.zeros((0, 4), np.uint64)
    c = np.concatenate([p[1] for p in parts]) if parts else np.zeros(0, np.int64)
    w = np.concatenate([p[2] for p in parts]) if parts else np.zeros(0, np.int64)
    if t.shape[0] == 0:
        return t, c, w
    v = np.ascontiguousarray(t).view(np.dtype((np.void, 32))).ravel()
    _, first, inv = np.unique(v, return_index=True, return_inverse=True)
    tot = np.zeros(first.shape[0], np.int64)
    np.add.at(tot, inv.ravel(), c)
    o = np.argsort(first, kind="stable")
    return t[first[o]], tot[o], w[first[o]]


def entry_point(argv, out=None, shard_factory=None, device=None, dev_index: int = 0, edge_chunk: int = host.CHUNK,
                dbg_chunk: int = host.CHUNK, stream_bases: int = STREAM_BASES, compact_at=None):
    """kmer.entry_point (:1971-2146) on every rank of an initialised process
    group; rank 0 prints.  `shard_factory(k)` makes the rank's backend
    (default: GpuShard on dev_index)."""
    import torch.distributed as dist
    from .kmer import manual_print, parse_args
    out = out or sys.stdout
    args = parse_args(argv)
    qry, kmer, Ns = args["-i"], int(args["-k"]), host.eval_number(args["-n"])
    bkt, dbs, rbk, rc, rdb = args["-r"], args["-d"], args["-R"], int(args["-c"]), args["-D"]
    if not qry:
        if dist.get_rank() == 0:
            manual_print(out)
        raise SystemExit()
    rc0, rc1 = (rc >> 1) == 1, (rc & 1) == 1
    k = min(max(1, kmer), 27)
    shard = shard_factory(k) if shard_factory else GpuShard(k, dev_index)
    comm = Comm(device)
    run = DistRun(qry, k, shard, comm, device=device, out=out, dev_index=dev_index, edge_chunk=edge_chunk,
                  dbg_chunk=dbg_chunk, stream_bases=stream_bases, compact_at=compact_at)
    if dbs or rdb:                                      # :2073-2101
        if not rdb:
            run.say("load dBG from disk")
            run.load_dbg(dbs, False, rc0)
            run.say("# build the reduced dBG")
            run.reduce(rc0)
        else:
            run.load_dbg(rdb, True, rc0)
        run.say("# find fr")
        run.graph(Ns, rc1, brkpt=rbk)
        return 0
    run.say("# build the dBG")
    st = time()
    run.build_dbg(Ns, rc0, brkpt=bkt)
    run.say("# finished in", time() - st, "seconds")
    run.say("# save dBG to disk")
    st = time()
    run.dump(qry + "_db")
    run.say("# finished in", time() - st, "seconds")
    run.say("# load dBG from disk")
    st = time()
    run.say("# finished in", time() - st, "seconds")
    run.say("# build the reduced dBG")
    st = time()
    run.reduce(rc0)
    run.say("# finished in", time() - st, "seconds")
    run.say("# find fr")
    st = time()
    run.graph(Ns, rc1, brkpt=rbk)
    run.say("# finished in", time() - st, "seconds")
    return 0


def main():
    """`python -m torch.distributed.run --nproc-per-node N -m pangenome_amd -i in.fa -k 27`:
    one rank per GPU over RCCL.  PG_DIST_BACKEND=gloo with PG_DIST_ONE_GPU=1
    puts every rank on cuda:0 (tests on a one-GPU box)."""
    import torch
    import torch.distributed as dist
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("PG_DIST_BACKEND", "nccl")
    dev_index = 0 if os.environ.get("PG_DIST_ONE_GPU") == "1" else local
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    torch.cuda.set_device(dev_index)
    device = torch.device("cuda", dev_index)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=device)
    else:
        dist.init_process_group(backend)
    try:
        return entry_point(sys.argv, device=device, dev_index=dev_index,
                           stream_bases=int(os.environ.get("PG_DIST_STREAM_BASES", STREAM_BASES)))
    finally:
        dist.destroy_process_group()

"""Multi-GPU dBG -> rdBG: one process per GPU, input sharded by record.

Every rank builds the OR-table of its own records (K1 + K3), owner-partitions
its entries (16-byte records: key+1, the 26-bit mask word of both
orientations) and sends each run to its owner with one all-to-all (RCCL over
xGMI; gloo in the CPU tests).  Owners OR-merge what they receive into a fresh
table and run the degree scan (K5) on their partition only.  A k-mer's mask
needs every occurrence, so this exchange is the path's one real collective;
RCCL has no bitwise-OR reduction and slot layouts differ per GPU, so an
all-reduce of "the count table" would not be exact — the all-to-all is
(SURVEY.md §8e).

The orchestration takes a `table` object (the GPU Context, or a CPU stand-in
in tests) with: partition(nparts) -> counts, partition(nparts, ptr, cap),
merge(ptr, n, sentinel=...), build_rdbg() -> stats (n_dbg, n_rdbg).
"""
from __future__ import annotations

import numpy as np


def _is_cuda(device) -> bool:
    return getattr(device, "type", str(device)).startswith("cuda")


def exchange_and_reduce(table, world: int, rank: int, device, sentinel_local: bool, group=None):
    """Returns (n_dbg_total, n_rdbg_total, n_rdbg_local, bytes_sent)."""
    import torch
    import torch.distributed as dist

    # gloo moves host tensors only: stage device buffers through host memory
    stage = _is_cuda(device) and dist.get_backend(group) == "gloo"
    comm = torch.device("cpu") if stage else device

    counts = table.partition(world)
    total = int(counts.sum())
    send = torch.empty((max(total, 1), 2), dtype=torch.int64, device=device)
    if total:
        table.partition(world, send.data_ptr(), total)
    send_counts = torch.tensor(counts.astype(np.int64), dtype=torch.int64, device=comm)
    recv_counts = torch.empty_like(send_counts)
    dist.all_to_all_single(recv_counts, send_counts, group=group)
    rsplit = recv_counts.cpu().tolist()
    nrecv = int(sum(rsplit))
    recv = torch.empty((max(nrecv, 1), 2), dtype=torch.int64, device=comm)
    dist.all_to_all_single(recv[:nrecv], (send.cpu() if stage else send)[:total], output_split_sizes=rsplit,
                           input_split_sizes=counts.astype(np.int64).tolist(), group=group)
    if stage:
        recv = recv.to(device)
    flag = torch.tensor([1 if sentinel_local else 0], dtype=torch.int64, device=comm)
    dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
    if _is_cuda(device):
        torch.cuda.synchronize(device)
    # the n<k sentinel key belongs to one owner: rank 0
    table.merge(recv.data_ptr(), nrecv, sentinel=bool(flag.item()) and rank == 0)
    st = table.build_rdbg()
    sums = torch.tensor([st.n_dbg, st.n_rdbg], dtype=torch.int64, device=comm)
    dist.all_reduce(sums, op=dist.ReduceOp.SUM, group=group)
    return int(sums[0].item()), int(sums[1].item()), int(st.n_rdbg), 16 * (total - int(counts[rank]))

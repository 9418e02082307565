"""Stream order between torch and the library (the cause of round 4's wrong
C5 counts).

The library runs on its own non-blocking HIP streams.  torch's caching
allocator hands a freed block to the next torch.empty on the same stream at
once, even while work queued on that stream (a clone, a wait on an RCCL
all-to-all) still reads it: stream order makes that safe for torch's own
kernels, not for a library kernel on another stream.  exchange_stream freed
each round's receive buffer right after queueing the copies of its sub-log
runs, and the next round's pg_dbg_partition scattered into a torch.empty of
the same size - the same block - without waiting.  With a 16 GB round sent to
self through RCCL (world 1, 512 MiB pieces) still in flight behind the next
chunk's build, the scatter overwrote records the all-to-all and the copies had
yet to move.  dist._fence (torch.cuda.synchronize before every native read or
write of torch memory) closed it; round 6's form is stream-ordered instead:
the library's streams wait on an event of torch's current stream
(pg_stream_wait), so the host never blocks for it.

The test reproduces the hazard deterministically: a long kernel keeps torch's
stream busy, a copy of a tensor is queued behind it, the tensor is freed and
its block handed to a new tensor the library scatters into.  Unfenced, the
copy reads the library's records; fenced, the original values.
"""
import os
import sys

import numpy as np
import pytest

from dist_util import ROOT

pytestmark = pytest.mark.gpu


def _table(ctx):
    from pangenome_amd import synth
    fa = synth.pangenome(4, 200_000, snp=0.01, indel=1e-3, seed=5)
    ctx.set_fasta(np.frombuffer(fa, np.uint8))
    ctx.parse()
    ctx.build_dbg(None, 0, True)
    return int(ctx.partition(1)[0])


@pytest.mark.timeout(300)
@pytest.mark.parametrize("fence", ["none", "sync", "event"])
def test_native_write_into_reused_torch_block(fence):
    """fence "sync": a device-wide synchronize; "event": the product form,
    the library's streams wait on an event of torch's current stream
    (pg_stream_wait), the host does not block."""
    fenced = fence != "none"
    sys.path.insert(0, ROOT)
    import torch
    from pangenome_amd import dist as pdist
    from pangenome_amd._lib import Context
    dev = torch.device("cuda", 0)
    ctx = Context(27, 0)
    try:
        n = _table(ctx)
        torch.cuda.synchronize()
        x = torch.full((n, 2), 7, dtype=torch.int64, device=dev)
        torch.cuda.synchronize()
        torch.cuda._sleep(200_000_000)                # torch's stream busy for ~0.1 s
        y = x.clone()                                  # queued behind it: reads x's block later
        ptr = x.data_ptr()
        del x                                          # the block is free for the current stream at once
        send = torch.empty((n, 2), dtype=torch.int64, device=dev)
        if send.data_ptr() != ptr:
            pytest.skip("the allocator did not hand out the freed block")
        if fence == "sync":
            pdist._fence(dev)
        elif fence == "event":
            pdist._fence(dev, ctx)
        ctx.partition(1, send.data_ptr(), n)           # the library's scatter, on its own stream
        torch.cuda.synchronize()
        intact = bool(torch.all(y == 7).item())
        print("fenced=%s: the queued copy read %s" % (fenced, "the original values" if intact else
                                                       "the library's records (overwritten)"))
        if fenced:
            assert intact
        else:
            assert not intact, "expected the unfenced scatter to overwrite the block before the copy read it"
        # the exchange's own path fences: a whole _route of this table is exact
        assert pdist.row_check_sum(send.cpu().numpy()) == int(ctx.partition_sums(1)[0])
    finally:
        ctx.close()

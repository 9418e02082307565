"""The multi-GPU path's kernels (pg_dbg_partition / pg_dbg_merge / K5 on the
owner partition) with 2 ranks sharing one MI355X; the collective is gloo with
host staging (RCCL needs one GPU per rank; the bench uses it).  The union of
the owners' rdBG keys must equal the single-process build exactly."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world, port, shard, q):
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from pangenome_amd._lib import Context
    from pangenome_amd.dist import exchange_and_reduce
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    ctx = Context(27, 0)
    ctx.set_fasta(shard)
    ctx.parse()
    st = ctx.build_dbg(None, 0, True)
    res = exchange_and_reduce(ctx, world, rank, dev, bool(st.sentinel))
    q.put((rank, res, ctx.rdbg()))
    dist.destroy_process_group()


def test_two_rank_exchange_on_one_gpu():
    from pangenome_amd import synth
    from pangenome_amd._lib import Context
    fasta = synth.pangenome(8, 200_000, snp=0.005, indel=5e-4, seed=99)
    recs = [b">" + r for r in fasta.split(b">")[1:]]
    shards = [b"".join(recs[0::2]), b"".join(recs[1::2]) + b">short\nACGTA\n"]
    whole = shards[0] + shards[1]
    ctx = Context(27, 0)
    ctx.set_fasta(whole)
    ctx.parse()
    ctx.build_dbg(None, 0, True)
    st = ctx.build_rdbg()
    ref_keys = ctx.rdbg()
    ctx.close()

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mpc = mp.get_context("spawn")
    q = mpc.Queue()
    procs = [mpc.Process(target=_worker, args=(r, 2, port, shards[r], q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict((r, (res, keys)) for r, res, keys in (q.get(timeout=300) for _ in range(2)))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for r in range(2):
        n_dbg, n_rdbg, _, _ = out[r][0]
        assert n_dbg == st.n_dbg and n_rdbg == st.n_rdbg
    union = np.sort(np.concatenate([out[0][1], out[1][1]]))
    assert np.array_equal(union, ref_keys)

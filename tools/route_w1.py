#!/usr/bin/env python3
"""Development timing (not part of the product): the routed exchange forced
through its N>1 path at world 1 on the C3 batch (HBM-resident input), phase
by phase (dist.exchange_routed's tm), beside pg_route_finish; run it under
rocprofv3 --kernel-trace for the kernels.

    python tools/route_w1.py [reps]
"""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    import numpy as np
    import torch
    import torch.distributed as dist
    from pangenome_amd import _lib, kmer, synth
    from pangenome_amd.dist import exchange_routed
    tmp = tempfile.mkdtemp(prefix="route_w1_")
    p = os.path.join(tmp, "c3a.fa")
    synth.write_pangenome(p, 100, 5_000_000, first_index=0, workers=16)
    d = torch.from_numpy(np.array(kmer.seq2bytes(p))).to("cuda:0")
    os.unlink(p)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:29633", rank=0, world_size=1, device_id=dev)
    ctx = _lib.Context(27, 0)
    tm, fin = {}, []
    for i in range(reps + 1):
        ctx.set_fasta_device(d.data_ptr(), d.numel(), keepalive=d)
        ctx.parse()
        res = exchange_routed(ctx, 1, 0, dev, None, 0, True, tm=tm if i else None, force=True)
        ctx.set_fasta_device(d.data_ptr(), d.numel(), keepalive=d)
        ctx.parse()
        ctx.route_stage_a(None, 0, True, 1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st = ctx.route_finish()
        torch.cuda.synchronize()
        if i:
            fin.append(time.perf_counter() - t0)
    rows = tm.pop("rows", 0) / reps
    out = {k: round(1e3 * v / reps, 3) for k, v in tm.items()}
    out.update(local_finish=round(1e3 * sum(fin) / reps, 3), rows=int(rows), counts=res[:2],
               finish_counts=(st.n_dbg, st.n_rdbg))
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

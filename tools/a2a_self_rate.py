#!/usr/bin/env python3
"""Development measurement (not part of the product): how long a world-1
all-to-all of one C5 round's records to self takes over RCCL in 512 MiB
pieces (dist._all_to_all_rows, self_copy=False) against a device copy, and
against the build that round 4's exchange_stream queued right behind it.
The RCCL form still running when the next chunk's partition reused the
receive buffer's block is the race DESIGN.md §6 describes."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist
    from pangenome_amd import dist as pdist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29655")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    for rows in (1 << 25, 1 << 28, 937_000_000):        # 512 MiB, 4 GiB, one C5 round's sub-log share x 4
        send = torch.randint(0, 1 << 62, (rows, 2), dtype=torch.int64, device=dev)
        recv = torch.empty_like(send)
        out = {"rows": rows, "gb": round(16 * rows / 1e9, 2)}
        for form, sc in (("rccl", False), ("copy", True)):
            for rep in range(2):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                pdist._all_to_all_rows(recv, send, [rows], [rows], dev, self_copy=sc)
                t_host = time.perf_counter() - t0          # the call returns once it is queued
                torch.cuda.synchronize()
                t = time.perf_counter() - t0
            out[form + "_ms"] = round(1e3 * t, 2)
            out[form + "_host_return_ms"] = round(1e3 * t_host, 2)
            out[form + "_gbs"] = round(16 * rows / t / 1e9, 1)
            out[form + "_exact"] = bool(torch.equal(recv, send))
            recv.zero_()
        print(json.dumps(out), flush=True)
        del send, recv
        torch.cuda.empty_cache()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""Development: does all_to_all_single over RCCL (world 1) return what was
sent, at growing message sizes?  python tools/rccl_a2a_check.py"""
import os

import torch
import torch.distributed as dist

os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ.get("MASTER_PORT", "29541"))
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
for rows in (1 << 20, 1 << 24, 1 << 26, 100_000_000, 125_000_000, 1 << 27):
    send = torch.arange(2 * rows, dtype=torch.int64, device=dev).view(rows, 2)
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, output_split_sizes=[rows], input_split_sizes=[rows])
    torch.cuda.synchronize()
    ok = bool(torch.equal(recv, send))
    bad = int((recv != send).any(dim=1).sum())
    recv2 = torch.empty_like(send)
    dist.all_to_all(list(recv2.split(rows)), list(send.split(rows)))
    torch.cuda.synchronize()
    print("rows %d bytes %.2f GB: all_to_all_single ok=%s (bad rows %d), all_to_all(list) ok=%s"
          % (rows, 16 * rows / 1e9, ok, bad, bool(torch.equal(recv2, send))), flush=True)
    del send, recv, recv2
dist.destroy_process_group()

"""The owner all-to-all's piecewise form (dist._all_to_all_rows) over RCCL.

RCCL 2.26.6 (ROCm 7 torch wheels) delivers only the first half of a
point-to-point message larger than 2^30 bytes: at world 1 an all_to_all of
2^30 + 4096 bytes to self comes back with every byte from offset ~2^29 on
wrong, for int64 and uint8 elements alike (a byte limit, not an element
count), for all_to_all_single and all_to_all(list) alike, while a device copy
of the same size is exact (tools/corruption_bracket.py,
profiles/r04_rccl_bracket.jsonl).  dist.A2A_ROWS (2^25 rows of 16 bytes =
512 MiB per peer and collective) keeps every message at half that limit.
This sends just over A2A_ROWS rows per peer, and a 1.34 GB message (past the
limit) through _all_to_all_rows, and checks every row; whether one
all_to_all_single of the big message is exact on this RCCL is printed.
"""
import os
import sys

import pytest

from dist_util import ROOT, spawn_ranks

pytestmark = pytest.mark.gpu


def _rank(rank, world, port, q):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from pangenome_amd import dist as pdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    out = {}
    for tag, rows in (("just_over", pdist.A2A_ROWS + 4096), ("past_limit", (1 << 26) + (1 << 24))):
        send = torch.arange(2 * rows, dtype=torch.int64, device=dev).view(rows, 2)
        send.mul_(-7046029254386353131).add_(12345)
        recv = torch.empty((rows, 2), dtype=torch.int64, device=dev)
        pdist._all_to_all_rows(recv, send, [rows], [rows], dev, self_copy=False)   # through RCCL
        torch.cuda.synchronize()
        out[tag] = bool(torch.equal(recv, send))
        recv.zero_()
        pdist._all_to_all_rows(recv, send, [rows], [rows], dev)                    # the product path: a copy
        torch.cuda.synchronize()
        out[tag + "_copy"] = bool(torch.equal(recv, send))
        if tag == "past_limit":
            recv.zero_()
            dist.all_to_all_single(recv, send, output_split_sizes=[rows], input_split_sizes=[rows])
            torch.cuda.synchronize()
            out["single_call_exact"] = bool(torch.equal(recv, send))
        del send, recv
        torch.cuda.empty_cache()
    q.put((rank, out))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_all_to_all_rows_pieces_over_rccl():
    out = spawn_ranks(1, _rank, (), timeout=240)[0]
    print("rccl all_to_all: %s" % out)
    assert out["just_over"] and out["past_limit"] and out["just_over_copy"] and out["past_limit_copy"]

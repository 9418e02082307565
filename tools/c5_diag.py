"""Development: the C5-form streamed exchange at world 1 with the device memory
held by the library (pg_device_bytes) and by torch printed after every step.

    python tools/c5_diag.py FASTA [chunk_bases] [gloo|nccl] [whole]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist
    from pangenome_amd import dist as pdist
    from pangenome_amd import kmer
    from pangenome_amd._lib import load
    path = sys.argv[1]
    chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 125_000_000
    backend = sys.argv[3] if len(sys.argv) > 3 else "gloo"
    whole = len(sys.argv) > 4 and sys.argv[4] == "whole"
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ.get("MASTER_PORT", "29533"))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    else:
        dist.init_process_group("gloo", rank=0, world_size=1)
    lib = load()
    t00 = time.time()

    def mem(tag):
        free, total = torch.cuda.mem_get_info(dev)
        print("%7.1f s %-28s lib %6.1f GB (peak %6.1f)  torch alloc %6.1f reserved %6.1f  device free %6.1f / %6.1f GB"
              % (time.time() - t00, tag, lib.pg_device_bytes(0) / 1e9, lib.pg_device_bytes(1) / 1e9,
                 torch.cuda.memory_allocated(dev) / 1e9, torch.cuda.memory_reserved(dev) / 1e9, free / 1e9,
                 total / 1e9), flush=True)

    sh = pdist.GpuShard(27, 0)
    meta = sh.load(kmer.seq2bytes(path))
    R = int(meta["seq_len"].shape[0])
    mem("parsed %d records" % R)
    if whole:
        sh.ctx.build_dbg(np.ones(R, np.uint8), 0, True)
        st = sh.ctx.build_rdbg()
        mem("whole build n_dbg=%d" % st.n_dbg)
        keys, masks = sh.ctx.dbg()
        mem("dbg export %d" % keys.shape[0])
        del keys, masks
    chunks = pdist.stream_chunks(np.ones(R, np.uint8), meta["seq_len"], chunk)
    orig_build, orig_merge, orig_part = sh.build, sh.merge, sh.partition

    def build(*a):
        r = orig_build(*a)
        mem("chunk build")
        return r

    def perm_bins(key):
        M = np.uint64((1 << 63) - 1)
        m1 = np.uint64((0x9E3779B97F4A7C15 & ((1 << 63) - 1)) | 1)
        m2 = np.uint64((0xC2B2AE3D27D4EB4F & ((1 << 63) - 1)) | 1)
        with np.errstate(over="ignore"):
            h = (key * m1) & M
            h ^= h >> np.uint64(31)
            h = (h * m2) & M
            h ^= h >> np.uint64(21)
        return (h >> np.uint64(57)).astype(np.int64)

    import ctypes
    hiprt = ctypes.CDLL("libamdhip64.so")

    def inspect(tag, ptr, n):
        torch.cuda.synchronize()
        rec = np.empty((n, 2), np.uint64)
        hiprt.hipMemcpy(ctypes.c_void_p(rec.ctypes.data), ctypes.c_void_p(ptr), ctypes.c_size_t(16 * n), 2)
        key = rec[:, 0] - np.uint64(1)
        cnt = np.bincount(perm_bins(key), minlength=64)
        print("   %s: unique keys %d of %d, zero key1 %d, key max %d, bins max/mean %.2f, min/mean %.2f"
              % (tag, np.unique(rec[:, 0]).shape[0], n, int((rec[:, 0] == 0).sum()), int(key.max()),
                 cnt.max() / cnt.mean(), cnt.min() / cnt.mean()), flush=True)

    def merge(ptr, n, sentinel=False):
        mem("merge of %d records ..." % n)
        if n:
            inspect("merge input", ptr, n)
        orig_merge(ptr, n, sentinel)
        mem("merged")

    def partition(nparts, ptr=None, cap=0):
        r = orig_part(nparts, ptr, cap)
        if ptr is not None and int(r.sum()):
            inspect("partition(%d) output" % nparts, ptr, int(r.sum()))
        return r

    sh.build, sh.merge, sh.partition = build, merge, partition
    res = pdist.exchange_stream(sh, 1, 0, dev, chunks, R, True, compact_at=1)
    mem("done n_dbg=%d n_rdbg=%d rounds=%d" % (res[0], res[1], res[4]))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

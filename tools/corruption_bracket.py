"""Development: bracket round 3's two silent corruptions on one MI355X.

1. RCCL all_to_all to self (world 1): at which message size does the receive
   buffer differ from what was sent?  Tried for all_to_all_single and
   all_to_all(list), in int64 and uint8 elements (a byte limit and an element
   limit then fail at different sizes), against a plain device copy of the
   same size.  For a failing case the first differing byte offset and the
   number of differing bytes are printed.
2. The sub-log split round 3 removed from dist.exchange_stream:
   recv[torch.argsort(sub, stable=True)] with sub = a hash of the key word,
   on (n, 2) int64 rows, checked against numpy on the host.

3. torch.cat / clone of (n, 2) int64 row tensors past 2^31 elements (the
   streamed exchange's sub-log concatenation at C5 size).

    python tools/corruption_bracket.py a2a|sort|cat > out.jsonl
One JSON line per case on stdout.
"""
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

GiB = 1 << 30


def emit(**kw):
    print(json.dumps(kw), flush=True)


def fill(nbytes, dev):
    """A byte pattern where every 8-byte word is its own index (so a shifted or
    missing piece never matches by accident)."""
    w = (nbytes + 7) // 8
    t = torch.arange(w, dtype=torch.int64, device=dev)
    t.mul_(0x9E3779B97F4A7C15 - (1 << 64)).add_(12345)
    return t.view(torch.uint8)[:nbytes]


def diff(a, b):
    ne = a != b
    n = int(ne.sum())
    if not n:
        return 0, -1, -1
    u = ne.to(torch.uint8)
    first = int(torch.argmax(u))
    last = u.numel() - 1 - int(torch.argmax(torch.flip(u, (0,))))
    return n, first, last


def a2a_cases(dev):
    sizes = [GiB - 4096, GiB, GiB + 4096, GiB + GiB // 2, 2 * GiB - 4096, 2 * GiB, 2 * GiB + 4096, 3 * GiB]
    for nbytes in sizes:
        src = fill(nbytes, dev)
        for dt, es in (("int64", 8), ("uint8", 1)):
            n = nbytes // es
            s = src[:n * es].view(torch.int64 if dt == "int64" else torch.uint8)
            for op in ("all_to_all_single", "all_to_all_list", "copy"):
                r = torch.full_like(s, 0x5A if dt == "uint8" else 0x5A5A5A5A5A5A5A5A)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                if op == "all_to_all_single":
                    dist.all_to_all_single(r, s, output_split_sizes=[n], input_split_sizes=[n])
                elif op == "all_to_all_list":
                    dist.all_to_all([r], [s])
                else:
                    r.copy_(s)
                torch.cuda.synchronize()
                dt_s = time.perf_counter() - t0
                bad, first, last = diff(r.view(torch.uint8), s.view(torch.uint8))
                emit(case="a2a", op=op, dtype=dt, elements=n, bytes=n * es, ok=bad == 0, bad_bytes=bad,
                     first_bad_byte=first, last_bad_byte=last, ms=round(1e3 * dt_s, 2))
                del r
        del src
        torch.cuda.empty_cache()


def sort_case(dev, rows, nsub, op):
    """One (rows, nsub, op) case in this process: op = argsort (stable) and
    the gather t[idx], or index_select, each synchronised so that an error is
    attributed to its op."""
    golden = -7046029254386353131                     # 0x9E3779B97F4A7C15 as int64 (wrapping multiply)
    host = np.random.default_rng(rows).integers(0, 1 << 62, size=(rows, 2), dtype=np.int64)
    t = torch.from_numpy(host).to(dev)
    stage = "sub"
    res = dict(case="sort", rows=rows, bytes=16 * rows, nsub=nsub, op=op)
    try:
        sub = ((t[:, 0] * golden) >> 20) & (nsub - 1)
        torch.cuda.synchronize()
        stage = "argsort"
        idx = torch.argsort(sub, stable=True)
        torch.cuda.synchronize()
        stage = op
        out = t[idx] if op == "gather" else torch.index_select(t, 0, idx)
        torch.cuda.synchronize()
    except Exception as e:                            # noqa: BLE001 (a launch error is reported, not raised on)
        res.update(ok=False, error_stage=stage, error=str(e).splitlines()[0])
        emit(**res)
        return False
    with np.errstate(over="ignore"):
        hsub = ((host[:, 0] * np.int64(golden)) >> 20) & (nsub - 1)
    hidx = np.argsort(hsub, kind="stable")
    o = out.cpu().numpy()
    ne = np.flatnonzero((o != host[hidx]).any(axis=1))
    res.update(ok=ne.shape[0] == 0, sub_ok=bool(np.array_equal(sub.cpu().numpy(), hsub)),
               argsort_ok=bool(np.array_equal(idx.cpu().numpy(), hidx)), bad_rows=int(ne.shape[0]),
               first_bad_row=int(ne[0]) if ne.shape[0] else -1)
    emit(**res)
    return res["ok"]


def sort_cases(dev):
    """Ascending sizes, each case in a fresh process (a launch error ends that
    process only); stops at the first failing size."""
    import subprocess
    for rows in (1 << 20, 1 << 22, 1 << 24, (1 << 24) + 1, 1 << 25, (1 << 25) + (1 << 24), (1 << 26) - 1, 1 << 26):
        fails = 0
        for op in ("gather", "index_select"):
            r = subprocess.run([sys.executable, "-u", __file__, "sort1", str(rows), "4", op], timeout=120)
            fails += r.returncode != 0
        if fails:
            break


def same(a, b, piece=1 << 26):
    """a == b row for row, compared in pieces (no full-size temporaries)."""
    n = a.shape[0]
    for o in range(0, n, piece):
        if not torch.equal(a[o:o + piece], b[o:o + piece]):
            ne = (a[o:o + piece] != b[o:o + piece]).any(dim=1)
            return o + int(torch.argmax(ne.to(torch.uint8)))
    return -1


def cat_case(dev, rows_a, rows_b, op):
    res = dict(case="cat", op=op, rows=rows_a + rows_b, elements=2 * (rows_a + rows_b),
               bytes=16 * (rows_a + rows_b))
    try:
        a = fill(16 * rows_a, dev).view(torch.int64).view(-1, 2)
        if op == "cat":
            b = fill(16 * rows_b, dev).view(torch.int64).view(-1, 2).flip(0).contiguous()
            c = torch.cat([a, b])
            torch.cuda.synchronize()
            fa, fb = same(c[:rows_a], a), same(c[rows_a:], b)
            res.update(ok=fa < 0 and fb < 0, first_bad_row=fa if fa >= 0 else (rows_a + fb if fb >= 0 else -1))
        else:                                          # clone of a row slice (the sub-log pieces)
            c = a[1:].clone()
            torch.cuda.synchronize()
            f = same(c, a[1:])
            res.update(ok=f < 0, first_bad_row=f)
    except Exception as e:                            # noqa: BLE001
        res.update(ok=False, error=str(e).splitlines()[0])
    emit(**res)
    return res["ok"]


def cat_cases():
    import subprocess
    G = 1 << 30
    for rows in ((G // 2, G // 2 - 1), (G // 2, G // 2), (G // 2, G // 2 + 1), (G // 2 + G // 8, G // 2),
                 (G, G // 2)):
        for op in ("cat", "clone"):
            subprocess.run([sys.executable, "-u", __file__, "cat1", str(rows[0]), str(rows[1]), op], timeout=300)


def repeat_cases(dev, reps=64, rows=1 << 25):
    """The exchange's per-piece pattern at world 1: all_to_all(list) of one
    A2A_ROWS-row piece (512 MiB) to self, `reps` times from different
    offsets of one large buffer, each checked."""
    n = rows * 8
    src = fill(16 * n, dev).view(torch.int64).view(-1, 2)
    dst = torch.zeros_like(src)
    bad = []
    for r in range(reps):
        o = (r % 8) * rows
        dist.all_to_all([dst[o:o + rows]], [src[o:o + rows]])
        torch.cuda.synchronize()
        f = same(dst[o:o + rows], src[o:o + rows])
        if f >= 0:
            bad.append((r, f))
        dst[o:o + rows].zero_()
    emit(case="repeat", op="all_to_all_list", rows=rows, bytes=16 * rows, reps=reps, ok=not bad, bad=bad[:8],
         n_bad=len(bad))


def main():
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    if what == "sort1":
        torch.cuda.set_device(0)
        ok = sort_case(torch.device("cuda", 0), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4])
        sys.exit(0 if ok else 1)
    if what == "cat1":
        torch.cuda.set_device(0)
        ok = cat_case(torch.device("cuda", 0), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4])
        sys.exit(0 if ok else 1)
    if what == "cat":
        emit(case="env", torch=torch.__version__, hip=torch.version.hip)
        cat_cases()
        return
    if what == "sort":                                # (the parent never touches the GPU)
        emit(case="env", torch=torch.__version__, hip=torch.version.hip)
        sort_cases(None)
        return
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ.get("MASTER_PORT", "29547"))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    emit(case="env", torch=torch.__version__, hip=torch.version.hip,
         rccl=".".join(map(str, torch.cuda.nccl.version())), device=torch.cuda.get_device_name(0))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    if what == "repeat":
        repeat_cases(dev)
    else:
        a2a_cases(dev)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Run tests/test_gpu_c5.py::test_c5_shard_full_size_properties (the 3.75 Gbp
C5 shard one rank holds at N = 8: streamed exchange at 2^30 and 2^29 bases
per chunk over gloo and at 2^30 over RCCL; parity unpinned, property checks)
outside pytest, with a heartbeat line every 30 s so a long quiet phase is not
taken for a hang.  Output: its log lines (profiles/r03_c5_shard.log)."""
import os
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ["PG_RUN_C5_FULL"] = "1"


def main():
    import pathlib
    import test_gpu_c5
    t0 = time.time()
    done = threading.Event()

    def beat():
        while not done.wait(30):
            print("c5_full: %.0f s" % (time.time() - t0), flush=True)
    threading.Thread(target=beat, daemon=True).start()
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as d:
        try:
            test_gpu_c5.test_c5_shard_full_size_properties(pathlib.Path(d))
        finally:
            done.set()
    print("c5_full: properties hold, %.0f s" % (time.time() - t0), flush=True)


if __name__ == "__main__":
    main()

"""Host-only checks of the kernels' shared arithmetic (pg_common.h), compiled
with hipcc for the CPU: no GPU needed."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("hipcc") is None, reason="hipcc not on PATH")
def test_rc_and_perm_host(tmp_path):
    exe = tmp_path / "common_check"
    src = os.path.join(ROOT, "tests", "native", "common_check.cpp")
    subprocess.run(["hipcc", "-O2", "-std=c++17", src, "-o", str(exe)], check=True, capture_output=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "bad 0" in r.stdout

"""Host-side pack machinery of libtxvote.so (go-txflow_amd/csrc/host_pack.hpp), tested on the CPU
with sanitizers: the worker pool under ThreadSanitizer (back-to-back jobs, every index visited
once), the TxHash -> TxVoteSet id table (ids in first-seen order as txflow/service.go:200-209
creates sets, capacity limit) and the validator address table under Address/UB sanitizers."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "cpu_host", "host_pack_test.cpp")


@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_host_pack_sanitized(tmp_path, san):
    if not shutil.which("g++"):
        pytest.skip("g++ missing")
    exe = str(tmp_path / "t")
    subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-pthread", f"-fsanitize={san}", SRC, "-o", exe], check=True)
    r = subprocess.run([exe, "60"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout and "WARNING" not in r.stderr, r.stdout + r.stderr[-3000:]

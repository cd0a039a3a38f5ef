"""The host worker pool (go-txflow_amd/csrc/host_pack.hpp WorkerPool) under concurrent callers:
tools/debug/workerpool_stress.cpp built with g++ and run with 1-3 caller threads posting
parallel_for jobs back to back; every chunk must run exactly once and no caller may hang (the
slot word packs sequence, parts and next chunk so a stale claim cannot land in the next job)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def stress_bin(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("wps") / "stress")
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", os.path.join(ROOT, "tools", "debug", "workerpool_stress.cpp"),
                    "-o", out], check=True)
    return out


@pytest.mark.parametrize("threads,callers,spin", [(8, 1, 0), (8, 3, 5), (8, 3, 200), (16, 2, 5), (2, 3, 5)])
def test_worker_pool_concurrent_callers(stress_bin, threads, callers, spin):
    env = dict(os.environ, TXV_HOST_SPIN_US=str(spin))
    r = subprocess.run([stress_bin, str(threads), str(callers), "40000"], env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0 and "bad=0" in r.stdout, r.stdout + r.stderr[-2000:]

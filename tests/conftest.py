import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "go-txflow_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"),
          os.path.join(ROOT, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and libtxvote.so")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def oracle_lib():
    import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session", params=[(None, 0), (4, 0), (8, 2), (12, 4), (None, 1), (12, 1), (None, 8)],
                ids=["wauto", "w4", "w8v2", "w12v4", "wauto_split", "w12_split", "wauto_v8"])
def gpu_ctx(request):
    """One context per verify-table window: auto (radix-2^16 for the small test registries,
    radix-2^24 base table, and for these small batches the split K1b/K1c path the library picks
    below 768K votes), radix-16 LDS-resident B table, radix-256 with the LDS-parked pair kernel,
    radix-4096 with 4 votes per lane, the split path configured explicitly over the auto and
    radix-4096 tables, and 8 votes per lane (the kernel the library picks by itself for batches
    of >= 768K votes)."""
    import txflow_amd as T
    w, lv = request.param
    ctx = T.Context(max_batch=1 << 18, max_txs=1 << 16, max_validators=256, table_w=w, lane_votes=lv)
    yield ctx
    ctx.close()


_torch_hip_ready = False


def pytest_runtest_setup(item):
    """PyTorch ships its own HIP runtime beside the /opt/rocm one libtxvote.so links.  Initialise
    torch's first, before any txv context exists (the order bench.py's N>1 path and the multi-rank
    tests use): brought up after many contexts of the other runtime had come and gone, its device
    enumeration once reported "No HIP GPUs are available" (profiles/r04/gpu_tests_call3.log)."""
    global _torch_hip_ready
    if _torch_hip_ready or item.get_closest_marker("gpu") is None:
        return
    _torch_hip_ready = True
    import torch
    if torch.cuda.is_available():
        torch.cuda.init()

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


@pytest.fixture(scope="session", params=[None, 4, 8, 12], ids=["wauto", "w4", "w8", "w12"])
def gpu_ctx(request):
    """One context per verify-table window: auto (radix-2^16 for the small test registries),
    radix-16 LDS-resident B table, radix-256 and radix-4096 L2/MALL tables."""
    import txflow_amd as T
    ctx = T.Context(max_batch=1 << 18, max_txs=1 << 16, max_validators=256, table_w=request.param)
    yield ctx
    ctx.close()

"""The drop-in boundary: libtxvote.so loads on a machine without a GPU and exports exactly the
entry points include/txvote.h declares (no compute calls here).  Also checks that creating a
context without a HIP device fails loudly instead of falling back to the CPU."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "txvote.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(txv_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_expected_surface():
    names = declared_functions()
    for must in ("txv_init", "txv_destroy", "txv_set_validators", "txv_verify_batch", "txv_add_votes",
                 "txv_query_tx", "txv_signbytes", "txv_txvote_size"):
        assert must in names


def test_library_exports_every_declared_symbol():
    import txflow_amd as T
    lib = ctypes.CDLL(T.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    assert sorted(T.EXPORTED_SYMBOLS) == declared_functions()


def test_no_cpu_fallback_without_gpu():
    import txflow_amd as T
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        pytest.skip("GPU present")
    with pytest.raises(T.TxvInfraError):
        T.Context()


def test_product_does_not_import_oracle():
    """Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may touch oracle/."""
    pkg = os.path.join(ROOT, "go-txflow_amd")
    for dp, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h", ".hpp")):
                txt = open(os.path.join(dp, f)).read()
                assert "import oracle" not in txt and "oracle.h" not in txt and "liboracle" not in txt, f

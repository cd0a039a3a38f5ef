"""Runs the HIP kernel SOURCE (fe.h / sc.h / sha2.h / ge.h / ed25519_dev.h, compiled for the host
by tests/cpu_emu/emu.hip) against the oracle's golden verdicts.  A CPU-side check of the kernel
logic (carry chains, Barrett reduction, recoding, table walk, decode rules); the device ISA
itself is covered by the -m gpu tests."""
import ctypes
import json
import os
import random
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
EMU_DIR = os.path.join(HERE, "cpu_emu")
EMU = os.path.join(EMU_DIR, "build", "libemu.so")
P = 2 ** 255 - 19
L = 2 ** 252 + 27742317777372353535851937790883648493


@pytest.fixture(scope="module")
def emu():
    src = os.path.join(EMU_DIR, "emu.hip")
    deps = [src] + [os.path.join(HERE, "..", "go-txflow_amd", "csrc", f)
                    for f in ("fe.h", "fe_inv_var.h", "sc.h", "sha2.h", "ge.h", "ed25519_dev.h", "wire_dev.h")]
    if not os.path.exists(EMU) or any(os.path.getmtime(d) > os.path.getmtime(EMU) for d in deps):
        os.makedirs(os.path.dirname(EMU), exist_ok=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "-O1", "-std=c++17", "-fPIC", "-shared", src, "-o", EMU], check=True)
    E = ctypes.CDLL(EMU)
    E.emu_verify.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32]
    E.emu_wire_fast_hits.restype = ctypes.c_uint64
    E.emu_wire_decode.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                  ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    return E


def w(x):
    return (ctypes.c_uint32 * 8)(*[(x >> (32 * i)) & 0xFFFFFFFF for i in range(8)])


def f(a):
    return sum(a[i] << (32 * i) for i in range(8))


def test_field_and_scalar_ops(emu):
    rnd = random.Random(1)
    edges = [0, 1, 19, 38, P - 1, P, P + 1, 2 ** 255 - 1, 2 ** 255, 2 ** 256 - 1, 2 ** 256 - 38]
    for op in range(8):
        for t in range(200):
            x = edges[t] if t < len(edges) else rnd.getrandbits(256)
            y = edges[-1 - t] if t < len(edges) else rnd.getrandbits(256)
            out = (ctypes.c_uint32 * 8)()
            emu.emu_fe(w(x), w(y), out, op)
            v = f(out)
            exp = [x * y % P, x * x % P, (x + y) % P, (x - y) % P, x % P, pow(x, P - 2, P), (x + (y << 256)) % L,
                   pow(x, P - 2, P)][op]
            assert v < 2 ** 256
            assert (v % P if op < 6 else v) == exp, (op, hex(x), hex(y))
            if op in (4, 7):   # canonical outputs (7: variable-time divstep inverse, K1b)
                assert v == exp


def test_verify_vectors_through_kernel_source(emu):
    vec = json.load(open(os.path.join(HERE, "golden", "verify_vectors.json")))
    rnd = random.Random(3)
    sample = [v for v in vec if v["kind"] != "valid"]
    sample = rnd.sample(sample, 60) + [v for v in vec if v["kind"] == "valid"][:6]
    for v in sample:
        pub, msg, sig = bytes.fromhex(v["pub"]), bytes.fromhex(v["msg"]), bytes.fromhex(v["sig"])
        got = bool(emu.emu_verify(pub, msg, len(msg), sig, len(sig)))
        assert got == v["expect"], v["kind"]


def test_wire_decoder_source_vs_oracle(emu):
    """txv_k_decode_msgs' parser (wire_dev.h) on the host against oracle/wire.c over the mixed
    canonical / non-canonical / corrupted stream of tests/wire_gen.py, at every source alignment."""
    import numpy as np
    import oracle as O
    import wire_gen as G
    d, p = O.wire_prefix()
    disamb, prefix = int.from_bytes(d, "little"), int.from_bytes(p, "little")
    i64 = np.zeros(2, np.int64)
    u32 = np.zeros(6, np.uint32)
    rows = np.zeros(29, np.uint32)
    import random
    rng = random.Random(9)
    canon = [G.message(G.rand_vote(rng), rng, False) for _ in range(3000)]
    mixed = G.messages(6000, seed=5)
    near = [G.mutate(m, rng) for m in canon[:3000]]   # one edit away from the fast path's layout
    h0 = emu.emu_wire_fast_hits()
    for k, m in enumerate(mixed + canon + near):
        mx = 300 if k % 5 == 0 else 1 << 20
        st = emu.emu_wire_decode(m, len(m), mx, disamb, prefix, k % 4, i64.ctypes.data, u32.ctypes.data,
                                 rows.ctypes.data)
        est, f = O.wire_decode(m, mx)
        assert st == est, (k, m.hex())
        if st != O.WIRE_OK:
            continue
        rb = rows.view(np.uint8).tobytes()
        al, sl = len(f["addr"]), len(f["sig"])
        assert (int(i64[0]), int(i64[1]), int(u32[0])) == (f["height"], f["ts_sec"], f["ts_nanos"]), k
        assert (int(u32[1]), int(u32[2]), int(u32[3]), int(u32[5])) == (f["txhash_off"], len(f["txhash"]), al, sl), k
        assert sl == 0 or int(u32[4]) == f["sig_off"], k
        assert rb[:32] == f["txkey"], k
        assert rb[32:52] == f["addr"][:20] + bytes(20 - min(al, 20)), k
        assert rb[52:116] == f["sig"][:64] + bytes(64 - min(sl, 64)), k
    assert emu.emu_wire_fast_hits() - h0 > 2500   # canonical messages with <= 7-byte varints: fast path

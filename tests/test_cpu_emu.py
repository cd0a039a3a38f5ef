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
                    for f in ("fe.h", "fe10.h", "fe_inv_var.h", "sc.h", "sha2.h", "ge.h", "ed25519_dev.h", "wire_dev.h")]
    if not os.path.exists(EMU) or any(os.path.getmtime(d) > os.path.getmtime(EMU) for d in deps):
        os.makedirs(os.path.dirname(EMU), exist_ok=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "-O1", "-std=c++17", "-fPIC", "-shared", src, "-o", EMU], check=True)
    E = ctypes.CDLL(EMU)
    E.emu_verify.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32]
    E.emu_wire_fast_hits.restype = ctypes.c_uint64
    E.emu_fe10.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int]
    E.emu_ge10_madd.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    E.emu_ge10_madd_rd.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    E.emu_entry.argtypes = [ctypes.c_void_p] * 3
    E.emu_digits.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    E.emu_inv_var.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    E.emu_inv_var_counts.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
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


def test_divstep_inverse_near_its_bound(emu):
    """fe_invert_var (K1b's shared inversion) on inputs chosen to need many divsteps: structured
    ones (powers of two, p - 2^k, all-ones patterns, Fibonacci-ratio values) and the worst of a
    hill-climbing search over the batch count; every result equals pow(z, p - 2, p) and g reaches
    0 well before the 32-batch cap (Bernstein-Yang: <= 724 divsteps = 25 batches for 255 bits)."""
    import numpy as np
    rnd = random.Random(17)
    out = (ctypes.c_uint32 * 8)()
    fib = [0, 1]
    while len(fib) < 400:
        fib.append(fib[-1] + fib[-2])
    cands = [1, 2, P - 1, P - 2, (P - 1) // 2, (P + 1) // 2, 2 ** 254, 2 ** 255 - 20]
    cands += [2 ** k % P for k in range(0, 255, 7)] + [(P - 2 ** k) % P for k in range(1, 255, 11)]
    cands += [int("10" * 127, 2), int("110" * 84, 2) % P, int("1" * 254, 2)]
    cands += [fib[k] % P for k in range(300, 400, 5)] + [fib[k] * pow(fib[k + 1], P - 2, P) % P for k in range(50, 380, 30)]

    def counts(xs):
        arr = np.array([[(x >> (32 * i)) & 0xFFFFFFFF for i in range(8)] for x in xs], np.uint32)
        c = np.zeros(len(xs), np.int32)
        emu.emu_inv_var_counts(arr.ctypes.data, len(xs), c.ctypes.data)
        return c

    pool = [rnd.randrange(1, P) for _ in range(2000)]
    c = counts(pool)
    best = [pool[i] for i in np.argsort(-c)[:32]]
    for _ in range(40):                      # mutate the worst inputs, keep the worse
        kids = [(x ^ (1 << rnd.randrange(255))) % P or 1 for x in best for _ in range(8)]
        kc = counts(kids)
        allx = best + kids
        allc = np.concatenate([counts(best), kc])
        best = [allx[i] for i in np.argsort(-allc)[:32]]
    worst = int(counts(best).max())
    for z in cands + best:
        n = emu.emu_inv_var(w(z), out)
        assert 0 < n <= 25, (hex(z), n)
        assert f(out) == pow(z, P - 2, P), hex(z)
    assert emu.emu_inv_var(w(0), out) in (-1, 0, 1) and f(out) == 0
    assert worst >= 19                        # random inputs: 17-19 batches (mean 18.1 over 20k)


W10 = [26 if i % 2 == 0 else 25 for i in range(10)]
O10 = [sum(W10[:i]) for i in range(10)]


def v10(limbs):
    return sum(int(x) << o for x, o in zip(limbs, O10))


def l10(x):
    return (ctypes.c_uint32 * 10)(*[(x >> o) & ((1 << w) - 1) for o, w in zip(O10, W10)])


def carried(limbs):
    return all(int(x) < (1 << w) for x, w in zip(limbs, W10)) or (
        all(int(x) < (1 << w) for i, (x, w) in enumerate(zip(limbs, W10)) if i != 1) and limbs[1] < 2 ** 25 + 2 ** 18)


def test_fe10_limb_arithmetic_at_its_bounds(emu):
    """fe10 (radix 2^25.5, K1b's table walk): mul at the documented operand bounds (f < 4 2^w,
    g < 3 2^w, incl. every limb at its maximum), add/sub/cneg/carry/strict and both conversions."""
    rnd = random.Random(11)
    out = (ctypes.c_uint32 * 10)()
    maxf = [4 * (1 << w) - 1 for w in W10]
    maxg = [3 * (1 << w) - 1 for w in W10]
    cases = [(maxf, maxg), ([0] * 10, maxg), (maxf, [0] * 10)]
    for _ in range(400):
        cases.append(([rnd.randrange(4 << w) for w in W10], [rnd.randrange(3 << w) for w in W10]))
        cases.append(([rnd.choice([0, (4 << w) - 1, rnd.randrange(4 << w)]) for w in W10],
                      [rnd.choice([0, (3 << w) - 1, rnd.randrange(3 << w)]) for w in W10]))
    out2 = (ctypes.c_uint32 * 20)()
    for fa, ga in cases:
        emu.emu_fe10((ctypes.c_uint32 * 10)(*fa), (ctypes.c_uint32 * 10)(*ga), out, 0)
        assert v10(out) % P == v10(fa) * v10(ga) % P and carried(list(out)), (fa, ga)
        if max(fa[i] - (3 << w) for i, w in enumerate(W10)) < 0:
            # fe10_mul2 (the walk's interleaved pair) = fe10_mul of each pair, limb for limb
            emu.emu_fe10((ctypes.c_uint32 * 10)(*fa), (ctypes.c_uint32 * 10)(*ga), out2, 9)
            assert list(out2[:10]) == list(out), (fa, ga)
            emu.emu_fe10((ctypes.c_uint32 * 10)(*ga), (ctypes.c_uint32 * 10)(*fa), out, 0)
            assert list(out2[10:]) == list(out), (fa, ga)
    for _ in range(300):
        a, b = rnd.randrange(P), rnd.randrange(P)
        for op, exp in ((1, a + b), (2, a - b), (3, -a)):
            emu.emu_fe10(l10(a), l10(b), out, op)
            assert v10(out) % P == exp % P, op
            assert all(int(x) < (3 << w) for x, w in zip(out, W10))
        big = [rnd.randrange(1 << 32 - 8) for _ in range(10)]
        emu.emu_fe10((ctypes.c_uint32 * 10)(*big), l10(0), out, 4)
        assert v10(out) % P == v10(big) % P and carried(list(out))
        emu.emu_fe10((ctypes.c_uint32 * 10)(*big), l10(0), out, 5)
        assert v10(out) % P == v10(big) % P and v10(out) < 2 ** 255
        assert all(int(x) < (1 << w) for x, w in zip(out, W10))
    o8 = (ctypes.c_uint32 * 8)()
    for x in [0, 1, P - 1, P, 2 ** 255 - 1, 2 ** 255, 2 ** 256 - 1] + [rnd.getrandbits(256) for _ in range(200)]:
        emu.emu_fe10(w(x), l10(0), out, 6)
        assert v10(out) % P == x % P
        emu.emu_fe10(out, l10(0), o8, 7)
        assert f(o8) % P == x % P and f(o8) < 2 ** 255 + 19


def _ed_add(p1, p2):
    d = -121665 * pow(121666, P - 2, P) % P
    (x1, y1), (x2, y2) = p1, p2
    t = d * x1 * x2 * y1 * y2 % P
    return ((x1 * y2 + y1 * x2) * pow(1 + t, P - 2, P) % P, (y1 * y2 + x1 * x2) * pow(1 - t, P - 2, P) % P)


def test_ge10_madd_half_niels(emu):
    """ge10_madd with the half-Niels entries ((y+x)/2, (y-x)/2, dxy) gives P + Q and P - Q as the
    same projective point (x = X/Z, y = Y/Z, XY = ZT), including the identity entry and Q = P."""
    by = 4 * pow(5, P - 2, P) % P
    d = -121665 * pow(121666, P - 2, P) % P
    u, v = (by * by - 1) % P, (d * by * by + 1) % P
    bx = pow(u * pow(v, P - 2, P), (P + 3) // 8, P)
    if (v * bx * bx - u) % P:
        bx = bx * pow(2, (P - 1) // 4, P) % P
    if bx & 1:
        bx = P - bx
    B = (bx, by)
    pts = [B]
    for _ in range(12):
        pts.append(_ed_add(pts[-1], B if len(pts) % 2 else pts[-1]))
    pts.append((0, 1))
    rnd = random.Random(5)
    e = (ctypes.c_uint32 * 32)()
    out = (ctypes.c_uint32 * 40)()
    for _ in range(60):
        p1, q = rnd.choice(pts), rnd.choice(pts + [pts[0]])
        z = rnd.randrange(1, P)
        X, Y, Z = p1[0] * z % P, p1[1] * z % P, z
        T = p1[0] * p1[1] * z % P
        limbs = [int(x) for c in (X, Y, Z, T) for x in l10(c)]
        emu.emu_entry(w(q[0]), w(q[1]), e)
        assert e[10] == 0 and e[11] == 0
        for neg in (0, 1):
            emu.emu_ge10_madd((ctypes.c_uint32 * 40)(*limbs), e, neg, out)
            X3, Y3, Z3, T3 = (v10(out[10 * i:10 * i + 10]) for i in range(4))
            assert carried(list(out[:10])) and carried(list(out[30:]))
            exp = _ed_add(p1, (P - q[0] if neg else q[0], q[1]))
            zi = pow(Z3, P - 2, P)
            assert (X3 * zi % P, Y3 * zi % P) == exp and (X3 * Y3 - Z3 * T3) % P == 0
            # the walk's form (product pairs) gives the same limbs; without T for the last addition
            out_rd = (ctypes.c_uint32 * 40)()
            emu.emu_ge10_madd_rd((ctypes.c_uint32 * 40)(*limbs), e, neg, out_rd, 1)
            assert list(out_rd) == list(out)
            emu.emu_ge10_madd_rd((ctypes.c_uint32 * 40)(*limbs), e, neg, out_rd, 0)
            assert list(out_rd[:30]) == list(out[:30])


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


def test_table_digits_cover_every_scalar_below_L(emu):
    """The walks' digit recoding (ed25519_dev.h table_digit / signed_digits): the digits of every
    scalar < L sum back to it, and each indexes an existing entry of its table position -- for
    the long-top radix-2^21 layout (Tab<21>: 12 positions, the top one unsigned in [0, 2^21 + 1])
    at the top of the range too, where 11 signed radix-2^21 digits alone cannot reach"""
    rnd = random.Random(21)
    edges = [0, 1, L - 1, L - 2, 2 ** 252, 2 ** 252 - 1, 2 ** 252 - 2 ** 231, 2 ** 252 - 2 ** 230,
             2 ** 252 + 2 ** 124, (2 ** 231 - 1) * (2 ** 21 + 1), sum(1 << (21 * i + 20) for i in range(12)) % L,
             sum(1 << (21 * i + 20) for i in range(11)), sum(1 << (21 * i + 19) for i in range(12)) % L]
    scalars = edges + [rnd.randrange(L) for _ in range(300)] + [L - 1 - rnd.getrandbits(130) for _ in range(50)]
    for wd, top_max in ((20, 1 << 19), (21, (1 << 21) + 1), (24, 1 << 23), (26, 1 << 25)):
        for mode in (0, 1):
            for x in scalars:
                out = (ctypes.c_int32 * 16)()
                n = emu.emu_digits(wd, w(x), mode, out)
                d = list(out[:n])
                assert sum(di << (wd * i) for i, di in enumerate(d)) == x, (wd, mode, hex(x))
                half = 1 << (wd - 1)
                for i, di in enumerate(d[:-1]):
                    assert -half <= di < half, (wd, i, di)
                if wd == 21:
                    assert n == 12 and 0 <= d[-1] <= top_max, (hex(x), d[-1])
                else:
                    assert n == -(-256 // wd) and -half <= d[-1] <= top_max

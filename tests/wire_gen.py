"""Deterministic generator of received TxVoteMessage wire bytes for the decode parity tests.

Canonical messages come from the oracle's encoder (cdc.MarshalBinaryBare(&TxVoteMessage{vote}),
txvotepool/reactor.go:248 on the sending side); the other categories exercise the amino decoder
rules restated in oracle/wire.c: disfix framing, overlong varints, explicit default fields,
skipped fields, extra fields of every typ3, non-minimal nested-struct lengths (the parent's
UvarintSize(len) advance), time bodies with unread bytes, truncations, byte flips and garbage.
Test infrastructure only.
"""
import random

import oracle as O

DISAMB, PREFIX = O.wire_prefix()


def uv(v: int, extra: int = 0) -> bytes:
    """uvarint of v (two's complement for negatives) with `extra` overlong bytes"""
    v &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            break
    if extra:
        out[-1] |= 0x80
        out += b"\x80" * (extra - 1) + b"\x00"
    return bytes(out)


def key(num: int, typ: int, extra: int = 0) -> bytes:
    return uv((num << 3) | typ, extra)


def lp(b: bytes, extra: int = 0) -> bytes:
    return uv(len(b), extra) + b


def rand_vote(rng: random.Random):
    r = rng.random()
    height = rng.choice([0, 1, 1, 1, 7, -1, -(1 << 63), (1 << 63) - 1, rng.getrandbits(40)])
    thl = rng.choice([64, 64, 64, 0, 1, 20, 127, 128, 300])
    txhash = bytes(rng.choice(b"0123456789ABCDEF") for _ in range(thl))
    ts = rng.choice([(1_700_000_000, rng.randrange(1, 10**9)), (0, 0), (0, 5), (-62135596800, 0),
                     (253402300799, 999999999), (1_700_000_000, 0), (-1, 1)])
    al = rng.choice([20, 20, 20, 0, 19, 21, 3])
    addr = bytes(rng.getrandbits(8) for _ in range(al))
    sl = rng.choice([64, 64, 64, 0, 63, 65, 100, 1000]) if r < 0.997 else 70000
    sig = bytes(rng.getrandbits(8) for _ in range(sl))
    txkey = bytes(32) if rng.random() < 0.7 else bytes(rng.getrandbits(8) for _ in range(32))
    return dict(height=height, txhash=txhash, ts=ts, addr=addr, sig=sig, txkey=txkey)


def time_body(sec, nanos, order=(1, 2), extra=b""):
    b = b""
    for f in order:
        if f == 1 and sec:
            b += key(1, 0) + uv(sec)
        if f == 2 and nanos:
            b += key(2, 0) + uv(nanos)
    return b + extra


def body(v, rng: random.Random, noncanon: bool):
    """TxVote body; with noncanon, random decoder-visible variations"""
    parts = []
    ov = (lambda: rng.choice([0, 0, 1, 3])) if noncanon else (lambda: 0)
    if v["height"] or (noncanon and rng.random() < 0.2):
        parts.append(key(1, 0, ov()) + uv(v["height"], ov()))
    if v["txhash"] or (noncanon and rng.random() < 0.1):
        parts.append(key(2, 2) + lp(v["txhash"], ov()))
    if not (noncanon and rng.random() < 0.1):   # TxKey may be skipped (default)
        parts.append(key(3, 2) + lp(v["txkey"], ov()))
    sec, nanos = v["ts"]
    tb = time_body(sec, nanos)
    if noncanon:
        c = rng.random()
        if c < 0.15:
            tb = time_body(sec, nanos, order=(2, 1))            # nanos first: seconds left unread
        elif c < 0.3:
            tb = tb + rng.choice([b"\x18\x01", b"\x08\x01", b"\x32\x00", bytes([rng.getrandbits(8)])])
    if tb or (noncanon and rng.random() < 0.1):
        parts.append(key(4, 2) + lp(tb, ov()))
    if v["addr"] or (noncanon and rng.random() < 0.1):
        parts.append(key(5, 2) + lp(v["addr"], ov()))
    if v["sig"] or (noncanon and rng.random() < 0.1):
        parts.append(key(6, 2) + lp(v["sig"], ov()))
    if noncanon and rng.random() < 0.3:   # extra fields, increasing numbers
        num = rng.choice([7, 8, 30, 1 << 20])
        for _ in range(rng.randrange(1, 3)):
            t = rng.choice([0, 1, 2, 5, 3, 7])
            val = {0: uv(rng.getrandbits(20)), 1: bytes(8), 2: lp(b"xyz"), 5: bytes(4), 3: b"", 7: b""}[t]
            parts.append(key(num, t) + val)
            num += rng.randrange(0, 3)        # sometimes equal: must be an error
    if noncanon and rng.random() < 0.05:
        rng.shuffle(parts)                     # out of order: errors or absent-field defaults
    return b"".join(parts)


def message(v, rng: random.Random, noncanon: bool) -> bytes:
    if not noncanon:
        m = O.wire_encode(v["height"], v["txhash"], v["ts"][0], v["ts"][1], v["addr"], v["sig"], v["txkey"])
        assert m is not None
        return m
    b = body(v, rng, True)
    framing = PREFIX if rng.random() < 0.7 else b"\x00" + DISAMB + PREFIX
    ext = rng.choice([0, 0, 0, 1, 2])         # non-minimal nested length: parent advance quirk
    m = framing + key(1, 2) + lp(b, ext)
    if rng.random() < 0.1:
        m += key(rng.choice([2, 3, 9]), rng.choice([0, 2])) + rng.choice([uv(5), lp(b"ab")])
    return m


def mutate(m: bytes, rng: random.Random) -> bytes:
    c = rng.random()
    b = bytearray(m)
    if c < 0.3 and b:
        return bytes(b[:rng.randrange(len(b))])
    if c < 0.6 and b:
        for _ in range(rng.randrange(1, 4)):
            i = rng.randrange(len(b))
            b[i] ^= 1 << rng.randrange(8)
        return bytes(b)
    if c < 0.75 and b:
        i = rng.randrange(len(b) + 1)
        return bytes(b[:i] + bytes([rng.getrandbits(8)]) + b[i:])
    if c < 0.85:
        return bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 12)))
    if c < 0.92:
        return PREFIX + bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 40)))
    return b""


def messages(n: int, seed: int, p_noncanon=0.35, p_mutate=0.25):
    """n wire messages: canonical / non-canonical-valid / mutated mix"""
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        v = rand_vote(rng)
        try:
            m = message(v, rng, rng.random() < p_noncanon)
        except AssertionError:
            m = b""
        if rng.random() < p_mutate:
            m = mutate(m, rng)
        out.append(m)
    return out

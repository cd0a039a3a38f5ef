"""Pins the CPU oracle (oracle/) before anything is checked against it (CPU only).

- ed25519: OpenSSL 3 vectors (RFC 8032 deterministic == Go ed25519.Sign) must be reproduced
  bit-for-bit (pub, sig) and accepted; adversarial vectors must get their recorded verdict
  (x/crypto@c2843e01d9a2 rules; OpenSSL agrees on all of them).
- SHA-2 against hashlib; ScReduce against Python integers.
- amino: SignBytes / Size fixtures incl. the reference's own pinned values
  (types/vote_test.go:62 zero time, txvotepool/txvotepool_test.go:102 Size()==114).
"""
import hashlib
import json
import os
import random

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
L = 2 ** 252 + 27742317777372353535851937790883648493


def load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def test_openssl_vectors(oracle_lib):
    O = oracle_lib
    for c in load("ed25519_openssl.json"):
        seed, msg = bytes.fromhex(c["seed"]), bytes.fromhex(c["msg"])
        assert O.pubkey(seed).hex() == c["pub"]
        assert O.sign(seed, msg).hex() == c["sig"]
        assert O.verify(bytes.fromhex(c["pub"]), msg, bytes.fromhex(c["sig"]))


def test_adversarial_verify_vectors(oracle_lib):
    O = oracle_lib
    vec = load("verify_vectors.json")
    kinds = set()
    for v in vec:
        got = O.verify(bytes.fromhex(v["pub"]), bytes.fromhex(v["msg"]), bytes.fromhex(v["sig"]))
        assert got == v["expect"], v["kind"]
        kinds.add(v["kind"])
    # the fixture covers the Appendix C classes
    for k in ("valid", "r_bitflip", "s_bitflip", "s_plus_L", "s_top_bit", "len63", "msg_changed",
              "torsion_canon_ord8", "torsion_noncanon_y_ord1", "torsion_negzero_ord2", "mixed_order_ord8",
              "ident_R_noncanon_y", "ident_R_negzero", "undecodable_pub"):
        assert k in kinds


def test_decode_rules(oracle_lib):
    """Appendix A.1 step 3: y >= p accepted, x = 0 with sign bit accepted, no-root rejected."""
    O = oracle_lib
    P = 2 ** 255 - 19
    ident = (1).to_bytes(32, "little")
    assert O.decode_ok(ident)
    assert O.decode_ok((1 | (1 << 255)).to_bytes(32, "little"))        # -0
    assert O.decode_ok((1 + P).to_bytes(32, "little"))                   # y >= p
    assert O.point_canonical((1 + P).to_bytes(32, "little")) == ident
    assert O.decode_ok((P - 1).to_bytes(32, "little"))                    # order 2
    assert not O.decode_ok((2).to_bytes(32, "little"))                    # y = 2 has no x


def test_hashes_and_scalars(oracle_lib):
    O = oracle_lib
    rnd = random.Random(9)
    for n in list(range(0, 260)) + [1000, 4096]:
        m = bytes(rnd.getrandbits(8) for _ in range(n))
        assert O.sha512(m) == hashlib.sha512(m).digest()
        assert O.sha256(m) == hashlib.sha256(m).digest()
    for _ in range(2000):
        x = rnd.getrandbits(512)
        assert O.sc_reduce64(x.to_bytes(64, "little")) == (x % L).to_bytes(32, "little")
    for s in (0, 1, L - 1, L, L + 1, 2 ** 253, 2 ** 256 - 1):
        assert O.sc_minimal(s.to_bytes(32, "little")) == (s < L)


def test_signbytes_fixtures(oracle_lib):
    O = oracle_lib
    cases = load("signbytes.json")
    # types/vote_test.go:62: Go zero time body
    zero = bytes.fromhex(cases[0]["hex"])
    assert zero.endswith(bytes([0x22, 0x0b, 0x08, 0x80, 0x92, 0xb8, 0xc3, 0x98, 0xfe, 0xff, 0xff, 0xff, 0x01]))
    for c in cases:
        got = O.signbytes(c["height"], c["txhash"].encode(), c["ts_sec"], c["ts_nanos"], c["chain"].encode())
        assert (None if got is None else got.hex()) == c["hex"]
    for c in load("size.json"):
        assert O.txvote_size(c["height"], c["txhash_len"], c["ts_sec"], c["ts_nanos"], c["addr_len"],
                             c["sig_len"]) == c["size"]


def test_product_host_encoder_matches_fixtures():
    """The product's C++ amino encoder (libtxvote.so host code, no device) on the same fixtures."""
    import txflow_amd as T
    for c in load("signbytes.json"):
        try:
            got = T.sign_bytes(c["height"], c["txhash"].encode(), c["ts_sec"], c["ts_nanos"], c["chain"])
        except ValueError:
            got = None
        assert (None if got is None else got.hex()) == c["hex"]
    for c in load("size.json"):
        assert T.txvote_size(c["height"], c["txhash_len"], c["ts_sec"], c["ts_nanos"], c["addr_len"],
                             c["sig_len"]) == c["size"]


def test_signbytes_random_vs_product(oracle_lib):
    import txflow_amd as T
    rnd = random.Random(5)
    for _ in range(400):
        h = bytes(rnd.choice(b"0123456789ABCDEF") for _ in range(rnd.choice([0, 1, 64, 127, 128, 300])))
        height = rnd.choice([0, 1, -1, 2 ** 63 - 1, -2 ** 63, 12345])
        sec = rnd.choice([0, 1, -1, 1_700_000_000, -62135596800, 253402300799, -62135596801, 253402300800])
        nanos = rnd.choice([0, 1, 999_999_999, 2 ** 28, 2 ** 28 - 1])
        chain = rnd.choice([b"", b"test_chain_id", b"x" * 200])
        exp = oracle_lib.signbytes(height, h, sec, nanos, chain)
        try:
            got = T.sign_bytes(height, h, sec, nanos, chain)
        except ValueError:
            got = None
        assert got == exp

"""GPU parity tests: libtxvote.so (HIP, gfx950) against the CPU oracle on identical inputs.

Bit-exact for every integer/byte result: field and scalar ops, public keys, signatures,
per-vote accept/reject, per-vote (added, err) codes incl. the commit-fire bit, per-tx sums."""
import os
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

P = 2 ** 255 - 19
L = 2 ** 252 + 27742317777372353535851937790883648493


def to_words(x: int) -> list:
    return [(x >> (32 * i)) & 0xFFFFFFFF for i in range(8)]


def from_words(w) -> int:
    return sum(int(v) << (32 * i) for i, v in enumerate(w))


def _edge_values():
    vals = [0, 1, 2, 19, 38, P - 1, P, P + 1, P + 18, 2 ** 255 - 1, 2 ** 255, 2 ** 256 - 1, 2 ** 256 - 38,
            2 ** 256 - 39, 2 ** 32 - 1, 2 ** 64 - 1, 2 ** 224, (2 ** 256 - 1) // 3]
    return vals


@pytest.mark.parametrize("op", [0, 1, 2, 3, 4, 5])
def test_field_ops_bit_exact(gpu_ctx, op):
    rnd = random.Random(op)
    A = _edge_values() + [rnd.getrandbits(256) for _ in range(2000)]
    B = list(reversed(_edge_values())) + [rnd.getrandbits(256) for _ in range(2000)]
    a = np.array([to_words(x) for x in A], np.uint32)
    b = np.array([to_words(x) for x in B], np.uint32)
    out = gpu_ctx.fe_selftest(a, b, op)
    for x, y, w in zip(A, B, out):
        r = from_words(w)
        assert r < 2 ** 256
        if op == 0:
            exp = x * y % P
        elif op == 1:
            exp = x * x % P
        elif op == 2:
            exp = (x + y) % P
        elif op == 3:
            exp = (x - y) % P
        elif op == 4:
            exp = x % P
            assert r == exp  # canonical
        else:
            exp = pow(x, P - 2, P)
        assert r % P == exp, (op, hex(x), hex(y), hex(r))


def test_scalar_reduce_bit_exact(gpu_ctx):
    rnd = random.Random(7)
    X = [rnd.getrandbits(512) for _ in range(3000)] + [0, L, L - 1, 2 * L, 2 ** 512 - 1, L * (2 ** 259)]
    a = np.array([to_words(x & (2 ** 256 - 1)) for x in X], np.uint32)
    b = np.array([to_words(x >> 256) for x in X], np.uint32)
    out = gpu_ctx.fe_selftest(a, b, 6)
    for x, w in zip(X, out):
        assert from_words(w) == x % L


def test_keygen_matches_oracle(gpu_ctx, oracle_lib):
    rnd = random.Random(3)
    seeds = [bytes(rnd.getrandbits(8) for _ in range(32)) for _ in range(64)]
    pubs = gpu_ctx.keygen(seeds)
    for s, p in zip(seeds, pubs):
        assert p == oracle_lib.pubkey(s)


def _mini_votes(T, n, rnd, chain_len_var=False):
    votes = []
    for i in range(n):
        h = "".join(rnd.choice("0123456789ABCDEF") for _ in range(64 if i % 7 else rnd.randrange(0, 300)))
        votes.append(T.TxVote(Height=rnd.choice([0, 1, 5, -3, 2 ** 40]), TxHash=h,
                              Timestamp=(rnd.choice([1_700_000_000, 0, -5, 253402300799]), rnd.randrange(0, 10 ** 9)),
                              ValidatorAddress=b"", Signature=b""))
    return votes


def test_sign_matches_oracle(gpu_ctx, oracle_lib):
    import txflow_amd as T
    rnd = random.Random(11)
    seeds = [bytes(rnd.getrandbits(8) for _ in range(32)) for _ in range(8)]
    pubs = gpu_ctx.keygen(seeds)
    votes = _mini_votes(T, 300, rnd)
    batch = T.VoteBatch.from_votes(votes)
    signer = np.array([rnd.randrange(8) for _ in votes], np.uint32)
    sigs = gpu_ctx.sign_votes(batch, signer, "test_chain_id")
    for i, v in enumerate(votes):
        msg = oracle_lib.signbytes(v.Height, v.TxHash.encode(), v.Timestamp[0], v.Timestamp[1], b"test_chain_id")
        assert msg is not None
        assert sigs[i].tobytes() == oracle_lib.sign(seeds[signer[i]], msg), i


def test_signbytes_host_encoder_matches_oracle(oracle_lib):
    import txflow_amd as T
    rnd = random.Random(5)
    for _ in range(500):
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


def _signed_set(gpu_ctx, T, n_vals, n_votes, rnd, n_txs=None):
    seeds = [bytes(rnd.getrandbits(8) for _ in range(32)) for _ in range(n_vals)]
    pubs = gpu_ctx.keygen(seeds)
    gpu_ctx.set_validators(pubs, [1 + (i % 3) for i in range(n_vals)], "test_chain_id")
    addrs, ok = gpu_ctx.validator_info()
    assert ok.all()
    n_txs = n_txs or max(1, n_votes // n_vals)
    hashes = ["".join(rnd.choice("0123456789ABCDEF") for _ in range(64)) for _ in range(n_txs)]
    votes, signer = [], []
    for i in range(n_votes):
        vi = rnd.randrange(n_vals)
        votes.append(T.TxVote(Height=1, TxHash=rnd.choice(hashes), Timestamp=(1_700_000_000, i + 1),
                              ValidatorAddress=addrs[vi], Signature=b""))
        signer.append(vi)
    b = T.VoteBatch.from_votes(votes)
    sigs = gpu_ctx.sign_votes(b, np.array(signer, np.uint32), "test_chain_id")
    for v, s in zip(votes, sigs):
        v.Signature = s.tobytes()
    return seeds, pubs, addrs, votes, signer


def test_verify_batch_valid_and_corrupt(gpu_ctx, oracle_lib):
    import txflow_amd as T
    rnd = random.Random(21)
    seeds, pubs, addrs, votes, signer = _signed_set(gpu_ctx, T, 16, 2000, rnd)
    # corrupt a third of them in assorted ways
    kinds = []
    for i, v in enumerate(votes):
        k = i % 9
        s = bytearray(v.Signature)
        if k == 1:
            s[rnd.randrange(32)] ^= 1 << rnd.randrange(8)          # R bit flip
        elif k == 2:
            s[32 + rnd.randrange(31)] ^= 1 << rnd.randrange(8)     # S bit flip
        elif k == 3:
            S = int.from_bytes(s[32:], "little") + L                # non-canonical s (s + L)
            if S < 2 ** 256:
                s[32:] = S.to_bytes(32, "little")
        elif k == 4:
            s[63] |= 0xE0
        elif k == 5:
            v.Timestamp = (v.Timestamp[0], v.Timestamp[1] + 1)     # message changed after signing
        elif k == 6:
            s = s[:63]                                              # length != 64
        v.Signature = bytes(s)
        kinds.append(k)
    b = T.VoteBatch.from_votes(votes)
    st = gpu_ctx.verify_batch(b)
    for i, v in enumerate(votes):
        msg = oracle_lib.signbytes(1, v.TxHash.encode(), v.Timestamp[0], v.Timestamp[1], b"test_chain_id")
        exp = oracle_lib.verify(pubs[signer[i]], msg, v.Signature)
        assert (st[i] == T.ADDED) == exp, (i, kinds[i], st[i])
    # explicit (caller-supplied) pubkeys: wrong key -> ErrVoteInvalidValidatorAddress
    keys = np.array([np.frombuffer(pubs[(signer[i] + (1 if i % 5 == 0 else 0)) % len(pubs)], np.uint8)
                     for i in range(len(votes))])
    st2 = gpu_ctx.verify_batch(b, keys)
    for i in range(len(votes)):
        if i % 5 == 0:
            assert st2[i] == T.ERR_INVALID_VALIDATOR_ADDRESS
        else:
            assert st2[i] == st[i]


def test_add_votes_matches_sequential_oracle(gpu_ctx, oracle_lib):
    import txflow_amd as T
    rnd = random.Random(33)
    seeds, pubs, addrs, votes, signer = _signed_set(gpu_ctx, T, 10, 3000, rnd, n_txs=40)
    # add replays, conflicts, bad sigs, unknown/empty validators, nil votes
    extra = []
    for i in range(600):
        base = rnd.choice(votes)
        k = i % 6
        v = T.TxVote(Height=base.Height, TxHash=base.TxHash, Timestamp=base.Timestamp,
                     ValidatorAddress=base.ValidatorAddress, Signature=base.Signature)
        if k == 1:
            v.Timestamp = (v.Timestamp[0], v.Timestamp[1] + 7)       # conflicting (different sig later)
        elif k == 2:
            s = bytearray(v.Signature); s[5] ^= 0x10; v.Signature = bytes(s)
        elif k == 3:
            v.ValidatorAddress = bytes(20)
        elif k == 4:
            v.ValidatorAddress = b""
        elif k == 5:
            v = None
        extra.append(v)
    allv = votes + extra
    rnd.shuffle(allv)
    flow = oracle_lib.Flow(pubs, [1 + (i % 3) for i in range(len(pubs))], b"test_chain_id")
    gpu_ctx.set_validators(pubs, [1 + (i % 3) for i in range(len(pubs))], "test_chain_id")
    # two batches to exercise cross-batch state
    cut = len(allv) // 2
    for part in (allv[:cut], allv[cut:]):
        b = T.VoteBatch.from_votes(part)
        st, ev = gpu_ctx.add_votes(b)
        od = [dict(nil=True) if v is None else dict(height=v.Height, txhash=v.TxHash.encode(), ts_sec=v.Timestamp[0],
                                                     ts_nanos=v.Timestamp[1], addr=v.ValidatorAddress,
                                                     sig=v.Signature) for v in part]
        ost, osum, ofired = flow.add_votes(od)
        exp = ost.astype(np.uint8) | (ofired.astype(np.uint8) << 7)
        bad = np.nonzero(st != exp)[0]
        assert len(bad) == 0, [(int(i), int(st[i]), int(exp[i])) for i in bad[:10]]
    for v in allv:
        if v is None:
            continue
        assert gpu_ctx.query_tx(v.TxHash.encode()) == flow.query(v.TxHash.encode())
    assert gpu_ctx.num_tx_sets() == flow.num_sets()


def _table_mb(w: int) -> float:
    return -(-256 // w) * ((1 << (w - 1)) + 1) * 128 / 2 ** 20     # 128-byte entries


@pytest.mark.parametrize("budget_mb,exp_w", [(1, 4), (100, 12), (1100, 16), (4100, 18), (0, 20)])
def test_window_policy_and_parity(oracle_lib, budget_mb, exp_w):
    """Auto window = largest of 20/18/16/14/12/10/8 whose per-validator tables fit the budget
    (0 = 112 GiB default), else 4; every window verifies bit-exactly like the oracle, through
    the registry and through caller-supplied keys on a context without a registry."""
    import txflow_amd as T
    n_vals = 16
    exp_fit = max([w for w in (8, 10, 12, 14, 16, 18, 20) if n_vals * _table_mb(w) <= (budget_mb or 114688)], default=4)
    assert exp_fit == exp_w
    ctx = T.Context(max_batch=1 << 14, max_txs=1 << 12, max_validators=64, table_budget_mb=budget_mb)
    try:
        assert ctx.table_w == 0
        rnd = random.Random(100 + exp_w)
        seeds, pubs, addrs, votes, signer = _signed_set(ctx, T, n_vals, 1500, rnd)
        assert ctx.table_w == exp_w
        for i, v in enumerate(votes):
            if i % 4 == 1:
                s = bytearray(v.Signature); s[rnd.randrange(64)] ^= 1 << rnd.randrange(8); v.Signature = bytes(s)
        b = T.VoteBatch.from_votes(votes)
        st = ctx.verify_batch(b)
        exp = np.array([oracle_lib.verify(pubs[signer[i]], oracle_lib.signbytes(
            1, v.TxHash.encode(), v.Timestamp[0], v.Timestamp[1], b"test_chain_id"), v.Signature)
            for i, v in enumerate(votes)])
        assert np.array_equal(st == T.ADDED, exp)
        keys = np.array([np.frombuffer(pubs[signer[i]], np.uint8) for i in range(len(votes))])
        assert np.array_equal(ctx.verify_batch(b, keys), st)
    finally:
        ctx.close()
    # caller-supplied keys against an empty registry (chain id only): their tables use the
    # registry's window when they fit the budget, else radix-16
    ctx2 = T.Context(max_batch=1 << 14, max_txs=1 << 12, max_validators=64, table_budget_mb=budget_mb)
    try:
        ctx2.set_validators([], [], "test_chain_id")
        assert np.array_equal(ctx2.verify_batch(b, keys), st)
    finally:
        ctx2.close()


@pytest.mark.parametrize("table_w,base_w,lane_votes,n_votes",
                         [(16, 20, 0, 800), (16, 24, 0, 800), (12, 24, 0, 800), (14, 24, 0, 800), (18, 24, 0, 800),
                          (20, 24, 0, 800), (16, 26, 0, 800), (18, 26, 0, 800), (20, 26, 0, 800),
                          (21, 26, 0, 800), (21, 26, 1, 3000), (21, 26, 4, 3000), (21, 26, 8, 20000)])
def test_wide_base_table_parity(oracle_lib, table_w, base_w, lane_votes, n_votes):
    """Radix-2^20 / 2^24 / 2^26 base-point tables (0.9 / 11.8 / 43 GB) over radix-2^12..2^21
    validator tables (21: the 12-position long-top layout, through the split, 4-vote and
    8-vote work-stealing K1b kernels): the same verdicts as the oracle on valid and corrupted
    votes."""
    import txflow_amd as T
    ctx = T.Context(max_batch=1 << 15, max_txs=1 << 12, max_validators=16, table_w=table_w, base_w=base_w,
                    lane_votes=lane_votes)
    try:
        rnd = random.Random(base_w * 100 + table_w + lane_votes)
        seeds, pubs, addrs, votes, signer = _signed_set(ctx, T, 4, n_votes, rnd)
        assert (ctx.table_w, ctx.base_w) == (table_w, base_w)
        for i, v in enumerate(votes):
            if i % 3 == 1:
                s = bytearray(v.Signature); s[rnd.randrange(64)] ^= 1 << rnd.randrange(8); v.Signature = bytes(s)
        st = ctx.verify_batch(T.VoteBatch.from_votes(votes))
        exp = np.array([oracle_lib.verify(pubs[signer[i]], oracle_lib.signbytes(
            1, v.TxHash.encode(), v.Timestamp[0], v.Timestamp[1], b"test_chain_id"), v.Signature)
            for i, v in enumerate(votes)])
        assert np.array_equal(st == T.ADDED, exp)
        assert exp.sum() > len(votes) // 2
    finally:
        ctx.close()


def test_golden_vectors_verify_bytes(gpu_ctx):
    """Every committed ed25519 fixture through PubKeyEd25519.VerifyBytes on the GPU
    (txv_verify_bytes): the OpenSSL RFC 8032 vectors must verify, and each adversarial vector
    (torsion / small-order / mixed-order / y >= p / "-0" / undecodable keys, non-canonical R,
    s + L, top bits, bit flips, lengths 0/63/65) must get its recorded x/crypto-rule verdict."""
    import json
    here = os.path.dirname(os.path.abspath(__file__))
    with open(os.path.join(here, "golden", "verify_vectors.json")) as f:
        vec = json.load(f)
    with open(os.path.join(here, "golden", "ed25519_openssl.json")) as f:
        ossl = json.load(f)
    cases = [(v["pub"], v["msg"], v["sig"], v["expect"], v["kind"]) for v in vec]
    cases += [(c["pub"], c["msg"], c["sig"], True, "openssl") for c in ossl]
    pubs = [bytes.fromhex(c[0]) for c in cases]
    msgs = [bytes.fromhex(c[1]) for c in cases]
    sigs = [bytes.fromhex(c[2]) for c in cases]
    got = gpu_ctx.verify_bytes(pubs, msgs, sigs)
    bad = [(c[4], bool(g)) for c, g in zip(cases, got) if bool(g) != c[3]]
    assert not bad, bad[:10]
    assert sum(c[3] for c in cases) > 60 and sum(not c[3] for c in cases) > 100


def test_c4_adversarial_stream_gate(oracle_lib):
    """C4 at test size: 3 batches x 64k adversarial votes across two
    TxFlow epochs -- bad signatures of every kind, crafted torsion / mixed-order / non-canonical
    keys with forged signatures, replays and conflicts across batches -- every per-vote status,
    fire bit, commit event, direct-Verify verdict and per-tx (sum, maj23) equal to the oracle's.
    The 10^8-vote run of the same stream is tools/gate/c4_gate.py."""
    import adversarial as A
    import txflow_amd as T
    ctx = T.Context(max_batch=1 << 17, max_txs=1 << 14, max_validators=256)
    try:
        st = A.run_gate(ctx, 3 * 65536, batch=65536, batches_per_epoch=2, threads=8, log=lambda s: None)
        assert st["mismatches"] == 0, st
        assert st["by_status"].get("ErrVoteInvalidSignature", 0) > 0 and st["events"] > 0
    finally:
        ctx.close()


def test_pipelined_submit_wait_matches_oracle(oracle_lib):
    """txv_submit_votes / txv_wait_votes with three batches in flight (uploads on the copy stream
    overlapping the previous batch's kernels) give exactly the sequential oracle's per-vote
    codes, fire bits and per-tx sums on a C4 adversarial stream (replays / conflicts across
    batches); a fourth batch in flight and waiting out of order are refused."""
    import adversarial as A
    import txflow_amd as T
    ctx = T.Context(max_batch=1 << 16, max_txs=1 << 14, max_validators=256)
    try:
        s = A.C4Stream(ctx, batch=20000, batches_per_epoch=8, oracle_threads=8)
        batches = [s.next_batch()[0] for _ in range(5)]
        exp = []
        for b in batches:
            st, _, fired = s.flow.add_batch(b, 8)
            exp.append(st.astype(np.uint8) | (fired.astype(np.uint8) << 7))
        got, inflight = [], []
        for b in batches:
            if len(inflight) == T.SUBMIT_RING:
                got.append(ctx.wait_votes(inflight.pop(0))[0])
            inflight.append(ctx.submit_votes(b))
            if len(inflight) == T.SUBMIT_RING and len(got) == 0:
                with pytest.raises(T.TxvInfraError):
                    ctx.submit_votes(b)          # a fourth batch in flight is refused
                with pytest.raises(T.TxvInfraError):
                    ctx.wait_votes(inflight[1])  # out of order
        while inflight:
            got.append(ctx.wait_votes(inflight.pop(0))[0])
        for g, e in zip(got, exp):
            assert np.array_equal(g, e), np.nonzero(g != e)[0][:10]
        assert s.check_sets() == 0
        # TxVoteSet.GetVotes: same accepted (validator, signature) per set as the oracle, and each
        # sequence number points at that vote in the submitted stream
        base = np.cumsum([0] + [b.n for b in batches])
        for j in range(0, s.epoch_txs, max(1, s.epoch_txs // 50)):
            h = s.hashes[j].tobytes()
            gv = ctx.get_votes(h)
            ov = s.flow.get_votes(h)
            assert [(v, sg) for v, _, sg in gv] == ov
            for v, seq, sg in gv:
                bi = int(np.searchsorted(base, seq, side="right") - 1)
                b, i = batches[bi], int(seq - base[bi])
                assert b.sig[64 * i:64 * i + 64].tobytes() == sg and b.txhash(i) == h
    finally:
        ctx.close()


@pytest.mark.parametrize("chain", [b"", b"c", b"test_chain_id", b"x" * 127, b"y" * 128, b"z" * 300])
def test_device_signbytes_edge_fields(gpu_ctx, oracle_lib, chain):
    """txv_k_signbytes byte-exact with the oracle's amino encoder on edge fields:
    Height 0 / negative / extremes (omitted field, 8-byte LE), Timestamp at the epoch (omitted),
    negative and extreme seconds (10-byte uvarint), nanos 0 / max, TxHash lengths across uvarint
    and word boundaries, chain ids of 0..300 bytes.  Checked through the device signer (which
    hashes the device-built SignBytes) against RFC 8032 signatures of the oracle's bytes, and
    through the AddVote path (the same votes must verify)."""
    import txflow_amd as T
    rnd = random.Random(len(chain) + 7)
    seeds = [bytes(rnd.getrandbits(8) for _ in range(32)) for _ in range(3)]
    pubs = gpu_ctx.keygen(seeds)
    heights = [0, 1, -1, 2 ** 63 - 1, -2 ** 63, 127, 128, 1 << 40]
    secs = [0, 1, -1, -62135596800, 253402300799, 1_700_000_000, 2 ** 35]
    nanos = [0, 1, 999_999_999, 127, 128]
    hlens = [0, 1, 7, 8, 63, 64, 127, 128, 200, 300]
    votes, signer = [], []
    for i in range(240):
        h = rnd.choice(heights)
        ts = (rnd.choice(secs), rnd.choice(nanos))
        th = "".join(rnd.choice("0123456789ABCDEF") for _ in range(rnd.choice(hlens)))
        votes.append(T.TxVote(Height=h, TxHash=th, Timestamp=ts, ValidatorAddress=b""))
        signer.append(i % 3)
    b = T.VoteBatch.from_votes(votes)
    sigs = gpu_ctx.sign_votes(b, np.array(signer, np.uint32), chain.decode())
    for i, v in enumerate(votes):
        msg = oracle_lib.signbytes(v.Height, v.TxHash.encode(), v.Timestamp[0], v.Timestamp[1], chain)
        assert msg is not None
        assert sigs[i].tobytes() == oracle_lib.sign(seeds[signer[i]], msg), (i, v)
    # the AddVote path builds the same bytes: every vote verifies and is ADDED (one per tx+val)
    ctx = T.Context(max_batch=1 << 12, max_txs=1 << 10, max_validators=8, table_w=8)
    try:
        ctx.set_validators(pubs, [1, 1, 1], chain.decode())
        addrs, _ = ctx.validator_info()
        for v, s, k in zip(votes, sigs, signer):
            v.ValidatorAddress = addrs[k]
            v.Signature = s.tobytes()
        st, _ = ctx.add_votes(T.VoteBatch.from_votes(votes))
        ok = (st & 0x7F)
        assert set(np.unique(ok)) <= {T.ADDED, T.DUPLICATE, T.ERR_NONDETERMINISTIC}, np.unique(ok)
        assert np.count_nonzero(ok == T.ADDED) > 0
        assert not np.any(ok == T.ERR_INVALID_SIGNATURE)
    finally:
        ctx.close()


def test_set_validators_same_keys_new_powers(oracle_lib):
    """txv_set_validators with the keys of the current registry (same order) keeps the validator
    tables (no K0 rebuild) but takes the new powers and resets the TxFlow: the tally then follows
    the new powers exactly (oracle with those powers); the same keys in another order keep their
    tables too (the table pool, test_set_validators_incremental_tables)."""
    import time
    import txflow_amd as T
    rnd = random.Random(35)
    ctx = T.Context(max_batch=1 << 14, max_txs=256, max_validators=16)
    try:
        seeds, pubs, addrs, votes, signer = _signed_set(ctx, T, 8, 600, rnd, n_txs=20)
        b = T.VoteBatch.from_votes(votes)
        od = [dict(height=v.Height, txhash=v.TxHash.encode(), ts_sec=v.Timestamp[0], ts_nanos=v.Timestamp[1],
                   addr=v.ValidatorAddress, sig=v.Signature) for v in votes]
        times = []
        for powers in ([1] * 8, [9, 1, 1, 1, 1, 1, 1, 1], [1, 2, 3, 4, 5, 6, 7, 8]):
            t0 = time.perf_counter()
            ctx.set_validators(pubs, powers, "test_chain_id")
            times.append(time.perf_counter() - t0)
            st, ev = ctx.add_votes(b)
            flow = oracle_lib.Flow(pubs, powers, b"test_chain_id")
            ost, osum, ofired = flow.add_votes(od)
            exp = ost.astype(np.uint8) | (ofired.astype(np.uint8) << 7)
            assert np.array_equal(st, exp), powers
            for v in votes:
                assert ctx.query_tx(v.TxHash.encode()) == flow.query(v.TxHash.encode())
        assert ctx.total_power() == sum([1, 2, 3, 4, 5, 6, 7, 8])
        assert ctx.tables_built == 0
        # a different key order is a different registry (validator indices move), tables kept
        ctx.set_validators(list(reversed(pubs)), [1] * 8, "test_chain_id")
        assert ctx.tables_built == 0
        st, _ = ctx.add_votes(b)
        flow = oracle_lib.Flow(list(reversed(pubs)), [1] * 8, b"test_chain_id")
        ost, _, ofired = flow.add_votes(od)
        assert np.array_equal(st, ost.astype(np.uint8) | (ofired.astype(np.uint8) << 7))
        print("set_validators seconds:", [round(t, 4) for t in times])
    finally:
        ctx.close()


def _pool_model(slots, gens, gen, keys, budget_slots):
    """the table pool's slot policy (runtime.cpp assign_tables) in Python: returns the number of
    keys K0 builds for the set `keys` and updates slots / gens in place"""
    taken = [False] * len(slots)
    held = {k: i for i, k in enumerate(slots) if k is not None}
    vs = [None] * len(keys)
    for i, k in enumerate(keys):
        s = held.get(k)
        if s is not None and not taken[s]:
            vs[i], taken[s] = s, True
    if len(keys) > len(slots):
        cap = max(len(keys), min(budget_slots, len(keys) + max(1, len(keys) // 8))) if slots else len(keys)
        kept = [s for s in range(len(slots)) if taken[s]]
        if kept:
            moved = {s: j for j, s in enumerate(kept)}
            new = [slots[s] for s in kept] + [None] * (cap - len(kept))
            slots[:] = new
            gens[:] = [0] * cap
            vs = [moved[v] if v is not None else None for v in vs]
            taken = [j < len(kept) for j in range(cap)]
        else:
            slots[:] = [None] * cap
            gens[:] = [0] * cap
            vs = [None] * len(keys)
            taken = [False] * cap
    free = sorted((s for s in range(len(slots)) if not taken[s]), key=lambda s: (slots[s] is not None, gens[s]))
    miss = [i for i in range(len(keys)) if vs[i] is None]
    for i, s in zip(miss, free):
        vs[i], slots[s] = s, keys[i]
    for s in vs:
        gens[s] = gen
    return len(miss)


def test_set_validators_incremental_tables(oracle_lib):
    """txv_set_validators keeps each key's tables in a slot of the context's pool: a new set that
    re-orders, drops, adds (growing the pool) or brings back validators builds K0 only for keys
    no slot holds (counted by txv_validator_tables_built, predicted by a model of the slot
    policy), and every set's verdicts -- votes of its validators, of validators outside it and
    with corrupted signatures -- equal the oracle TxFlow's for that set."""
    import hashlib
    import time

    import txflow_amd as T
    rnd = random.Random(36)
    ctx = T.Context(max_batch=1 << 14, max_txs=512, max_validators=24)
    try:
        seeds = [bytes(rnd.getrandbits(8) for _ in range(32)) for _ in range(14)]
        pubs = ctx.keygen(seeds)
        addr = [hashlib.sha256(p).digest()[:20] for p in pubs]
        hashes = ["".join(rnd.choice("0123456789ABCDEF") for _ in range(64)) for _ in range(30)]
        sets = [list(range(8)), list(range(7, -1, -1)), [0, 1, 2, 3, 4, 5, 8, 9], [0, 1, 2, 3, 4, 5, 8, 9, 6],
                [9, 8, 6, 5, 4, 3, 2, 1, 0, 7], [3, 1, 10, 11], list(range(10)), [12, 13] + list(range(10)),
                [13, 0]]
        slots, gens = [], []
        budget_slots = (112 << 30) // int(_table_mb(20) * 2 ** 20)
        times = []
        for gen, ks in enumerate(sets, 1):
            powers = [1 + (k % 4) for k in ks]
            t0 = time.perf_counter()
            ctx.set_validators([pubs[k] for k in ks], powers, "test_chain_id")
            times.append(round(time.perf_counter() - t0, 4))
            exp_built = _pool_model(slots, gens, gen, [pubs[k] for k in ks], budget_slots)
            assert ctx.tables_built == exp_built, (gen, ks, ctx.tables_built, exp_built)
            got_addr, ok = ctx.validator_info()
            assert ok.all() and [bytes(a) for a in got_addr] == [addr[k] for k in ks]
            votes, signer = [], []
            for i in range(900):
                k = rnd.choice(ks) if i % 9 else rnd.randrange(14)        # some from outside the set
                votes.append(T.TxVote(Height=1, TxHash=rnd.choice(hashes), Timestamp=(1_700_000_000, i + 1),
                                      ValidatorAddress=addr[k], Signature=b""))
                signer.append(k)
            ctx.keygen(seeds)                                         # sign with key index k
            sigs = ctx.sign_votes(T.VoteBatch.from_votes(votes), np.array(signer, np.uint32), "test_chain_id")
            for i, (v, s) in enumerate(zip(votes, sigs)):
                s = bytearray(s.tobytes())
                if i % 11 == 3:
                    s[rnd.randrange(64)] ^= 1 << rnd.randrange(8)
                v.Signature = bytes(s)
            st, _ = ctx.add_votes(T.VoteBatch.from_votes(votes))
            flow = oracle_lib.Flow([pubs[k] for k in ks], powers, b"test_chain_id")
            od = [dict(height=v.Height, txhash=v.TxHash.encode(), ts_sec=v.Timestamp[0], ts_nanos=v.Timestamp[1],
                       addr=v.ValidatorAddress, sig=v.Signature) for v in votes]
            ost, _, ofired = flow.add_votes(od)
            exp = ost.astype(np.uint8) | (ofired.astype(np.uint8) << 7)
            bad = np.nonzero(st != exp)[0]
            assert len(bad) == 0, (gen, [(int(i), int(st[i]), int(exp[i])) for i in bad[:10]])
            assert ((st & 0x7F) == T.ADDED).sum() >= 2 * len(ks)
        print("set_validators seconds:", times, "slots:", len(slots))
    finally:
        ctx.close()


def test_event_ranks_after_flow_reallocated(oracle_lib):
    """the fused status / event kernel (batches of <= 128 scan tiles) ranks commit events
    by a look-back over words tagged with the batch stamp, and txv_set_validators restarts the
    stamps (alloc_tally).  After each restart, new batches -- other votes, so other event counts
    per tile -- must still list their commit events exactly in arrival order: the words an earlier
    run left under the same tag are cleared when a new tag cycle starts (runtime.cpp run_slot)."""
    import txflow_amd as T
    ctx = T.Context(max_batch=1 << 15, max_txs=1 << 12, max_validators=16)
    try:
        rnd = random.Random(505)
        seeds, pubs, addrs, votes, signer = _signed_set(ctx, T, 8, 36000, rnd, n_txs=2500)
        powers = [1 + (i % 3) for i in range(len(pubs))]
        for rep in range(3):
            ctx.set_validators(pubs, powers, "test_chain_id")     # a new TxFlow: stamps start again
            flow = oracle_lib.Flow(pubs, powers, b"test_chain_id")
            order = list(range(len(votes)))
            rnd.shuffle(order)
            order = order[:24000 - 4000 * rep]
            committed = set()
            for lo in range(0, len(order), 12000):
                part = [votes[i] for i in order[lo:lo + 12000]]
                st, ev = ctx.add_votes(T.VoteBatch.from_votes(part))
                ost, _, ofired = flow.add_votes([dict(height=v.Height, txhash=v.TxHash.encode(), ts_sec=v.Timestamp[0],
                                                      ts_nanos=v.Timestamp[1], addr=v.ValidatorAddress, sig=v.Signature)
                                                 for v in part])
                exp = ost.astype(np.uint8) | (ofired.astype(np.uint8) << 7)
                assert np.array_equal(st, exp), f"rep {rep} batch {lo}"
                first = []
                for i in np.nonzero(ofired)[0]:
                    h = part[int(i)].TxHash
                    if h not in committed:
                        committed.add(h)
                        first.append(int(i))
                assert [int(e["vote_index"]) for e in ev] == first, f"rep {rep} batch {lo}: event order"
                assert len(first) > 50
    finally:
        ctx.close()

"""TxVoteMessage wire decode (Reactor.Receive / decodeMsg, txvotepool/reactor.go:170-190, 273-291).

CPU: the oracle codec (oracle/wire.c) round-trips the reference's encoder output, reproduces the
reference's pinned message size (txMessageSize = Size() + 1 + 4 + 1, txvotepool/txvotepool_test.go:
301-303, asserted against the encoded length at :344-345) and the restated amino rules case by case.
The amino decoder itself (go-amino v0.15.1, external) is not in the container: beyond those pins the
decode verdicts are PARITY UNPINNED (restated rules, oracle/wire.c header).

GPU: txv_decode_msgs (kernels_wire.hip) against the oracle on every field of every message of a
mixed canonical / non-canonical / corrupted stream (staged-in-LDS and global-memory blocks, too-large
and empty messages), txv_pool_receive against decode + the oracle pool, and decoded votes through
txv_add_votes against the original votes.
"""
import hashlib
import random

import numpy as np
import pytest

import oracle as O
import wire_gen as G

MAX = 1 << 20


@pytest.fixture(scope="module")
def wctx():
    """one small context (radix-16 tables): the decode does not depend on the verify windows"""
    import txflow_amd as T
    ctx = T.Context(max_batch=1 << 16, max_txs=1 << 12, max_validators=16, table_w=4)
    yield ctx
    ctx.close()


def enc(height=1, txhash=b"AB" * 32, ts=(1_700_000_000, 5), addr=b"\x01" * 20, sig=b"\x02" * 64, txkey=bytes(32)):
    return O.wire_encode(height, txhash, ts[0], ts[1], addr, sig, txkey)


def dec(m, mx=MAX):
    return O.wire_decode(m, mx)


# ------------------------------------------------------------------ oracle (CPU)
def test_prefix_bytes():
    """nameToDisfix: SHA-256(name), zero bytes skipped, 3 disambiguation + 4 prefix bytes.  The same
    derivation gives tendermint's published PubKeyEd25519 prefix 0x1624DE64."""
    d, p = O.wire_prefix()
    h = hashlib.sha256(b"tendermint/txvotepool/TxVoteMessage").digest()
    assert h[0] != 0 and d == h[:3] and h[3] != 0 and p == h[3:7]
    assert (d.hex(), p.hex()) == ("67af1f", "d736a47f")
    assert hashlib.sha256(b"tendermint/PubKeyEd25519").digest()[3:7].hex() == "1624de64"


def test_roundtrip_and_pinned_message_size():
    rng = random.Random(7)
    for _ in range(3000):
        v = G.rand_vote(rng)
        m = G.message(v, rng, False)
        st, f = dec(m)
        assert st == O.WIRE_OK
        assert (f["height"], f["txhash"], f["txkey"], f["ts_sec"], f["ts_nanos"], f["addr"], f["sig"]) == \
            (v["height"], v["txhash"], v["txkey"], v["ts"][0], v["ts"][1], v["addr"], v["sig"])
        size = O.txvote_size(v["height"], len(v["txhash"]), v["ts"][0], v["ts"][1], len(v["addr"]), len(v["sig"]))
        if size < 128:   # txMessageSize assumes a one-byte length prefix
            assert len(m) == size + 1 + 4 + 1
        else:
            assert len(m) == size + 1 + 4 + len(G.uv(size))


def test_reference_max_msg_size_cases():
    """TestMempoolMaxMsgSize (txvotepool_test.go:305-355) vote shape: TxVote{i, TxHash(tx), TxKey(tx),
    now, nil, tx} -- the encoded message is txMessageSize(vote) bytes, and decodeMsg rejects it as
    ErrTxTooLarge exactly when it exceeds MaxMsgBytes."""
    for i, ln in enumerate([10, 100, 126]):
        tx = bytes([i % 256]) * ln
        th = hashlib.sha256(tx).hexdigest().upper().encode()
        m = enc(height=i, txhash=th, txkey=hashlib.sha256(tx).digest(), addr=b"", sig=tx)
        size = O.txvote_size(i, len(th), 1_700_000_000, 5, 0, ln)
        assert len(m) == size + len(G.uv(size)) + 5
        assert dec(m, len(m))[0] == O.WIRE_OK
        assert dec(m, len(m) - 1)[0] == O.WIRE_TOO_LARGE


def body_msg(body: bytes, framing=None, ext=0, tail=b""):
    return (framing or G.PREFIX) + G.key(1, 2) + G.lp(body, ext) + tail


def test_rules():
    K, uv, lp = G.key, G.uv, G.lp
    good = K(1, 0) + uv(1) + K(2, 2) + lp(b"AB") + K(3, 2) + lp(bytes(32)) + K(4, 2) + lp(K(1, 0) + uv(5)) + \
        K(5, 2) + lp(b"\x01" * 20) + K(6, 2) + lp(b"\x02" * 64)
    assert dec(body_msg(good))[0] == O.WIRE_OK
    assert dec(b"")[0] == O.WIRE_NIL
    assert dec(G.PREFIX)[0] == O.WIRE_OK                               # no fields: zero TxVoteMessage
    assert dec(G.PREFIX[:3])[0] == O.WIRE_ERR_DECODE                   # < 4 bytes
    assert dec(b"\x00" + G.DISAMB + G.PREFIX + K(1, 2) + lp(good))[0] == O.WIRE_OK   # disfix framing
    assert dec(b"\x00" + G.DISAMB[:2] + b"\x00" + G.PREFIX + K(1, 2) + lp(good))[0] == O.WIRE_ERR_DECODE
    assert dec(b"\x00" + G.DISAMB + G.PREFIX[:3])[0] == O.WIRE_ERR_DECODE           # disfix < 8 bytes
    assert dec(b"\x01" + G.PREFIX[1:] + K(1, 2) + lp(good))[0] == O.WIRE_ERR_DECODE  # unknown prefix
    assert dec(body_msg(good, tail=b"\x00"))[0] == O.WIRE_ERR_DECODE   # trailing byte: key 0 <= last
    assert dec(body_msg(good, tail=K(2, 0) + uv(9)))[0] == O.WIRE_OK   # extra message field
    assert dec(body_msg(good, tail=K(1, 2) + lp(b"")))[0] == O.WIRE_ERR_DECODE   # repeated field 1
    # TxVote body rules
    assert dec(body_msg(K(1, 0) + uv(1) + K(1, 0) + uv(2)))[0] == O.WIRE_ERR_DECODE   # repeated
    assert dec(body_msg(K(2, 2) + lp(b"A") + K(1, 0) + uv(2)))[0] == O.WIRE_ERR_DECODE  # out of order
    assert dec(body_msg(K(1, 2) + lp(b"A")))[0] == O.WIRE_ERR_DECODE   # wrong typ3 for Height
    st, f = dec(body_msg(K(1, 0, 3) + uv(7, 2)))                        # overlong key and value
    assert st == O.WIRE_OK and f["height"] == 7
    assert dec(body_msg(K(1, 0) + b"\x80" * 10 + b"\x01"))[0] == O.WIRE_ERR_DECODE   # 11-byte varint
    assert dec(body_msg(K(1, 0) + b"\xff" * 9 + b"\x02"))[0] == O.WIRE_ERR_DECODE    # 10th byte > 1
    st, f = dec(body_msg(K(1, 0) + b"\xff" * 9 + b"\x01"))
    assert st == O.WIRE_OK and f["height"] == -1
    assert dec(body_msg(K(3, 2) + lp(bytes(31))))[0] == O.WIRE_ERR_DECODE          # TxKey length 31
    assert dec(body_msg(K(3, 2) + lp(bytes(33))))[0] == O.WIRE_ERR_DECODE
    assert dec(body_msg(K(2, 2) + uv(5) + b"ab"))[0] == O.WIRE_ERR_DECODE           # short string
    for t, val, ok in [(0, uv(3), True), (1, bytes(8), True), (2, lp(b"x"), True), (5, bytes(4), True),
                       (3, b"", False), (4, b"", False), (6, b"", False), (7, b"", False), (1, bytes(7), False)]:
        st, _ = dec(body_msg(good + K(9, t) + val))
        assert (st == O.WIRE_OK) == ok, (t, ok)
    assert dec(body_msg(good + K(9, 0) + uv(1) + K(9, 0) + uv(1)))[0] == O.WIRE_ERR_DECODE
    assert dec(body_msg(good + K((1 << 29) - 1, 0) + uv(1)))[0] == O.WIRE_OK
    assert dec(body_msg(good + uv((1 << 29) << 3)))[0] == O.WIRE_ERR_DECODE         # field num > 2^29-1
    # absent fields keep their defaults; a later field is read again for the next one
    st, f = dec(body_msg(K(6, 2) + lp(b"\x05" * 64)))
    assert st == O.WIRE_OK and f["sig"] == b"\x05" * 64 and f["height"] == 0 and f["txkey"] == bytes(32)
    # time body
    tb = lambda b: body_msg(K(4, 2) + lp(b))
    assert dec(tb(K(2, 0) + uv(10**9)))[0] == O.WIRE_ERR_DECODE
    assert dec(tb(K(2, 0) + uv(10**9 - 1)))[1]["ts_nanos"] == 10**9 - 1
    assert dec(tb(K(1, 0) + uv(253402300800)))[0] == O.WIRE_ERR_DECODE
    assert dec(tb(K(1, 0) + uv(-62135596801)))[0] == O.WIRE_ERR_DECODE
    assert dec(tb(K(1, 0) + uv(-62135596800)))[1]["ts_sec"] == -62135596800
    # nanos first: seconds stay 0, the nanos are read, the rest of the body is left unread and the
    # TxVote decoder reads it again as its own next key: here K(1,0) (Height) after Timestamp -> error
    assert dec(tb(K(2, 0) + uv(3) + K(1, 0) + uv(4)))[0] == O.WIRE_ERR_DECODE
    # unread time bytes that parse as a later TxVote field are taken as that field
    st, f = dec(tb(K(1, 0) + uv(4) + K(2, 0) + uv(3) + K(6, 2) + lp(b"\x07" * 2)))
    assert st == O.WIRE_OK and (f["ts_sec"], f["ts_nanos"], f["sig"]) == (4, 3, b"\x07\x07")
    # non-minimal nested TxVote length: the message decoder advances by UvarintSize(len) + len,
    # one byte short, and reads the body's last byte again as a key
    m = body_msg(K(6, 2) + lp(b"\x02" * 63 + b"\x10"), ext=1)   # last body byte 0x10 = key(2, 0)
    st, f = dec(m + b"")
    assert st == O.WIRE_ERR_DECODE                               # ... whose varint value is missing
    st, f = dec(body_msg(K(6, 2) + lp(b"\x02" * 63 + b"\x10"), ext=1, tail=b"\x05"))
    assert st == O.WIRE_OK and f["sig"] == b"\x02" * 63 + b"\x10"


def test_fuzz_no_crash_and_determinism():
    msgs = G.messages(3000, seed=11)
    a = [dec(m) for m in msgs]
    b = [dec(m) for m in msgs]
    assert a == b
    counts = np.bincount([s for s, _ in a], minlength=4)
    assert counts[O.WIRE_OK] > 1500 and counts[O.WIRE_ERR_DECODE] > 300 and counts[O.WIRE_NIL] > 0


# ------------------------------------------------------------------ GPU parity
def oracle_decode_all(wb, mx):
    out = []
    for i in range(wb.n):
        out.append(dec(wb.msg(i), mx))
    return out


def check_decoded(d, wb, ref):
    """mismatching messages (sig_off is only defined for a non-empty signature)"""
    mism = 0
    for i, (st, f) in enumerate(ref):
        if int(d.status[i]) != st:
            mism += 1
            continue
        if st != O.WIRE_OK:
            assert d.height[i] == 0 and d.sig_len[i] == 0 and not d.sig[i].any(), i
            continue
        o = int(wb.off[i])
        al, sl = len(f["addr"]), len(f["sig"])
        got = (int(d.height[i]), int(d.txhash_off[i]) - o, int(d.txhash_len[i]), d.txkey[i].tobytes(),
               int(d.ts_sec[i]), int(d.ts_nanos[i]), int(d.addr_len[i]), d.addr[i].tobytes(),
               int(d.sig_len[i]), (int(d.sig_off[i]) - o) if int(d.sig_len[i]) else 0, d.sig[i].tobytes())
        exp = (f["height"], f["txhash_off"], len(f["txhash"]), f["txkey"], f["ts_sec"], f["ts_nanos"], al,
               f["addr"][:20] + bytes(20 - min(al, 20)), sl, f["sig_off"] if sl else 0,
               f["sig"][:64] + bytes(64 - min(sl, 64)))
        if got != exp:
            mism += 1
    return mism


@pytest.mark.gpu
@pytest.mark.parametrize("mx", [MAX, 300])
def test_gpu_decode_parity(wctx, mx):
    import txflow_amd as T
    msgs = G.messages(40000, seed=2024 + mx)
    wb = T.WireBatch(msgs)
    d = wctx.decode_msgs(wb, mx)
    ref = oracle_decode_all(wb, mx)
    assert check_decoded(d, wb, ref) == 0
    st = np.bincount(d.status[:wb.n], minlength=4)
    assert st[T.WIRE_OK] > 10000 and st[T.WIRE_ERR_DECODE] > 1000 and st[T.WIRE_NIL] > 0
    if mx == 300:
        assert st[T.WIRE_TOO_LARGE] > 1000


@pytest.mark.gpu
def test_gpu_decode_scattered_offsets(wctx):
    """messages in a shuffled order inside the buffer, with gaps: spans exceed the LDS stage and
    the blocks fall back to global memory"""
    import txflow_amd as T
    msgs = G.messages(5000, seed=99, p_mutate=0.1)
    rng = random.Random(5)
    order = list(range(len(msgs)))
    rng.shuffle(order)
    buf, off = bytearray(), np.zeros(len(msgs), np.uint64)
    for i in order:
        buf += bytes(rng.randrange(0, 7))
        off[i] = len(buf)
        buf += msgs[i]
    wb = T.WireBatch(wire=np.frombuffer(bytes(buf), np.uint8), off=off,
                     length=np.array([len(m) for m in msgs], np.uint32))
    d = wctx.decode_msgs(wb)
    assert check_decoded(d, wb, oracle_decode_all(wb, MAX)) == 0


@pytest.mark.gpu
def test_gpu_decode_edges(wctx):
    import txflow_amd as T
    d = wctx.decode_msgs(T.WireBatch([]))
    assert d.n == 0
    msgs = [b"", G.PREFIX, enc(), enc()[:-1], b"\x00" + G.DISAMB + enc(), b"\x00" + G.DISAMB[:2] + enc()]
    wb = T.WireBatch(msgs)
    d = wctx.decode_msgs(wb)
    assert list(d.status[:6]) == [T.WIRE_NIL, T.WIRE_OK, T.WIRE_OK, T.WIRE_ERR_DECODE, T.WIRE_OK, T.WIRE_ERR_DECODE]
    assert check_decoded(d, wb, oracle_decode_all(wb, MAX)) == 0
    with pytest.raises(T.TxvInfraError):   # message outside the buffer: refused on the host
        bad = T.WireBatch(wire=np.zeros(10, np.uint8), off=np.array([8], np.uint64), length=np.array([4], np.uint32))
        wctx.decode_msgs(bad)


@pytest.mark.gpu
def test_gpu_pool_receive(wctx):
    """Reactor.Receive over a stream with duplicates: decode + CheckTxWithInfo vs the oracle"""
    import txflow_amd as T
    rng = random.Random(3)
    base = G.messages(3000, seed=77, p_noncanon=0.2, p_mutate=0.2)
    msgs = base + [base[rng.randrange(len(base))] for _ in range(1500)]
    wb = T.WireBatch(msgs)
    pool = T.TxVotePool(wctx, size=2500, cache_size=2000, max_msg_bytes=4096)
    ws, ps = pool.receive(wb)
    op = O.Pool(size=2500, cache_size=2000, max_msg_bytes=4096)
    for i, m in enumerate(msgs):
        st, f = dec(m, 4096)
        assert ws[i] == st, i
        if st != O.WIRE_OK:
            assert ps[i] == T.POOL_NOT_CHECKED
            continue
        ov = dict(height=f["height"], txhash=f["txhash"], ts_sec=f["ts_sec"], ts_nanos=f["ts_nanos"],
                  addr=f["addr"], sig=f["sig"])
        assert ps[i] == op.check([ov])[0], i
    assert pool.Size() == op.size() and pool.TxsBytes() == op.txs_bytes()


@pytest.mark.gpu
def test_gpu_decoded_votes_through_txflow(wctx):
    """signed votes -> wire -> GPU decode -> txv_add_votes gives the statuses of the original votes"""
    import txflow_amd as T
    rng = random.Random(8)
    seeds = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(6)]
    pubs = wctx.keygen(seeds)
    wctx.set_validators(pubs, [1, 2, 3, 1, 1, 1], "test_chain_id")
    addrs, _ = wctx.validator_info()
    votes, signer = [], []
    for t in range(40):
        h = hashlib.sha256(b"tx%d" % t).hexdigest().upper()
        for v in range(6):
            votes.append(T.TxVote(Height=1, TxHash=h, Timestamp=(1_700_000_000, 1 + len(votes)),
                                  ValidatorAddress=addrs[v]))
            signer.append(v)
    sigs = wctx.sign_votes(T.VoteBatch.from_votes(votes), np.array(signer, np.uint32), "test_chain_id")
    for v, s in zip(votes, sigs):
        v.Signature = s.tobytes()
    for i in range(0, len(votes), 7):   # some corrupt signatures
        s = bytearray(votes[i].Signature); s[5] ^= 1; votes[i].Signature = bytes(s)
    rng.shuffle(votes)
    wire = [O.wire_encode(v.Height, v.TxHash.encode(), v.Timestamp[0], v.Timestamp[1], v.ValidatorAddress,
                          v.Signature, v.TxKey) for v in votes]
    d = wctx.decode_msgs(T.WireBatch(wire))
    assert (d.status[:len(votes)] == T.WIRE_OK).all()
    wctx.reset_flow()
    st_wire, _ = wctx.add_votes(d.batch())
    wctx.reset_flow()
    st_direct, _ = wctx.add_votes(T.VoteBatch.from_votes(votes))
    assert (st_wire == st_direct).all()
    assert (st_wire & 0x7F == T.ADDED).sum() > 150


def test_host_encoder_matches_oracle():
    """txv_encode_msgs (host C++, the sender's MarshalBinaryBare) == the oracle encoder, byte for byte"""
    import txflow_amd as T
    rng = random.Random(21)
    votes, keys = [], []
    while len(votes) < 400:
        v = G.rand_vote(rng)
        if len(v["addr"]) > 20 or len(v["sig"]) > 64:
            continue
        votes.append(T.TxVote(Height=v["height"], TxHash=v["txhash"].decode(), Timestamp=v["ts"],
                              ValidatorAddress=v["addr"], Signature=v["sig"] or None))
        keys.append(v["txkey"])
    wb = T.encode_msgs(T.VoteBatch.from_votes(votes), np.frombuffer(b"".join(keys), np.uint8))
    for i, v in enumerate(votes):
        exp = O.wire_encode(v.Height, v.TxHash.encode(), v.Timestamp[0], v.Timestamp[1], v.ValidatorAddress,
                            v.Signature or b"", keys[i])
        assert wb.msg(i) == exp, i
    with pytest.raises(T.TxvInfraError):   # amino rejects the time: MustMarshalBinaryBare panics
        T.encode_msgs(T.VoteBatch.from_votes([T.TxVote(Height=1, TxHash="A", Timestamp=(1 << 40, 0))]))


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["sync", "pipelined", "pipelined_registered", "three_stage", "sync_device",
                                  "three_stage_device", "four_stage", "four_stage_device"])
def test_gpu_ingest_chain_matches_oracle(mode):
    """txv_ingest_msgs (Reactor.Receive -> CheckTxWithInfo -> TryAddVote with the decoded votes
    kept in HBM) over batches of received messages against the oracle's decoder, pool and
    sequential TxFlow: signed votes, exact replays of earlier messages (ErrTxInCache while the
    bounded LRU still holds their key, DUPLICATE once it evicted it), conflicting signatures,
    corrupted ones, a 65-byte signature (its key hashes all 65 bytes), non-canonical framings and
    undecodable / oversize messages.  Per message: wire status, pool status, flow status + fired
    bit; commit events by message index; the pool and TxFlow state at the end.
    mode "sync": three batches through txv_ingest_msgs; "pipelined": five batches through
    txv_ingest_submit / txv_ingest_wait with two in flight (batch k+1 decoded and pool-checked
    while batch k's TxFlow chain runs; reactor.go:170-190 -> txvotepool.go:187-261 ->
    txflow/service.go:123-166); "pipelined_registered": the same with the receive buffers
    registered (txv_host_register: the wire bytes are DMA'd without a staging copy); "three_stage":
    txv_ingest_decode / txv_ingest_admit / txv_ingest_wait with three batches in the ring (batch
    k+2 decoded while k+1 is admitted and k's TxFlow chain runs); "four_stage": the admission in
    its two halves (txv_ingest_admit_submit / _finish), batches k+1 and k+2 submitted to the pool
    before batch k's statuses are collected; "*_device": the same with the
    pool's cache in HBM (TXV_POOL_DEVICE_CACHE: CheckTx decided on the GPU from the keys, sizes and
    decode statuses the decode left there)."""
    import txflow_amd as T
    rng = random.Random(31)
    ctx = T.Context(max_batch=1 << 14, max_txs=1 << 12, max_validators=16)
    try:
        seeds = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(7)]
        powers = [1, 2, 3, 1, 1, 2, 1]
        pubs = ctx.keygen(seeds)
        ctx.set_validators(pubs, powers, "test_chain_id")
        addrs, _ = ctx.validator_info()
        votes, signer = [], []
        for t in range(60):
            h = hashlib.sha256(b"ingest%d" % t).hexdigest().upper()
            tk = hashlib.sha256(b"key%d" % t).digest()
            for v in range(7):
                votes.append(T.TxVote(Height=1 + (t % 3 == 0), TxHash=h, TxKey=tk,
                                      Timestamp=(1_700_000_000, 1 + len(votes)), ValidatorAddress=addrs[v]))
                signer.append(v)
        sigs = ctx.sign_votes(T.VoteBatch.from_votes(votes), np.array(signer, np.uint32), "test_chain_id")
        for v, s in zip(votes, sigs):
            v.Signature = s.tobytes()

        def wire_of(v):
            return O.wire_encode(v.Height, v.TxHash.encode(), v.Timestamp[0], v.Timestamp[1], v.ValidatorAddress,
                                 v.Signature, v.TxKey)

        order = list(range(len(votes)))
        rng.shuffle(order)
        stream = []
        for j in order:
            v = votes[j]
            if rng.random() < 0.05:                       # a corrupted copy ahead of the vote itself
                c = T.TxVote(Height=v.Height, TxHash=v.TxHash, TxKey=v.TxKey, Timestamp=v.Timestamp,
                             ValidatorAddress=v.ValidatorAddress, Signature=v.Signature[:40] + bytes([v.Signature[40] ^ 1]) + v.Signature[41:])
                stream.append(wire_of(c))
            stream.append(wire_of(v))
            r = rng.random()
            if r < 0.08:                                  # a replay of an earlier message
                stream.append(stream[rng.randrange(len(stream))])
            elif r < 0.14:                                # same validator + tx, another signature
                c = T.TxVote(Height=v.Height, TxHash=v.TxHash, TxKey=v.TxKey, Timestamp=v.Timestamp,
                             ValidatorAddress=v.ValidatorAddress, Signature=bytes([v.Signature[0] ^ 4]) + v.Signature[1:])
                stream.append(wire_of(c))
            elif r < 0.17:                                # a 65-byte signature
                c = T.TxVote(Height=v.Height, TxHash=v.TxHash, TxKey=v.TxKey, Timestamp=v.Timestamp,
                             ValidatorAddress=v.ValidatorAddress, Signature=v.Signature + b"\x07")
                stream.append(wire_of(c))
        junk = G.messages(120, seed=5, p_noncanon=0.3, p_mutate=0.5) + [b"", b"\x01" * 5000]
        for m in junk:
            stream.insert(rng.randrange(len(stream) + 1), m)
        max_msg = 4096
        pool = T.TxVotePool(ctx, size=1 << 20, cache_size=150, max_txs_bytes=1 << 30, max_msg_bytes=max_msg,
                            device_cache=mode.endswith("_device"))
        mode = mode.replace("_device", "")
        opool = O.Pool(size=1 << 20, cache_size=150, max_txs_bytes=1 << 30, max_msg_bytes=max_msg)
        flow = O.Flow(pubs, powers, b"test_chain_id")
        nb = 3 if mode == "sync" else 5
        committed, cuts = set(), [len(stream) * k // nb for k in range(nb + 1)]
        seen = {"cache": 0, "dup": 0, "fired": 0, "undecoded": 0, "nondet": 0, "invalid": 0}
        parts = [stream[cuts[b]:cuts[b + 1]] for b in range(nb)]
        if mode == "sync":
            results = [pool.ingest(T.WireBatch(part)) for part in parts]
        elif mode == "three_stage":
            wbs = [T.WireBatch(part) for part in parts]
            for w in wbs:
                ctx.host_register(w.wire)
            results, dec, adm = [None] * nb, [], []
            for k, w in enumerate(wbs):
                dec.append((k, pool.ingest_decode(w)))
                if len(dec) == 2:
                    kk, tk = dec.pop(0)
                    adm.append((kk, pool.ingest_admit(tk)))
                if len(adm) == 2:
                    kk, tk = adm.pop(0)
                    results[kk] = pool.ingest_wait(tk)
            for kk, tk in dec:
                adm.append((kk, pool.ingest_admit(tk)))
            for kk, tk in adm:
                results[kk] = pool.ingest_wait(tk)
        elif mode == "four_stage":
            wbs = [T.WireBatch(part) for part in parts]
            for w in wbs:
                ctx.host_register(w.wire)
            results, ring = [None] * nb, []
            for k, w in enumerate(wbs):
                tk = pool.ingest_decode(w)
                ring.append((k, pool.ingest_admit_submit(tk)))
                if len(ring) == 3:
                    kk, tk = ring.pop(0)
                    results[kk] = pool.ingest_wait(pool.ingest_admit_finish(tk))
            for kk, tk in ring:
                results[kk] = pool.ingest_wait(pool.ingest_admit_finish(tk))
        else:
            results, inflight = [], []
            wbs = [T.WireBatch(part) for part in parts]
            if mode == "pipelined_registered":
                for w in wbs:
                    ctx.host_register(w.wire)
            for w in wbs:
                inflight.append(pool.ingest_submit(w))
                if len(inflight) == 2:
                    results.append(pool.ingest_wait(inflight.pop(0)))
            while inflight:
                results.append(pool.ingest_wait(inflight.pop(0)))
            assert len(results) == nb
        for b in range(nb):
            part = parts[b]
            ws, ps, fs, ev = results[b]
            exp_fired = []
            for i, m in enumerate(part):
                st, f = O.wire_decode(m, max_msg)
                assert ws[i] == st, (b, i)
                if st != O.WIRE_OK:
                    seen["undecoded"] += 1
                    assert ps[i] == T.POOL_NOT_CHECKED and fs[i] == T.FLOW_NOT_ADDED, (b, i)
                    continue
                ov = dict(height=f["height"], txhash=f["txhash"], ts_sec=f["ts_sec"], ts_nanos=f["ts_nanos"],
                          addr=f["addr"], sig=f["sig"])
                op = opool.check([ov])[0]
                assert ps[i] == op, (b, i, int(ps[i]), int(op))
                if op != T.POOL_OK:
                    seen["cache"] += op == T.POOL_ERR_IN_CACHE
                    assert fs[i] == T.FLOW_NOT_ADDED, (b, i)
                    continue
                ost, _, ofired = flow.add_votes([ov])
                exp = int(ost[0]) | (int(ofired[0]) << 7)
                assert fs[i] == exp, (b, i, int(fs[i]), exp)
                seen["dup"] += ost[0] == T.DUPLICATE
                seen["nondet"] += ost[0] == 5
                seen["invalid"] += ost[0] == 6
                if ofired[0] and f["txhash"] not in committed:
                    committed.add(f["txhash"])
                    exp_fired.append(i)
                seen["fired"] += int(ofired[0])
            assert sorted(int(e["vote_index"]) for e in ev) == exp_fired, b
        assert pool.Size() == opool.size() and pool.TxsBytes() == opool.txs_bytes()
        assert np.array_equal(pool.cache_keys(), opool.cache_keys())      # the LRU order too
        for t in range(60):
            h = hashlib.sha256(b"ingest%d" % t).hexdigest().upper().encode()
            assert ctx.query_tx(h) == flow.query(h)
        assert all(seen[k] > 0 for k in seen), seen
        pool.close()
    finally:
        ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("device_cache", [False, True], ids=["host-cache", "device-cache"])
def test_gpu_ingest_capacity_overflow_reports_not_run(device_cache):
    """a TxFlow capacity overflow after the pool stage must not strand the admitted
    votes silently.  A context with room for 8 TxVoteSets receives messages for 40 txs: the call
    fails with TXV_ECAPACITY, every pool-admitted message carries FLOW_NOT_RUN (in the pool, not in
    TxFlow: resending one is ErrTxInCache), the rest FLOW_NOT_ADDED; after txv_reset_flow the
    admitted votes re-fed through txv_add_votes (from txv_decode_msgs' columns) are ADDED."""
    import txflow_amd as T
    rng = random.Random(7)
    ctx = T.Context(max_batch=1 << 12, max_txs=8, max_validators=8)
    try:
        seeds = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(4)]
        pubs = ctx.keygen(seeds)
        ctx.set_validators(pubs, [1, 1, 1, 1], "test_chain_id")
        addrs, _ = ctx.validator_info()
        votes, signer = [], []
        for t in range(40):
            h = hashlib.sha256(b"over%d" % t).hexdigest().upper()
            for v in range(2):
                votes.append(T.TxVote(Height=1, TxHash=h, Timestamp=(1_700_000_000, 1 + len(votes)),
                                      ValidatorAddress=addrs[v]))
                signer.append(v)
        sigs = ctx.sign_votes(T.VoteBatch.from_votes(votes), np.array(signer, np.uint32), "test_chain_id")
        wire = [O.wire_encode(v.Height, v.TxHash.encode(), v.Timestamp[0], v.Timestamp[1], v.ValidatorAddress,
                              s.tobytes(), b"\0" * 32) for v, s in zip(votes, sigs)]
        wire.insert(5, b"\x01\x02")                       # undecodable: never reaches the pool
        pool = T.TxVotePool(ctx, size=1 << 12, cache_size=1 << 12, max_txs_bytes=1 << 30, max_msg_bytes=4096,
                            device_cache=device_cache)
        with pytest.raises(T.IngestError) as ei:
            pool.ingest(T.WireBatch(wire))
        ws, ps, fs, _ = ei.value.result
        assert ei.value.rc == -28                          # TXV_ECAPACITY
        adm = (ws == T.WIRE_OK) & (ps == T.POOL_OK)
        assert adm.sum() == len(votes)
        assert (fs[adm] == T.FLOW_NOT_RUN).all() and (fs[~adm] == T.FLOW_NOT_ADDED).all()
        assert pool.Size() == len(votes)
        ws2, ps2 = pool.receive(T.WireBatch(wire[:3]))   # resent: in the cache already
        assert (ps2 == T.POOL_ERR_IN_CACHE).all()
        # the caller's recovery: a fresh TxFlow with room, the admitted votes re-fed
        ctx.reset_flow()
        with pytest.raises(T.TxvInfraError):              # still over capacity in one batch
            ctx.add_votes(T.VoteBatch.from_votes(votes), ev_cap=len(votes))
        ctx.reset_flow()
        for k in range(0, 16, 2):                         # 8 txs fit
            v2 = votes[k:k + 2]
            for v, s in zip(v2, sigs[k:k + 2]):
                v.Signature = s.tobytes()
            st, _ = ctx.add_votes(T.VoteBatch.from_votes(v2), ev_cap=2)
            assert ((st & 0x7F) == T.ADDED).all()
        pool.close()
    finally:
        ctx.close()

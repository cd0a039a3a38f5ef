"""Every BASELINE.json config as a -m gpu oracle-parity test, plus the commit side effects (§8f4)
and the capacity semantics of the accepted-vote arena.

  C2  100 validators x 10k txs = 1M votes (the bench workload) through txv_add_votes: every
      per-vote status + fired bit, the commit events, every TxVoteSet's (sum, maj23) and the set
      count equal the oracle's (ed25519 verify on every host core + the sequential tally)
  C3  the sharded layout: two shards of the C3 workload on two contexts of one GPU, the per-shard
      state packed ON THE DEVICE (txv_pack_commit_state), equal to the host pack of the oracle's
      state, merged via the C-ABI unpack and equal to one global sequential run
  C4  the adversarial stream at 2^20 votes: zero mismatches
  C5  1000 weighted validators, 64k-vote batches through TxVotePool.CheckTx (txv_pool_check) and
      two TxFlow batches in flight (txv_submit_votes / txv_wait_votes) vs the oracle pool + flow
The 10^8-vote C4 gate is tools/gate/c4_gate.py (records under profiles/)."""
import os
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _cores():
    n = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()
        if q != "max":
            n = min(n, max(1, -(-int(q) // int(p))))
    except Exception:
        pass
    return max(1, n)


def _expected(ost, ofired):
    return ost.astype(np.uint8) | (ofired.astype(np.uint8) << 7)


def _first_fired(batch, ofired, committed):
    """vote index of each tx's first fired vote in this batch (its commit event), txs not yet committed"""
    out, seen = [], set()
    for i in np.nonzero(ofired)[0]:
        h = batch.txhash(int(i))
        if h in committed or h in seen:
            continue
        seen.add(h)
        out.append(int(i))
    committed.update(seen)
    return sorted(out)


def test_c2_full_size_matches_oracle(oracle_lib):
    import txflow_amd as T
    from txflow_amd.workload import Workload, SEEDS
    ctx = T.Context(max_batch=1 << 20, max_txs=10064, max_validators=100)
    try:
        wl = Workload(ctx, 100, 10_000, SEEDS["c2"])
        st, ev = ctx.add_votes(wl.batch, ev_cap=wl.n_txs + 1)
        flow = oracle_lib.Flow(wl.pubs, wl.powers, b"test_chain_id")
        ost, _, ofired = flow.add_batch(wl.batch, _cores())
        exp = _expected(ost, ofired)
        bad = np.nonzero(st != exp)[0]
        if len(bad):
            # which side moved: the oracle again on one thread over the first 2,000 votes, and the
            # device's own verdicts on them through txv_verify_batch with the registry keys
            head = wl.head(2000)
            o1, _, _ = oracle_lib.Flow(wl.pubs, wl.powers, b"test_chain_id").add_batch(head, 1)
            pubs = np.frombuffer(b"".join(wl.pubs), np.uint8).reshape(-1, 32)[wl.val_of[:2000]]
            dv = ctx.verify_batch(head, pubs)
            raise AssertionError(f"{len(bad)} mismatches {[(int(i), int(st[i]), int(exp[i])) for i in bad[:10]]}; "
                                 f"oracle 1-thread ADDED {int((o1 == 0).sum())}/2000, device verify ok "
                                 f"{int((dv == 0).sum())}/2000, cores {_cores()}")
        assert sorted(int(e["vote_index"]) for e in ev) == _first_fired(wl.batch, ofired, set())
        hashes = [h.tobytes() for h in wl.hashes]
        ex, sums, maj, txkeys = ctx.query_txs(hashes)
        for j, h in enumerate(hashes):
            assert (int(sums[j]), bool(maj[j])) == flow.query(h)
        assert ex.all() and ctx.num_tx_sets() == flow.num_sets() == wl.n_txs
        assert np.array_equal(txkeys, wl.txkeys)      # each set keeps its first vote's TxKey
        # the same batch again on a fresh TxFlow through the pipelined entry points
        ctx.reset_flow()
        t = ctx.submit_votes(wl.batch)
        st2, ev2 = ctx.wait_votes(t, ev_cap=wl.n_txs + 1)
        assert np.array_equal(st2, st) and len(ev2) == len(ev)
    finally:
        ctx.close()


def test_c4_adversarial_1m_gate(oracle_lib):
    import adversarial as A
    import txflow_amd as T
    ctx = T.Context(max_batch=1 << 18, max_txs=1 << 16, max_validators=256)
    try:
        st = A.run_gate(ctx, 1 << 20, batch=1 << 18, batches_per_epoch=2, threads=_cores(), log=lambda s: None)
        assert st["mismatches"] == 0, st
        assert st["votes"] >= 1 << 20 and st["events"] > 0
        for k in ("ErrVoteInvalidSignature", "ErrVoteNonDeterministicSignature", "DUPLICATE",
                  "ErrVoteInvalidValidatorIndex", "ErrVoteNil"):
            assert st["by_status"].get(k, 0) > 0, (k, st["by_status"])
    finally:
        ctx.close()


@pytest.mark.parametrize("pool_device", [False, True], ids=["host-cache", "device-cache"])
def test_c4_adversarial_with_pool_stage(oracle_lib, pool_device):
    """C4 with the pool in front (Appendix C): every batch through TxVotePool.CheckTx on the device
    and in the oracle (outcomes compared per vote), the admitted votes through the pipelined
    TxFlow; a small LRU (64k keys) so that some replays are ErrTxInCache and others, evicted,
    reach the tally as DUPLICATE.  device-cache: the LRU in HBM (TXV_POOL_DEVICE_CACHE)."""
    import adversarial as A
    import txflow_amd as T
    ctx = T.Context(max_batch=1 << 18, max_txs=1 << 16, max_validators=256)
    try:
        st = A.run_gate(ctx, 1 << 20, batch=1 << 18, batches_per_epoch=2, threads=_cores(), log=lambda s: None,
                        pool_stage=True, pool_cache=1 << 16, pool_device=pool_device)
        assert st["mismatches"] == 0 and st["pool_mismatches"] == 0, st
        assert st["pool_by_status"].get("ErrTxInCache", 0) > 0 and st["by_status"].get("DUPLICATE", 0) > 0, st
        assert st["by_status"].get("ErrVoteNonDeterministicSignature", 0) > 0, st
        # every Appendix C class survives CheckTx in (at least) 80 % of its share of the stream
        for name, share in (("ErrVoteInvalidValidatorAddress(empty)", 0.0025),
                            ("ErrVoteInvalidValidatorIndex", 0.005), ("ErrVoteNil", 0.001)):
            assert st["by_status"].get(name, 0) >= 0.8 * share * st["votes"], (name, st)
        # ... counted per generated class: all but the two whose signatures repeat by construction
        # (exact replays; the identity key's non-canonical R with s = 0 has four signatures in all),
        # which CheckTx keys by SHA-256(Signature) and drops as ErrTxInCache while cached
        for name, c in st["class_share_at_txflow"].items():
            if name not in ("exact_replay", "noncanonical_r"):
                assert c["ratio"] >= 0.8, (name, c)
    finally:
        ctx.close()


def test_c5_weighted_streaming_matches_oracle(oracle_lib):
    import txflow_amd as T
    from txflow_amd.workload import StreamWorkload, SEEDS
    n_vals, n_txs, batch = 1000, 256, 65536
    ctx = T.Context(max_batch=batch, max_txs=n_txs + 64, max_validators=n_vals)
    pool = None
    try:
        wl = StreamWorkload(ctx, n_vals, n_txs, SEEDS["c5"], batch)
        pool = T.TxVotePool(ctx, size=wl.n + 1, cache_size=wl.n + 1, max_txs_bytes=1 << 40)
        opool = oracle_lib.Pool(size=wl.n + 1, cache_size=wl.n + 1, max_txs_bytes=1 << 40)
        flow = oracle_lib.Flow(wl.pubs, wl.powers, b"test_chain_id")
        exp, events, committed = [], [], set()
        for b in wl.batches:
            ps = pool.check_batch(b)
            ops = opool.check([dict(height=int(b.height[i]), txhash=b.txhash(i), ts_sec=int(b.ts_sec[i]),
                                    ts_nanos=int(b.ts_nanos[i]), addr=b.addr[20 * i:20 * i + 20].tobytes(),
                                    sig=b.sig[64 * i:64 * i + 64].tobytes()) for i in range(b.n)])
            assert np.array_equal(ps, ops)
            ost, _, ofired = flow.add_batch(b, _cores())
            exp.append(_expected(ost, ofired))
            events.append(_first_fired(b, ofired, committed))
        got, inflight = [], []
        for b in wl.batches:
            if len(inflight) == 2:
                got.append(ctx.wait_votes(inflight.pop(0), ev_cap=b.n))
            inflight.append(ctx.submit_votes(b))
        while inflight:
            got.append(ctx.wait_votes(inflight.pop(0), ev_cap=batch))
        for k, ((st, ev), e) in enumerate(zip(got, exp)):
            bad = np.nonzero(st != e)[0]
            assert len(bad) == 0, (k, [(int(i), int(st[i]), int(e[i])) for i in bad[:10]])
            assert sorted(int(x["vote_index"]) for x in ev) == events[k]
        for h in wl.hashes:
            assert ctx.query_tx(h.tobytes()) == flow.query(h.tobytes())
        assert sum(len(e) for e in events) == n_txs
        assert pool.Size() == opool.size() == wl.n
    finally:
        if pool is not None:
            pool.close()
        ctx.close()


def test_c3_two_shard_layout_device_pack(oracle_lib):
    """C3's sharded layout at reduced size on one GPU: shard r of the C3 workload (2 shards of
    4,000 txs x 100 validators) on context r; each context's packed commit state written by the
    device equals the host pack of the oracle's per-shard state, and the merge of both equals one
    global sequential run."""
    import txflow_amd as T
    from txflow_amd import sharding
    from txflow_amd.workload import Workload, SEEDS
    world, n_txs, cap = 2, 4000, 4096
    keys_all, packed = [], []
    for r in range(world):
        ctx = T.Context(max_batch=1 << 19, max_txs=cap, max_validators=100, table_w=16)
        try:
            wl = Workload(ctx, 100, n_txs, SEEDS["c3"], shard=r, n_shards=world)
            st, ev = ctx.add_votes(wl.batch, ev_cap=wl.n_txs + 1)
            assert np.count_nonzero((st & 0x7F) == T.ADDED) == wl.n and len(ev) == wl.n_txs
            packed.append(ctx.read_commit_state(cap))      # packed by txv_k_pack on the device
            # first-seen order of the shard's TxHashes = its set ids
            keys, seen = [], set()
            for i in range(wl.n):
                h = wl.batch.txhash(i)
                if h not in seen:
                    seen.add(h)
                    keys.append(h)
            keys_all.append(keys)
            flow = oracle_lib.Flow(wl.pubs, wl.powers, b"test_chain_id")
            ost, _, _ = flow.add_batch(wl.batch, _cores())
            assert (ost == 0).all()
            com = np.array([flow.query(k)[1] for k in keys], np.uint8)
            sums = np.array([flow.query(k)[0] for k in keys], np.int64)
            dig = np.array([np.frombuffer(T.tx_digest(k), np.uint8) for k in keys])
            assert np.array_equal(packed[-1], T.commit_state_pack_host(com, sums, cap, dig))
        finally:
            ctx.close()
    gathered = np.concatenate(packed)
    # every set named by the digest its owner packed: no host-side keys of the other shard
    merged, stakes = sharding.merge_states(gathered, world, cap)
    union = set(T.tx_digest(k) for ks in keys_all for k in ks)
    assert len(union) == n_txs and merged == union
    assert all(stakes[k] == 100 for k in union)


def test_arena_holds_accepted_votes_only(oracle_lib):
    """The accepted-vote arena grows by ADDED votes only (the reference's votes map,
    types/vote_set.go:154): a stream of many more submitted than max_accepted votes -- replays,
    conflicts, bad signatures -- never reports TXV_ECAPACITY while the accepted votes fit; one that
    exceeds it does, and txv_reset_flow recovers the context."""
    import txflow_amd as T
    rnd = random.Random(9)
    ctx = T.Context(max_batch=1 << 14, max_txs=1024, max_validators=16, max_accepted=2100)
    try:
        seeds = [bytes(rnd.getrandbits(8) for _ in range(32)) for _ in range(10)]
        pubs = ctx.keygen(seeds)
        ctx.set_validators(pubs, [1] * 10, "test_chain_id")
        addrs, _ = ctx.validator_info()
        flow = oracle_lib.Flow(pubs, [1] * 10, b"test_chain_id")
        hashes = ["%064X" % rnd.getrandbits(256) for _ in range(200)]
        base = [T.TxVote(Height=1, TxHash=h, Timestamp=(1_700_000_000, 1 + j), ValidatorAddress=addrs[v])
                for j, (h, v) in enumerate((h, v) for h in hashes for v in range(10))]
        sigs = ctx.sign_votes(T.VoteBatch.from_votes(base), np.array([j % 10 for j in range(len(base))], np.uint32),
                              "test_chain_id")
        for v, s in zip(base, sigs):
            v.Signature = s.tobytes()
        submitted = 0
        for k in range(8):   # 8 x 6000 = 48000 votes, 2000 of them accepted
            part = []
            for _ in range(6000):
                v = rnd.choice(base)
                x = T.TxVote(Height=1, TxHash=v.TxHash, Timestamp=v.Timestamp, ValidatorAddress=v.ValidatorAddress,
                             Signature=v.Signature)
                if rnd.random() < 0.2:
                    x.Signature = bytes([x.Signature[0] ^ 1]) + x.Signature[1:]
                part.append(x)
            st, _ = ctx.add_votes(T.VoteBatch.from_votes(part))
            ost, _, ofired = flow.add_votes([dict(height=1, txhash=v.TxHash.encode(), ts_sec=v.Timestamp[0],
                                                  ts_nanos=v.Timestamp[1], addr=v.ValidatorAddress, sig=v.Signature)
                                             for v in part])
            assert np.array_equal(st, _expected(ost, ofired))
            submitted += len(part)
        assert submitted > 20 * 2100
        # 200 new sets x 1 validator: 2000 + 200 > 2100 accepted votes
        extra = [T.TxVote(Height=1, TxHash="%064X" % rnd.getrandbits(256), Timestamp=(1_700_000_000, 7),
                          ValidatorAddress=addrs[0]) for _ in range(200)]
        es = ctx.sign_votes(T.VoteBatch.from_votes(extra), np.zeros(200, np.uint32), "test_chain_id")
        for v, s in zip(extra, es):
            v.Signature = s.tobytes()
        with pytest.raises(T.TxvInfraError):
            ctx.add_votes(T.VoteBatch.from_votes(extra))
        with pytest.raises(T.TxvInfraError):           # poisoned until the reset
            ctx.add_votes(T.VoteBatch.from_votes(extra[:1]))
        ctx.reset_flow()
        st, ev = ctx.add_votes(T.VoteBatch.from_votes(base))
        assert (st & 0x7F == T.ADDED).all() and len(ev) == 200
    finally:
        ctx.close()


def test_make_commit_and_save_tx_match_oracle(oracle_lib):
    """TxVoteSet.MakeCommit / TxStore.SaveTx bytes (types/vote_set.go:242-259, tx/store.go:83-117):
    the CommitSigs are the accepted votes in full (each with its own TxKey and timestamp), listed
    in validator order (the reference's Go map order is arbitrary; each CommitSig's bytes are
    exact); the stored TxVoteSet carries the TxKey of the set's FIRST vote (txflow/service.go:
    201-207), whatever that vote's fate; no +2/3 -> the reference panics (TXV_ESTATE)."""
    import txflow_amd as T
    rnd = random.Random(21)
    n_vals = 7
    ctx = T.Context(max_batch=1 << 14, max_txs=1024, max_validators=16)
    try:
        seeds = [bytes(rnd.getrandbits(8) for _ in range(32)) for _ in range(n_vals)]
        pubs = ctx.keygen(seeds)
        powers = [1 + (i % 3) for i in range(n_vals)]
        ctx.set_validators(pubs, powers, "test_chain_id")
        addrs, _ = ctx.validator_info()
        hashes = ["%064X" % rnd.getrandbits(256) for _ in range(30)] + ["X" * 100, "short"]
        votes, signer = [], []
        for i in range(600):
            v = rnd.randrange(n_vals)
            votes.append(T.TxVote(Height=rnd.choice([1, 2, 0]), TxHash=rnd.choice(hashes),
                                  TxKey=bytes(rnd.getrandbits(8) for _ in range(32)),
                                  Timestamp=(1_700_000_000 + rnd.randrange(3), rnd.randrange(0, 10 ** 9)),
                                  ValidatorAddress=addrs[v]))
            signer.append(v)
        sigs = ctx.sign_votes(T.VoteBatch.from_votes(votes), np.array(signer, np.uint32), "test_chain_id")
        for i, (v, s) in enumerate(zip(votes, sigs)):
            v.Signature = s.tobytes()
            if i % 5 == 0:
                v.Signature = bytes([v.Signature[0] ^ 2]) + v.Signature[1:]
        flow = oracle_lib.Flow(pubs, powers, b"test_chain_id")
        by_sig = {}
        for part in (votes[:300], votes[300:]):
            st, _ = ctx.add_votes(T.VoteBatch.from_votes(part))
            ost, _, ofired = flow.add_votes([dict(height=v.Height, txhash=v.TxHash.encode(), ts_sec=v.Timestamp[0],
                                                  ts_nanos=v.Timestamp[1], addr=v.ValidatorAddress, sig=v.Signature)
                                             for v in part])
            assert np.array_equal(st, _expected(ost, ofired))
        for v in votes:
            by_sig.setdefault((v.TxHash, v.Signature), v)
        first_key = {}
        for v in votes:
            first_key.setdefault(v.TxHash, v.TxKey)
        n_commit = 0
        for h in hashes:
            hb = h.encode()
            q = flow.query(hb)
            ex, _, _, tk = ctx.query_txs([hb])
            if q is None:
                assert not ex[0]
                continue
            assert tk[0].tobytes() == first_key[h]
            if not q[1]:
                with pytest.raises(T.TxvInfraError):
                    ctx.make_commit(hb)
                continue
            n_commit += 1
            acc = []
            for val, sig in flow.get_votes(hb):
                v = by_sig[(h, sig)]
                acc.append(dict(height=v.Height, ts_sec=v.Timestamp[0], ts_nanos=v.Timestamp[1], addr=addrs[val],
                                sig=sig, txkey=v.TxKey))
            exp = oracle_lib.commit_bytes(hb, acc)
            assert ctx.make_commit(hb) == exp
            assert ctx.save_tx_bytes(hb) == oracle_lib.save_tx_bytes(hb, first_key[h], acc)
        assert n_commit > 5
    finally:
        ctx.close()


def test_txkey_spelled_by_txhash_is_not_uploaded(oracle_lib):
    """TxKey = SHA-256(tx) and TxHash = its upper-hex %X (types/tx_vote.go:38-45): a batch whose
    every non-nil vote's TxKey is the 32 bytes its TxHash spells does not upload the TxKey column
    (txv_staged_bytes: exactly 32 B per vote less), the device decodes it from the TxHash arena;
    one vote whose TxKey differs (or a lower-case TxHash) uploads the column.  Either way the
    statuses, each set's first-vote TxKey, MakeCommit and SaveTx bytes (every accepted vote's own
    TxKey) equal the oracle's."""
    import txflow_amd as T
    rnd = random.Random(23)
    n_vals = 5
    ctx = T.Context(max_batch=1 << 14, max_txs=1024, max_validators=8)
    try:
        seeds = [bytes(rnd.getrandbits(8) for _ in range(32)) for _ in range(n_vals)]
        pubs = ctx.keygen(seeds)
        powers = [1] * n_vals
        ctx.set_validators(pubs, powers, "test_chain_id")
        addrs, _ = ctx.validator_info()
        hashes = ["%064X" % rnd.getrandbits(256) for _ in range(24)]
        votes, signer = [], []
        for i in range(600):
            v = rnd.randrange(n_vals)
            h = rnd.choice(hashes)
            if 300 <= i < 450 and i % 40 == 3:
                h = h.lower()                                 # batch 3: TxHashes in lower case
            votes.append(T.TxVote(Height=1, TxHash=h, TxKey=bytes.fromhex(h),
                                  Timestamp=(1_700_000_000, rnd.randrange(0, 10 ** 9)), ValidatorAddress=addrs[v]))
            signer.append(v)
        sigs = ctx.sign_votes(T.VoteBatch.from_votes(votes), np.array(signer, np.uint32), "test_chain_id")
        for v, s in zip(votes, sigs):
            v.Signature = s.tobytes()
        for i in range(600):
            if (i % 150) % 37 == 0:
                votes[i] = None                               # nil votes carry no TxKey
        votes[150 + 7].TxKey = bytes(rnd.getrandbits(8) for _ in range(32))   # batch 2: one differs
        flow = oracle_lib.Flow(pubs, powers, b"test_chain_id")
        staged = []
        parts = (votes[:150], votes[150:300], votes[300:450], votes[450:])
        for part in parts:
            st, _ = ctx.add_votes(T.VoteBatch.from_votes(part))
            staged.append(ctx.staged_bytes())
            ost, _, ofired = flow.add_votes([dict(nil=True) if v is None else dict(
                height=v.Height, txhash=v.TxHash.encode(), ts_sec=v.Timestamp[0], ts_nanos=v.Timestamp[1],
                addr=v.ValidatorAddress, sig=v.Signature) for v in part])
            assert np.array_equal(st, _expected(ost, ofired))
        # the four batches have the same shape: only the TxKey column comes and goes
        assert staged[3] == staged[0] and staged[1] == staged[2] == staged[0] + 32 * 150, staged
        allv = [v for p in parts for v in p if v is not None]
        first_key, by_sig = {}, {}
        for v in allv:
            first_key.setdefault(v.TxHash, v.TxKey)
            by_sig.setdefault((v.TxHash, v.Signature), v)
        n_commit = 0
        for h in sorted({v.TxHash for v in allv}):
            hb = h.encode()
            q = flow.query(hb)
            ex, _, _, tk = ctx.query_txs([hb])
            if q is None:
                assert not ex[0]
                continue
            assert tk[0].tobytes() == first_key[h]
            if not q[1]:
                continue
            n_commit += 1
            acc = []
            for val, sig in flow.get_votes(hb):
                v = by_sig[(h, sig)]
                acc.append(dict(height=v.Height, ts_sec=v.Timestamp[0], ts_nanos=v.Timestamp[1], addr=addrs[val],
                                sig=sig, txkey=v.TxKey))
            assert ctx.make_commit(hb) == oracle_lib.commit_bytes(hb, acc)
            assert ctx.save_tx_bytes(hb) == oracle_lib.save_tx_bytes(hb, first_key[h], acc)
        assert n_commit > 10
    finally:
        ctx.close()


def test_lane_votes_8_without_the_wide_base_table(oracle_lib):
    """A configured V = 8 runs the V = 4 kernel whenever the base table is not the radix-2^24 one
    (small windows, caller-supplied keys): verdicts equal the oracle's."""
    import txflow_amd as T
    rnd = random.Random(3)
    for w in (8, 12):
        ctx = T.Context(max_batch=1 << 14, max_txs=1024, max_validators=16, table_w=w, lane_votes=8)
        try:
            seeds = [bytes(rnd.getrandbits(8) for _ in range(32)) for _ in range(4)]
            pubs = ctx.keygen(seeds)
            ctx.set_validators(pubs, [1] * 4, "test_chain_id")
            addrs, _ = ctx.validator_info()
            votes = [T.TxVote(Height=1, TxHash="%064X" % rnd.getrandbits(256), Timestamp=(1_700_000_000, i + 1),
                              ValidatorAddress=addrs[i % 4]) for i in range(500)]
            sigs = ctx.sign_votes(T.VoteBatch.from_votes(votes), np.array([i % 4 for i in range(500)], np.uint32),
                                  "test_chain_id")
            for i, (v, s) in enumerate(zip(votes, sigs)):
                v.Signature = s.tobytes() if i % 3 else bytes([s[1] ^ 4]) + s.tobytes()[1:]
            b = T.VoteBatch.from_votes(votes)
            st = ctx.verify_batch(b)
            keys = np.array([np.frombuffer(pubs[i % 4], np.uint8) for i in range(500)])
            st2 = ctx.verify_batch(b, keys)
            exp = np.array([oracle_lib.verify(pubs[i % 4], oracle_lib.signbytes(
                1, v.TxHash.encode(), v.Timestamp[0], v.Timestamp[1], b"test_chain_id"), v.Signature)
                for i, v in enumerate(votes)])
            assert np.array_equal(st == T.ADDED, exp) and np.array_equal(st2, st)
            st3, _ = ctx.add_votes(b)
            assert np.array_equal((st3 & 0x7F) == T.ADDED, exp)
        finally:
            ctx.close()


def test_staged_two_in_flight_with_commit_sinks(oracle_lib):
    """Two device-resident batches in flight (txv_run_staged returns at once; batch k+1's verify
    chain runs beside batch k's tally): consecutive C5-shaped batches whose txs straddle the
    batch boundary give the sequential oracle's per-vote codes and events, and each slot's commit
    sink (txv_set_commit_sink, packed on the device at the end of its batch) holds the state as
    of that batch although the next batch is already running.  Then the same with a fresh TxFlow
    per batch (txv_reset_flow between launches) and all three staged slots enqueued, as bench.py
    replays its workload."""
    import torch
    import txflow_amd as T
    from txflow_amd.workload import StreamWorkload, SEEDS
    n_vals, n_txs, batch, cap = 64, 700, 8192, 1024
    ctx = T.Context(max_batch=batch, max_txs=cap, max_validators=n_vals)
    try:
        wl = StreamWorkload(ctx, n_vals, n_txs, SEEDS["c5"] + 7, batch, window=96)
        flow = oracle_lib.Flow(wl.pubs, wl.powers, b"test_chain_id")
        exp, events, states, committed, seen = [], [], [], set(), []
        for b in wl.batches:
            ost, _, ofired = flow.add_batch(b, _cores())
            exp.append(_expected(ost, ofired))
            events.append(_first_fired(b, ofired, committed))
            for i in range(b.n):
                h = b.txhash(i)
                if h not in seen:
                    seen.append(h)
            q = [flow.query(h) for h in seen]
            states.append(T.commit_state_pack_host(np.array([m for _, m in q], np.uint8),
                                                   np.array([s for s, _ in q], np.int64), cap,
                                                   np.array([np.frombuffer(T.tx_digest(h), np.uint8) for h in seen])))
        words = T.commit_state_bytes(cap) // 4
        sinks = [torch.zeros(words, dtype=torch.int32, device="cuda:0") for _ in range(2)]
        for sl in range(2):
            ctx.set_commit_sink(sl, sinks[sl].data_ptr(), cap)

        def check(k, st, ev, exp_state):
            bad = np.nonzero(st != exp[k])[0]
            assert len(bad) == 0, (k, [(int(i), int(st[i]), int(exp[k][i])) for i in bad[:10]])
            assert sorted(int(x["vote_index"]) for x in ev) == events[k]
            if exp_state is not None:
                got = sinks[k % 2].cpu().numpy().view(np.uint8)
                assert np.array_equal(got, exp_state), k

        nb = len(wl.batches)
        assert nb >= 4
        ctx.stage(0, wl.batches[0])
        ctx.run_staged(0)
        ctx.stage(1, wl.batches[1])
        ctx.run_staged(1)
        # steady state: fetch k-1 while k runs, restage slot (k+1) % 2 after its fetch
        st, ev = ctx.fetch_staged(0, wl.batches[0].n, ev_cap=batch)
        check(0, st, ev, states[0])
        for k in range(2, nb):
            ctx.stage(k % 2, wl.batches[k])
            ctx.run_staged(k % 2)
            st, ev = ctx.fetch_staged((k - 1) % 2, wl.batches[k - 1].n, ev_cap=batch)
            check(k - 1, st, ev, states[k - 1])
        st, ev = ctx.fetch_staged((nb - 1) % 2, wl.batches[nb - 1].n, ev_cap=batch)
        check(nb - 1, st, ev, states[nb - 1])
        for h in wl.hashes:
            assert ctx.query_tx(h.tobytes()) == flow.query(h.tobytes())
        assert ctx.num_tx_sets() == n_txs
        ms = ctx.slot_kernel_ms((nb - 1) % 2)
        assert all(x >= 0 for x in ms) and ms[3] >= ms[1] > 0
        k1a, k1b = ctx.slot_verify_ms((nb - 1) % 2)      # the verify time split at the K1a | K1b event
        assert k1a > 0 and k1b > 0 and abs(k1a + k1b - ms[1]) < 0.01 + 0.01 * ms[1]

        # fresh TxFlow per launch, three slots enqueued (as bench.py runs): every run of batch 0
        # gives batch 0's results and its sink batch 0's state
        sinks.append(torch.zeros(words, dtype=torch.int32, device="cuda:0"))
        ctx.set_commit_sink(2, sinks[2].data_ptr(), cap)
        for sl in range(3):
            ctx.stage(sl, wl.batches[0])
        for k in range(8):
            ctx.reset_flow()
            ctx.run_staged(k % 3)
            if k >= 2:
                st, ev = ctx.fetch_staged((k - 2) % 3, wl.batches[0].n, ev_cap=batch)
                check(0, st, ev, None)
                assert np.array_equal(sinks[(k - 2) % 3].cpu().numpy().view(np.uint8), states[0])
        for k in (6, 7):
            st, ev = ctx.fetch_staged(k % 3, wl.batches[0].n, ev_cap=batch)
            check(0, st, ev, None)
            assert np.array_equal(sinks[k % 3].cpu().numpy().view(np.uint8), states[0])
        for sl in range(3):
            ctx.set_commit_sink(sl, None)
    finally:
        ctx.close()


def _signed_votes(ctx, T, addrs, hashes, n_vals, rnd, ts0=1):
    """every validator votes every tx of `hashes` (arrival order shuffled), device-signed"""
    votes, signer = [], []
    for h in hashes:
        for v in range(n_vals):
            votes.append(T.TxVote(Height=1, TxHash=h, Timestamp=(1_700_000_000, ts0 + len(votes)),
                                  ValidatorAddress=addrs[v]))
            signer.append(v)
    order = list(range(len(votes)))
    rnd.shuffle(order)
    votes = [votes[i] for i in order]
    signer = np.array([signer[i] for i in order], np.uint32)
    sigs = ctx.sign_votes(T.VoteBatch.from_votes(votes), signer, "test_chain_id")
    for v, s in zip(votes, sigs):
        v.Signature = s.tobytes()
    return votes


def _odicts(votes):
    return [dict(height=v.Height, txhash=v.TxHash.encode(), ts_sec=v.Timestamp[0], ts_nanos=v.Timestamp[1],
                 addr=v.ValidatorAddress, sig=v.Signature) for v in votes]


def test_fetch_out_of_run_order_keeps_every_set_tallied(oracle_lib):
    """a staged slot fetched after a later txv_submit_votes batch was waited (an older
    summary arriving last), and a slot re-staged and run again before its results were fetched,
    must not shrink the touched-set bound of later batches: every new TxVoteSet of the following
    batches is still tallied, its commit event reported and its stake summed, as the sequential
    TxFlow.addVote does (txflow/service.go:192-234)."""
    import txflow_amd as T
    rnd = random.Random(77)
    n_vals = 16
    ctx = T.Context(max_batch=1 << 14, max_txs=2048, max_validators=n_vals)
    try:
        seeds = [bytes(rnd.getrandbits(8) for _ in range(32)) for _ in range(n_vals)]
        pubs = ctx.keygen(seeds)
        ctx.set_validators(pubs, [1] * n_vals, "test_chain_id")
        addrs, _ = ctx.validator_info()
        flow = oracle_lib.Flow(pubs, [1] * n_vals, b"test_chain_id")
        hx = lambda k: ["%064X" % rnd.getrandbits(256) for _ in range(k)]
        b0 = _signed_votes(ctx, T, addrs, hx(100), n_vals, rnd, 1)       # slot 2, staged
        b1 = _signed_votes(ctx, T, addrs, hx(200), n_vals, rnd, 10 ** 6)  # submit ring (slot 0)
        b2 = _signed_votes(ctx, T, addrs, hx(1), n_vals, rnd, 2 * 10 ** 6)
        b3 = _signed_votes(ctx, T, addrs, hx(1), n_vals, rnd, 3 * 10 ** 6)    # slot 3, never fetched
        b4 = _signed_votes(ctx, T, addrs, hx(40), n_vals, rnd, 4 * 10 ** 6)   # slot 3 again
        b5 = _signed_votes(ctx, T, addrs, hx(1), n_vals, rnd, 5 * 10 ** 6)

        def expect(votes):
            ost, _, ofired = flow.add_votes(_odicts(votes))
            return _expected(ost, ofired)

        e0, e1, e2, _, e4, e5 = (expect(b) for b in (b0, b1, b2, b3, b4, b5))
        ctx.stage(2, T.VoteBatch.from_votes(b0))
        ctx.run_staged(2)
        t = ctx.submit_votes(T.VoteBatch.from_votes(b1))
        st1, ev1 = ctx.wait_votes(t, ev_cap=len(b1))
        st0, ev0 = ctx.fetch_staged(2, len(b0), ev_cap=len(b0))       # the older summary, fetched last
        assert np.array_equal(st0, e0) and np.array_equal(st1, e1) and len(ev0) == 100 and len(ev1) == 200
        assert ctx.num_tx_sets() == 300
        st2, ev2 = ctx.add_votes(T.VoteBatch.from_votes(b2))
        assert np.array_equal(st2, e2) and len(ev2) == 1
        ctx.stage(3, T.VoteBatch.from_votes(b3))
        ctx.run_staged(3)
        ctx.stage(3, T.VoteBatch.from_votes(b4))                      # re-staged before its fetch
        ctx.run_staged(3)
        st4, ev4 = ctx.fetch_staged(3, len(b4), ev_cap=len(b4))
        assert np.array_equal(st4, e4) and len(ev4) == 40
        st5, ev5 = ctx.add_votes(T.VoteBatch.from_votes(b5))
        assert np.array_equal(st5, e5) and len(ev5) == 1
        for v in b0[:1] + b1[:1] + b2[:1] + b3[:1] + b4[:1] + b5[:1]:
            assert ctx.query_tx(v.TxHash.encode()) == flow.query(v.TxHash.encode())
        assert ctx.num_tx_sets() == flow.num_sets() == 343
    finally:
        ctx.close()


def test_c1_full_config_matches_oracle(oracle_lib):
    """C1 (BASELINE.json configs[0]) at its own size: 4 validators x 2,500 txs = 10,000 signed
    TxVotes, shuffled, through txv_add_votes and again through the pipelined submit / wait path;
    every per-vote status + fired bit, every commit event and every TxVoteSet's (sum, maj23) equal
    the sequential oracle's (verify on every host core)."""
    import txflow_amd as T
    from txflow_amd.workload import Workload, SEEDS
    ctx = T.Context(max_batch=16384, max_txs=4096, max_validators=8)
    try:
        wl = Workload(ctx, 4, 2500, SEEDS["c1"])
        assert wl.n == 10_000
        flow = oracle_lib.Flow(wl.pubs, wl.powers, b"test_chain_id")
        ost, _, ofired = flow.add_batch(wl.batch, _cores())
        exp = _expected(ost, ofired)
        st, ev = ctx.add_votes(wl.batch, ev_cap=wl.n_txs + 1)
        assert np.array_equal(st, exp)
        assert sorted(int(e["vote_index"]) for e in ev) == _first_fired(wl.batch, ofired, set())
        # quorum of 4 x power 1 = 3: the 3rd and 4th vote of every tx fire
        assert int(np.count_nonzero(st & 0x80)) == 2 * wl.n_txs
        hashes = [h.tobytes() for h in wl.hashes]
        ex, sums, maj, _ = ctx.query_txs(hashes)
        assert ex.all() and all((int(sums[j]), bool(maj[j])) == flow.query(h) for j, h in enumerate(hashes))
        ctx.reset_flow()
        t = ctx.submit_votes(wl.batch)
        st2, ev2 = ctx.wait_votes(t, ev_cap=wl.n_txs + 1)
        assert np.array_equal(st2, exp) and len(ev2) == len(ev)
    finally:
        ctx.close()


def test_c3_one_rank_full_shard_matches_oracle(oracle_lib):
    """C3 (BASELINE.json configs[2]) at one rank's real size: the full C3 workload (160,000 txs x
    100 validators = 16M votes) sharded by SHA-256(TxHash)[0] mod 8, shard 3 (~20k txs, ~2M
    votes) on one context, as bench.py's rank 3 of 8 holds it: every per-vote status + fired bit
    and commit event equals the oracle's, and the packed commit state written by the device
    equals the host pack of the oracle's per-set state."""
    import txflow_amd as T
    from txflow_amd.workload import Workload, SEEDS
    world, rank = 8, 3
    cap = 22_000
    ctx = T.Context(max_batch=(cap + 64) * 100, max_txs=cap + 64, max_validators=100)
    try:
        wl = Workload(ctx, 100, 160_000, SEEDS["c3"], shard=rank, n_shards=world)
        assert 19_000 < wl.n_txs < cap and wl.n == wl.n_txs * 100
        st, ev = ctx.add_votes(wl.batch, ev_cap=wl.n_txs + 1)
        flow = oracle_lib.Flow(wl.pubs, wl.powers, b"test_chain_id")
        ost, _, ofired = flow.add_batch(wl.batch, _cores())
        bad = np.nonzero(st != _expected(ost, ofired))[0]
        assert len(bad) == 0, [(int(i), int(st[i])) for i in bad[:10]]
        assert sorted(int(e["vote_index"]) for e in ev) == _first_fired(wl.batch, ofired, set())
        keys, seen = [], set()
        for i in range(wl.n):
            h = wl.batch.txhash(i)
            if h not in seen:
                seen.add(h)
                keys.append(h)
        q = [flow.query(k) for k in keys]
        host = T.commit_state_pack_host(np.array([m for _, m in q], np.uint8), np.array([s for s, _ in q], np.int64),
                                        cap, np.array([np.frombuffer(T.tx_digest(k), np.uint8) for k in keys]))
        assert np.array_equal(ctx.read_commit_state(cap), host)
        assert ctx.num_tx_sets() == flow.num_sets() == wl.n_txs
    finally:
        ctx.close()

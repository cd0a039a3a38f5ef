"""TxVotePool.Update cadence, on the oracle pool and TxFlow (CPU).

The reference's commit path runs after EVERY fired vote -- the ADDED vote that crosses 2/3 and each
later ADDED vote of a committed set -- and calls txV.Update(height, set.GetVotes()) with the set's
whole vote list each time (txflow/service.go:216-227 -> txvotepool.go:329-359: every vote's key
pushed to the LRU cache, the vote removed from the pool list).  bench.py's C5 legs issue, once per
batch, one Update holding the sets that fired in the batch, ordered by their last fired vote, each
set's accepted votes in one block (bench.c5_commit_updates).  A key's LRU place depends only on its
last push and removals are idempotent, so both leave the same pool: the same cache keys in the same
order, the same pool list, Size and TxsBytes -- checked here after every batch on a stream whose
small cache evicts inside the Updates.  GetVotes iterates a Go map, so the reference's order inside
a set's block is unspecified; both cadences take arrival order.  The cadence rounds 4-5 used (each
batch's newly ADDED votes of sets committed earlier, without the rest of their set) is shown to
differ, so the test can tell them apart."""
import hashlib
import random
import struct

import numpy as np

import oracle as O

CHAIN = b"test_chain_id"


def _stream(rnd, n_vals=6, n_txs=40, replay=0.08):
    seeds = [hashlib.sha512(b"cadence" + struct.pack("<I", i)).digest()[:32] for i in range(n_vals)]
    pubs = [O.pubkey(s) for s in seeds]
    addrs = [O.sha256(p)[:20] for p in pubs]
    hashes = [hashlib.sha256(b"cadence-tx%d" % t).hexdigest().upper().encode() for t in range(n_txs)]
    pairs = [(t, v) for t in range(n_txs) for v in range(n_vals)]
    pairs.sort(key=lambda tv: tv[0] + rnd.random() * 6)          # a tx's votes straddle a few batches
    votes = []
    for i, (t, v) in enumerate(pairs):
        msg = O.signbytes(1, hashes[t], 1_700_000_000, i + 1, CHAIN)
        votes.append(dict(height=1, txhash=hashes[t], ts_sec=1_700_000_000, ts_nanos=i + 1, addr=addrs[v],
                          sig=O.sign(seeds[v], msg), tx=t))
        if rnd.random() < replay:
            votes.append(dict(votes[rnd.randrange(len(votes))]))
    return pubs, [1 + (i % 3) for i in range(n_vals)], votes


def _state(pool):
    keys, sizes = pool.reap(-1)
    return pool.cache_keys().tobytes(), keys.tobytes(), sizes.tobytes(), pool.size(), pool.txs_bytes()


def _run(cadence, pubs, powers, votes, batch=48, cache=30):
    pool = O.Pool(size=1 << 20, cache_size=cache, max_txs_bytes=1 << 40)
    flow = O.Flow(pubs, powers, CHAIN)
    added = {}                       # tx -> its ADDED votes in arrival order (GetVotes)
    states = []
    for s in range(0, len(votes), batch):
        part = votes[s:s + batch]
        ps = pool.check(part)
        adm = [v for v, x in zip(part, ps) if x == 0]
        if cadence == "reference":
            # TryAddVote one vote at a time; Update(GetVotes) right after every fired vote
            for v in adm:
                st, _, fired = flow.add_votes([v])
                if st[0] == 0:
                    added.setdefault(v["tx"], []).append(v)
                if fired[0]:
                    pool.update(1, added[v["tx"]])
        else:
            st, _, fired = flow.add_votes(adm)
            last, newly = {}, []
            for j, v in enumerate(adm):
                if st[j] == 0:
                    added.setdefault(v["tx"], []).append(v)
                if fired[j]:
                    last[v["tx"]] = j
                    newly.append(v)
            if cadence == "grouped":           # bench.c5_commit_updates
                upd = [u for t in sorted(last, key=last.get) for u in added[t]]
            else:                              # "old": the crossing sets whole, later sets' new votes only
                first = set()
                upd = []
                for t in sorted(last, key=last.get):
                    if t not in _run.committed:
                        upd += added[t]
                        first.add(t)
                upd += [v for v in newly if v["tx"] not in first and v["tx"] in _run.committed]
                _run.committed |= first
            if upd:
                pool.update(1, upd)
        states.append(_state(pool))
    return states


def test_grouped_update_cadence_equals_per_vote_refire():
    rnd = random.Random(2026)
    pubs, powers, votes = _stream(rnd)
    ref = _run("reference", pubs, powers, votes)
    grp = _run("grouped", pubs, powers, votes)
    assert len(ref) == len(grp) > 5
    for b, (x, y) in enumerate(zip(ref, grp)):
        assert x[0] == y[0], f"batch {b}: LRU cache order differs"
        assert x[1:] == y[1:], f"batch {b}: pool list / Size / TxsBytes differ"
    assert len(ref[-1][0]) == 30 * 32                      # the cache filled (evictions happened)
    _run.committed = set()
    old = _run("old", pubs, powers, votes)
    assert any(x[0] != y[0] for x, y in zip(ref, old)), "the earlier cadence should differ somewhere"


_run.committed = set()

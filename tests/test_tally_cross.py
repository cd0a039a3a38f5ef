"""The crossing step (txv_k_tally_cross) against the oracle's sequential addVerifiedVote
(types/vote_set.go:143-166: sum += power; maj23 |= sum >= Total*2/3 + 1, in arrival order), at
the shapes its two code paths and its digit search see:

  * more ADDED votes in one set than the LDS list holds (1100 validators > kListCap = 1024): the
    histogram levels re-read the set's row;
  * skewed stake (a few validators hold most of it), so the crossing vote sits at an arbitrary
    arrival position, with invalid signatures among the votes (not ADDED, no stake);
  * a set that crosses in a later batch than its first votes (prior stake > 0) and keeps
    re-firing afterwards.
Every per-vote status + fired bit, the commit events and every set's (sum, maj23) equal the oracle."""
import numpy as np
import pytest

from test_configs import _cores, _expected, _first_fired

pytestmark = pytest.mark.gpu


def _slice(T, b, s, e):
    return T.VoteBatch(e - s, height=b.height[s:e], txhash_arena=b.txhash_arena, txhash_off=b.txhash_off[s:e],
                       txhash_len=b.txhash_len[s:e], ts_sec=b.ts_sec[s:e], ts_nanos=b.ts_nanos[s:e],
                       addr=b.addr[20 * s:20 * e], addr_len=b.addr_len[s:e], sig=b.sig[64 * s:64 * e],
                       sig_len=b.sig_len[s:e], txkey=None if b.txkey is None else b.txkey[32 * s:32 * e])


def _run(oracle_lib, n_vals, n_txs, powers, cuts, bad_frac, seed):
    import txflow_amd as T
    from txflow_amd.workload import Workload
    ctx = T.Context(max_batch=1 << 16, max_txs=n_txs + 64, max_validators=n_vals, table_w=8)
    try:
        wl = Workload(ctx, n_vals, n_txs, seed, powers=powers)
        rng = np.random.default_rng(seed + 1)
        sig = wl.batch.sig.reshape(wl.n, 64)
        bad = rng.random(wl.n) < bad_frac
        sig[bad, 5] ^= 0x10                           # R bit flip: ErrVoteInvalidSignature, no stake
        flow = oracle_lib.Flow(wl.pubs, wl.powers, b"test_chain_id")
        committed = set()
        bounds = [0] + list(cuts) + [wl.n]
        for k in range(len(bounds) - 1):
            b = _slice(T, wl.batch, bounds[k], bounds[k + 1])
            st, ev = ctx.add_votes(b, ev_cap=b.n)
            ost, _, ofired = flow.add_batch(b, _cores())
            exp = _expected(ost, ofired)
            mism = np.nonzero(st != exp)[0]
            assert len(mism) == 0, (k, [(int(i), int(st[i]), int(exp[i])) for i in mism[:10]])
            assert sorted(int(x["vote_index"]) for x in ev) == _first_fired(b, ofired, committed)
        for h in wl.hashes:
            assert ctx.query_tx(h.tobytes()) == flow.query(h.tobytes())
        return len(committed)
    finally:
        ctx.close()


def test_cross_sets_larger_than_lds_list(oracle_lib):
    rng = np.random.default_rng(11)
    powers = 1 + rng.integers(0, 1_000_000, 1100)
    n = _run(oracle_lib, 1100, 6, powers, cuts=(2500, 4100), bad_frac=0.03, seed=0x7478763101)
    assert n == 6


def test_cross_skewed_stake_with_invalid_votes(oracle_lib):
    powers = np.ones(700, np.int64)
    powers[[3, 77, 150, 400, 699]] = 10**9           # five validators hold ~all of the stake
    n = _run(oracle_lib, 700, 16, powers, cuts=(3000, 7000, 7001), bad_frac=0.05, seed=0x7478763102)
    assert n > 0


def test_cross_in_later_batch_refires(oracle_lib):
    # every tx's votes spread over four batches: the crossing batch has prior stake, the later ones re-fire
    n = _run(oracle_lib, 200, 40, np.arange(1, 201, dtype=np.int64), cuts=(2000, 4000, 6000), bad_frac=0.02,
             seed=0x7478763103)
    assert n == 40

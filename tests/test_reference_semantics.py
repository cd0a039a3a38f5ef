"""The reference's own TxVoteSet / TxFlow tests, restated against the CODE semantics
(several reference tests were copied from Tendermint's per-BlockID VoteSet and
contradict types/vote_set.go; parity is defined against the code).  CPU: the sequential
oracle.  GPU (-m gpu): the same scenarios through libtxvote.so must give identical results.

Scenario sources (Fantom-foundation/go-txflow):
  TestAddVote              types/vote_set_test.go:84-116  (consistent with the code)
  Test2_3Majority          types/vote_set_test.go:118-152 (restated: quorum = 10*2/3+1 = 7 of 10)
  TestBadVotes             types/vote_set_test.go:233-290 (restated: wrong height is NOT checked)
  TestConflicts            types/vote_set_test.go:292-393 (restated: second vote -> NonDeterministic)
  TestVoteVerify           types/vote_test.go:143-159     (wrong key -> InvalidValidatorAddress)
"""
import random

import numpy as np
import pytest

CHAIN = b"test_chain_id"


def _keys(rnd, n):
    import oracle as O
    seeds = [bytes(rnd.getrandbits(8) for _ in range(32)) for _ in range(n)]
    pubs = [O.pubkey(s) for s in seeds]
    addrs = [O.sha256(p)[:20] for p in pubs]
    return seeds, pubs, addrs


def _vote(O, seed, addr, txhash, height=1, ts=(1_700_000_000, 1), chain=CHAIN, sig=None):
    msg = O.signbytes(height, txhash, ts[0], ts[1], chain)
    return dict(height=height, txhash=txhash, ts_sec=ts[0], ts_nanos=ts[1], addr=addr,
                sig=O.sign(seed, msg) if sig is None else sig)


def scenario_votes(O):
    """A list of (votes, expected_status, expected_fired) per restated reference test."""
    rnd = random.Random(2019)
    seeds, pubs, addrs = _keys(rnd, 10)
    tx1 = O.sha256(b"0x1").hex().upper().encode()
    tx2 = O.sha256(b"0x2").hex().upper().encode()
    out = []
    # TestAddVote: one vote from val0 -> added, no 2/3
    out.append(("TestAddVote", [_vote(O, seeds[0], addrs[0], tx1)], [0], [0]))
    # Test2_3Majority (code semantics): 6 votes -> no maj; 7th -> maj (fires); 8th added & fires again
    vs = [_vote(O, seeds[i], addrs[i], tx1, ts=(1_700_000_000, 10 + i)) for i in range(8)]
    out.append(("Test2_3Majority", vs, [0] * 8, [0] * 6 + [1, 1]))
    # TestBadVotes: (a) dup of val0's vote -> (false, nil); (b) val0 re-signs a different timestamp ->
    # NonDeterministic; (c) wrong height from val1 is NOT checked by the code -> added;
    # (d) TxHash differs -> routed to a different TxVoteSet -> added there; (e) unknown validator.
    v0 = _vote(O, seeds[0], addrs[0], tx1, ts=(1_700_000_000, 100))
    bad = [v0, dict(v0), _vote(O, seeds[0], addrs[0], tx1, ts=(1_700_000_000, 101)),
           _vote(O, seeds[1], addrs[1], tx1, height=2), _vote(O, seeds[2], addrs[2], tx2),
           _vote(O, bytes(32), O.sha256(O.pubkey(bytes(32)))[:20], tx1)]
    out.append(("TestBadVotes", bad, [0, 1, 5, 0, 0, 4], [0] * 6))
    # TestConflicts: conflicting signatures from the same validator; first wins, wrong-chain sig fails
    c = [_vote(O, seeds[3], addrs[3], tx2, ts=(1_700_000_000, 5), chain=b"incorrect-chain-id"),
         _vote(O, seeds[3], addrs[3], tx2, ts=(1_700_000_000, 6)),
         _vote(O, seeds[3], addrs[3], tx2, ts=(1_700_000_000, 7))]
    out.append(("TestConflicts", c, [6, 0, 5], [0, 0, 0]))
    # nil / empty address
    out.append(("NilAndEmpty", [dict(nil=True), dict(_vote(O, seeds[4], addrs[4], tx1), addr=b"")], [2, 3], [0, 0]))
    # SignBytes is only reached inside Verify, AFTER the accepted-vote check (vote_set.go:108-117):
    # an out-of-amino-range timestamp (year 10000) is a SignBytes error only when the group has
    # no accepted vote; against an accepted vote it is a duplicate / non-deterministic signature.
    far = (253402300800, 0)
    ok5 = _vote(O, seeds[5], addrs[5], tx1, ts=(1_700_000_000, 300))
    sb = [dict(ok5, ts_sec=far[0], ts_nanos=far[1], sig=_vote(O, seeds[5], addrs[5], tx1)["sig"]),
          ok5,
          dict(ok5, ts_sec=far[0], ts_nanos=far[1]),
          dict(ok5, ts_sec=far[0], ts_nanos=far[1], sig=bytes(64)),
          dict(_vote(O, seeds[6], addrs[6], tx1), ts_sec=far[0], ts_nanos=far[1])]
    out.append(("SignBytesAfterAccepted", sb, [8, 0, 1, 5, 8], [0] * 5))
    return pubs, out


def test_reference_scenarios_oracle(oracle_lib):
    O = oracle_lib
    pubs, scen = scenario_votes(O)
    for name, votes, exp, fired in scen:
        flow = O.Flow(pubs, [1] * len(pubs), CHAIN)
        st, sums, fr = flow.add_votes(votes)
        assert list(st) == exp, name
        assert list(fr) == fired, name


def test_vote_verify_errors_oracle(oracle_lib):
    """types/vote_test.go:143-159: wrong pubkey -> ErrVoteInvalidValidatorAddress; unsigned ->
    ErrVoteInvalidSignature (via the TxVote.Verify restatement)."""
    O = oracle_lib
    rnd = random.Random(1)
    seeds, pubs, addrs = _keys(rnd, 2)
    th = b"AB" * 32
    v = _vote(O, seeds[0], addrs[0], th)
    import ctypes
    from oracle import _Vote, lib

    def verify(vote, pub):
        bufs = [ctypes.create_string_buffer(vote[k] or b"\0", max(1, len(vote[k]))) for k in ("txhash", "addr", "sig")]
        cv = _Vote(0, vote["height"], ctypes.addressof(bufs[0]), len(vote["txhash"]), vote["ts_sec"],
                   vote["ts_nanos"], ctypes.addressof(bufs[1]), len(vote["addr"]), ctypes.addressof(bufs[2]),
                   len(vote["sig"]))
        lib().orc_txvote_verify.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
        return lib().orc_txvote_verify(ctypes.byref(cv), CHAIN, len(CHAIN), pub)

    assert verify(v, pubs[0]) == O.ADDED
    assert verify(v, pubs[1]) == O.ERR_INVALID_VALIDATOR_ADDRESS
    assert verify(dict(v, sig=b""), pubs[0]) == O.ERR_INVALID_SIGNATURE


@pytest.mark.gpu
def test_reference_scenarios_gpu(gpu_ctx, oracle_lib):
    import txflow_amd as T
    O = oracle_lib
    pubs, scen = scenario_votes(O)
    for name, votes, exp, fired in scen:
        gpu_ctx.set_validators(pubs, [1] * len(pubs), CHAIN.decode())
        tv = [None if v.get("nil") else
              T.TxVote(Height=v["height"], TxHash=v["txhash"].decode(), Timestamp=(v["ts_sec"], v["ts_nanos"]),
                       ValidatorAddress=v["addr"], Signature=v["sig"]) for v in votes]
        st, _ = gpu_ctx.add_votes(T.VoteBatch.from_votes(tv))
        assert list(st & 0x7F) == exp, name
        assert list((st >> 7) & 1) == fired, name


@pytest.mark.gpu
def test_txflow_api_gpu(gpu_ctx, oracle_lib):
    """TxFlow.TryAddVote / TxVoteSet readers (reference-shaped API) on the device tally."""
    import txflow_amd as T
    O = oracle_lib
    rnd = random.Random(4)
    seeds, pubs, addrs = _keys(rnd, 4)
    flow = T.TxFlow(gpu_ctx, pubs, [1, 1, 1, 1], "test_chain_id")
    th = "C0FFEE" * 10 + "ABCD"
    added = []
    for i in range(4):
        msg = O.signbytes(1, th.encode(), 1_700_000_000, i + 1, CHAIN)
        v = T.TxVote(Height=1, TxHash=th, Timestamp=(1_700_000_000, i + 1), ValidatorAddress=addrs[i],
                     Signature=O.sign(seeds[i], msg))
        added.append(flow.TryAddVote(v))
        again = flow.TryAddVote(v)
        assert again == (False, None)            # duplicate: (false, nil)
    assert [a for a, _ in added] == [True] * 4
    vs = flow.TxVoteSet(th)
    assert vs.Stake() == 4 and vs.HasTwoThirdsMajority() and vs.HasAll() and vs.HasTwoThirdsAny()
    assert vs.TotalStake() == 2
    ok, err = flow.TryAddVote(T.TxVote(Height=1, TxHash=th, Timestamp=(1, 1), ValidatorAddress=bytes(20),
                                       Signature=bytes(64)))
    assert not ok and err.code == T.ERR_UNKNOWN_VALIDATOR
    assert flow.commits and flow.commits[0][0] == th

"""CPU check of the C4 adversarial stream generator (tests/adversarial.py) before it is used as the
GPU gate: a stand-in context built from the oracle (keygen / sign / a second sequential Flow)
runs a small stream; it must agree with the checker trivially (0 mismatches) and -- the real
point -- the stream must exercise every outcome the gate is meant to cover."""
import numpy as np
import pytest


class OracleCtx:
    """Implements the Context methods adversarial.C4Stream calls, on the CPU oracle."""

    def __init__(self):
        import oracle as O
        self.O = O
        self.flow = None

    def keygen(self, seeds):
        self.seeds = list(seeds)              # the signer keys, as txv_keygen sets them
        return [self.O.pubkey(s) for s in seeds]

    def set_validators(self, pubs, powers, chain):
        self.pubs, self.powers, self.chain = list(pubs), np.asarray(powers), chain.encode()

    def validator_info(self):
        return [self.O.sha256(p)[:20] for p in self.pubs], np.array([self.O.decode_ok(p) for p in self.pubs])

    def sign_votes(self, b, signer, chain):
        out = np.zeros((b.n, 64), np.uint8)
        for i in range(b.n):
            m = self.O.signbytes(int(b.height[i]), b.txhash(i), int(b.ts_sec[i]), int(b.ts_nanos[i]), chain.encode())
            out[i] = np.frombuffer(self.O.sign(self.seeds[int(signer[i])], m), np.uint8)
        return out

    def reset_flow(self):
        self.flow = None

    def add_votes(self, b, ev_cap=0):
        if self.flow is None:
            self.flow = self.O.Flow(self.pubs, self.powers, self.chain)
            self.done = set()
        st, _, fired = self.flow.add_batch(b, 4)
        ev = []
        for i in np.nonzero(fired)[0]:
            h = b.txhash(int(i))
            if h not in self.done:
                self.done.add(h)
                ev.append({"vote_index": int(i)})
        return st.astype(np.uint8) | (fired.astype(np.uint8) << 7), ev

    def verify_batch(self, b, pubs):
        return self.O.txvote_verify_batch(b, pubs, self.chain, 4)

    def query_tx(self, h):
        q = self.flow.query(h)
        return q


def test_c4_stream_covers_every_outcome(oracle_lib):
    import adversarial as A
    import txflow_amd as T
    ctx = OracleCtx()
    s = A.C4Stream(ctx, batch=6000, batches_per_epoch=2, oracle_threads=4, verify_slice=512)
    for _ in range(3):
        r = s.run_batch()
        assert r["status_mismatches"] == 0 and r["events_ok"] and r["verify_mismatches"] == 0
    s.stats["mismatches"] += s.check_sets()
    assert s.stats["mismatches"] == 0
    seen = s.stats["by_status"]
    for code in (T.ADDED, T.DUPLICATE, T.ERR_NIL, T.ERR_EMPTY_ADDR, T.ERR_UNKNOWN_VALIDATOR,
                 T.ERR_NONDETERMINISTIC, T.ERR_INVALID_SIGNATURE):
        assert seen.get(T.STATUS_NAMES[code], 0) > 0, (T.STATUS_NAMES[code], seen)
    assert s.stats["events"] > 0
    for name, share in A.CLASSES:               # every Appendix C class is generated at about its share
        if share:
            got = s.stats["class_generated"].get(name, 0) / s.stats["generated"]
            assert 0.7 * share <= got <= 1.4 * share, (name, got, share)
    # crafted keys: identity forgeries verify, order-2/4/8 and mixed-order forgeries verify only
    # when [k]T = 0, the undecodable key never -- so both verdicts occur among crafted votes
    names = [k[0] for k in s.crafted]
    for must in ("identity", "identity_y+p", "identity_negzero", "order2", "order4", "order8", "mixed8",
                 "undecodable"):
        assert must in names


def test_c4_keyless_classes_survive_checktx(oracle_lib):
    """Unknown-validator, empty-address and nil votes carry distinct signatures, so CheckTx's LRU
    (keyed by SHA-256(Signature), txvotepool.go:467-469) admits them and Appendix C's shares of
    those classes reach TxFlow (with shared / all-zero signatures only a few
    dozen empty-address votes survived 10^8)."""
    import adversarial as A
    import txflow_amd as T
    n = 40000
    s = A.C4Stream(OracleCtx(), batch=n, batches_per_epoch=2, oracle_threads=4, verify_slice=0)
    b, f = s.next_batch()
    gossip = np.nonzero(f["is_nil"] == 0)[0]
    m = len(gossip)
    sub = T.VoteBatch(m, height=f["height"][gossip], txhash_arena=b.txhash_arena, txhash_off=f["txoff"][gossip],
                      txhash_len=np.full(m, 64, np.uint32), ts_sec=np.full(m, 1_700_000_000, np.int64),
                      ts_nanos=f["ts_nanos"][gossip], addr=f["addr"][gossip], addr_len=f["addr_len"][gossip],
                      sig=f["sig"][gossip], sig_len=f["sig_len"][gossip])
    long_sigs = {int(q): sub.sig[64 * q:64 * q + 64].tobytes() + bytes(int(sub.sig_len[q]) - 64)
                 for q in np.nonzero(sub.sig_len > 64)[0]}
    pool = oracle_lib.Pool(size=(1 << 31) - 1, cache_size=1 << 16, max_txs_bytes=1 << 40)
    ops = pool.check_batch(sub, long_sigs)
    kind = f["kind"][gossip]
    for k, share in ((3, 0.005), (4, 0.0025)):
        admitted = int(np.count_nonzero((kind == k) & (ops == T.POOL_OK)))
        assert admitted >= 0.8 * share * n, (k, admitted)
    assert int(np.count_nonzero(f["is_nil"])) >= 0.8 * 0.001 * n

"""The configuration the C2 headline ships, fed adversarial keys and signatures on the GPU.

bench.py's C2 context runs radix-2^21 validator tables in the 12-position long-top layout
(``Tab<21>``, ed25519_dev.h: the top position takes an unsigned digit up to 2^21 + 1) over the
radix-2^26 base-point table, i.e. ``txv_k_scalarmult_dyn<512, 26, 21, 8, 2>`` for its 1M-vote
batches and ``txv_k_scalarmult_split<26, 21>`` + K1c below 768K votes (runtime.cpp
``launch_lane_votes``).  The rest of the GPU suite runs the library's automatic windows, so these
tests pin exactly that instantiation against the oracle (x/crypto ``ed25519.Verify`` rules,
SURVEY.md Appendix A; reference call sites ``types/tx_vote.go:110-119`` and
``types/vote_set.go:92-166``):

* every committed ed25519 vector -- 48 OpenSSL RFC 8032 signatures and 291 adversarial ones
  (all 8 torsion points with canonical / y >= p / "-0" encodings, mixed-order keys, undecodable
  keys, non-canonical R, s + L, top bits, bit flips, lengths 0 / 63 / 65) -- through
  ``txv_verify_bytes`` with its 81 distinct keys built into radix-2^21 tables, once at its own
  size (split kernel) and once tiled past 768K items (the V = 8 work-stealing kernel);
* the C4 adversarial stream (identity / order-2/4/8 / mixed-order / y >= p /
  "-0" / undecodable validator keys with forged signatures, bad signatures of every class,
  replays, conflicts) through TxFlow at 1M-vote batches (V = 8) and at 64k-vote batches (split),
  every per-vote status, fire bit, commit event, direct-Verify verdict and per-tx (sum, maj23)
  compared with the sequential oracle.

HBM: 81 keys x 1.70 GB of radix-2^21 tables (138 GB) + the 43 GB base table for the vectors;
43 registry keys (73 GB) + 43 GB for the stream -- one context at a time (the 1e8 gate runs the
full 111-key set in a process of its own)."""
import json
import os
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
SHIPPED = dict(table_w=21, base_w=26)
V8_MIN = 3 << 18          # launch_lane_votes: the V = 8 kernel from 768K work items


def _golden_cases():
    with open(os.path.join(HERE, "golden", "verify_vectors.json")) as f:
        vec = json.load(f)
    with open(os.path.join(HERE, "golden", "ed25519_openssl.json")) as f:
        ossl = json.load(f)
    cases = [(v["pub"], v["msg"], v["sig"], v["expect"], v["kind"]) for v in vec]
    cases += [(c["pub"], c["msg"], c["sig"], True, "openssl") for c in ossl]
    return cases


def test_shipped_windows_golden_vectors(oracle_lib):
    """All 339 fixtures at windows 26/21: the split kernel at their own size, the V = 8
    work-stealing kernel with the set tiled to 800k items (each item's verdict checked, and the
    oracle's verdict of every distinct triple equal to the recorded one)."""
    import txflow_amd as T
    cases = _golden_cases()
    keys = {c[0] for c in cases}
    # the caller-key tables take the registry's window only within the table budget
    budget_mb = int(len(keys) * 1.75 * 1024) + 4096
    ctx = T.Context(max_batch=1 << 20, max_txs=1 << 10, max_validators=16, table_budget_mb=budget_mb, **SHIPPED)
    try:
        rnd = random.Random(2106)
        seeds = [bytes(rnd.getrandbits(8) for _ in range(32)) for _ in range(4)]
        ctx.set_validators(ctx.keygen(seeds), [1, 1, 1, 1], "test_chain_id")
        assert (ctx.table_w, ctx.base_w) == (21, 26)
        pubs = [bytes.fromhex(c[0]) for c in cases]
        msgs = [bytes.fromhex(c[1]) for c in cases]
        sigs = [bytes.fromhex(c[2]) for c in cases]
        exp = np.array([c[3] for c in cases])
        orc = np.array([oracle_lib.verify(p, m, s) for p, m, s in zip(pubs, msgs, sigs)])
        assert np.array_equal(orc, exp), "oracle disagrees with the recorded verdicts"
        got = ctx.verify_bytes(pubs, msgs, sigs)
        bad = [(cases[i][4], bool(got[i])) for i in np.nonzero(got != exp)[0]]
        assert not bad, bad[:10]
        # tiled past the V = 8 threshold, in a shuffled order (kinds mixed inside every wave)
        n = 800_000
        perm = np.random.default_rng(2106).integers(0, len(cases), n)
        got8 = ctx.verify_bytes([pubs[i] for i in perm], [msgs[i] for i in perm], [sigs[i] for i in perm])
        bad8 = np.nonzero(got8 != exp[perm])[0]
        assert len(bad8) == 0, [(int(i), cases[int(perm[i])][4]) for i in bad8[:10]]
        assert exp.sum() > 60 and (~exp).sum() > 100
    finally:
        ctx.close()


def test_shipped_windows_c4_stream(oracle_lib):
    """C4 through TxFlow at windows 26/21: two epochs of 1M-vote batches (the V = 8 kernel the
    C2 bench runs) and three 64k-vote batches (split kernel), a 43-key validator set with all 11
    crafted keys, against the sequential oracle."""
    import gc
    import adversarial as A
    import txflow_amd as T
    import torch
    gc.collect()                    # contexts and tensors of earlier tests no one holds any more
    if torch.cuda.is_available():
        torch.cuda.empty_cache()
    free = torch.cuda.mem_get_info()[0] if torch.cuda.is_available() else 0
    ctx = T.Context(max_batch=(1 << 20) + (1 << 18), max_txs=1 << 17, max_validators=256, **SHIPPED)
    try:
        # 32 honest validators + the 11 crafted keys: 43 x 1.70 GB of radix-2^21 tables beside the
        # 43 GB base table, within what the suite's other resident contexts leave of the 288 GB
        # (the 1e8 gate, tools/gate/c4_gate.py --table-w 21 --base-w 26, runs all 100 + 11 alone)
        try:
            st = A.run_gate(ctx, 2 << 20, batch=1 << 20, batches_per_epoch=2, threads=16, log=lambda s: None,
                            n_honest=32)
        except Exception as e:
            raise AssertionError(f"{e} (free HBM before the context: {free / 2**30:.1f} GiB)") from e
        assert (ctx.table_w, ctx.base_w) == (21, 26)
        assert st["mismatches"] == 0, st
        assert st["votes"] >= 2 << 20 and st["events"] > 0
        assert st["by_status"].get("ErrVoteInvalidSignature", 0) > 0
        assert st["class_at_txflow"].get("crafted_key", 0) > 0
        st2 = A.run_gate(ctx, 3 * 65536, batch=65536, batches_per_epoch=3, threads=16, log=lambda s: None,
                         seed=0x7478763034 + 21, n_honest=32)
        assert st2["mismatches"] == 0, st2
        assert st2["class_at_txflow"].get("crafted_key", 0) > 0
    finally:
        ctx.close()

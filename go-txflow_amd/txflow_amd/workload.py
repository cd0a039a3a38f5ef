"""Synthetic TxVote workloads of BASELINE.json / SURVEY.md §8d (deterministic by seed).

    chainID "test_chain_id", Height 1, Timestamp = 1.7e9 s + (i+1) ns (non-zero nanos),
    tx_j = le64(j) || 24 PRNG bytes, TxHash = upper-hex(SHA-256(tx_j))  (types/tx_vote.go:43-45),
    TxKey = SHA-256(tx_j) (types/tx_vote.go:38-40; every vote of the tx carries it, reactor.go:113-118),
    validator seeds = SHA-512("txflow-val" || le32(i))[:32], keys derived on the GPU (RFC 8032).
Signatures are produced by the device signer (txv_sign_votes, mirroring MockPV.SignTxVote,
types/priv_validator.go:83-95).  The PRNG is numpy PCG64 seeded with the config seed.
"""
from __future__ import annotations

import hashlib
import struct

import numpy as np

from . import Context, VoteBatch

CHAIN_ID = "test_chain_id"
SEEDS = {"c1": 0x7478763031, "c2": 0x7478763032, "c3": 0x7478763033, "c4": 0x7478763034, "c5": 0x7478763035}


def validator_seeds(n: int, offset: int = 0):
    return [hashlib.sha512(b"txflow-val" + struct.pack("<I", offset + i)).digest()[:32] for i in range(n)]


def tx_hashes(n_txs: int, rng: np.random.Generator, first: int = 0) -> np.ndarray:
    """[n_txs, 64] uint8 upper-hex TxHash strings."""
    tail = rng.integers(0, 256, size=(n_txs, 24), dtype=np.uint8)
    out = np.zeros((n_txs, 64), np.uint8)
    for j in range(n_txs):
        tx = struct.pack("<Q", first + j) + tail[j].tobytes()
        out[j] = np.frombuffer(hashlib.sha256(tx).hexdigest().upper().encode(), np.uint8)
    return out


def tx_keys(hashes: np.ndarray) -> np.ndarray:
    """[n_txs, 32] TxKey = SHA-256(tx): the bytes the upper-hex TxHash spells"""
    return np.frombuffer(bytes.fromhex(hashes.tobytes().decode()), np.uint8).reshape(len(hashes), 32)


class Workload:
    """Every validator votes every tx (C1/C2/C3 shape), arrival order shuffled."""

    def __init__(self, ctx: Context, n_vals: int, n_txs: int, seed: int, powers=None, shard=None, n_shards=1,
                 tx_first: int = 0):
        self.rng = np.random.default_rng(seed)
        self.n_vals, self.n_txs = n_vals, n_txs
        self.seeds = validator_seeds(n_vals)
        self.pubs = ctx.keygen(self.seeds)
        self.powers = np.ones(n_vals, np.int64) if powers is None else np.asarray(powers, np.int64)
        ctx.set_validators(self.pubs, self.powers, CHAIN_ID)
        addrs, ok = ctx.validator_info()
        assert ok.all()
        self.addrs = np.frombuffer(b"".join(addrs), np.uint8).reshape(n_vals, 20)
        hashes = tx_hashes(n_txs, self.rng, tx_first)
        if n_shards > 1:
            # shard = SHA-256(TxHash)[0] mod G (txv_shard_of)
            from . import shard_of
            keep = shard_of([h.tobytes() for h in hashes], n_shards) == shard
            hashes = hashes[keep]
        self.hashes = hashes
        self.n_txs = len(hashes)
        n = self.n_txs * n_vals
        tx_of = np.repeat(np.arange(self.n_txs, dtype=np.uint32), n_vals)
        val_of = np.tile(np.arange(n_vals, dtype=np.uint32), self.n_txs)
        perm = self.rng.permutation(n)
        self.tx_of, self.val_of = tx_of[perm], val_of[perm]
        self.n = n
        self.txkeys = tx_keys(self.hashes)
        self.batch = VoteBatch(
            n, height=np.ones(n, np.int64), txhash_arena=self.hashes.reshape(-1),
            txhash_off=self.tx_of.astype(np.uint32) * 64, txhash_len=np.full(n, 64, np.uint32),
            ts_sec=np.full(n, 1_700_000_000, np.int64), ts_nanos=(np.arange(n, dtype=np.int64) % 999_999_999 + 1),
            addr=self.addrs[self.val_of], addr_len=np.full(n, 20, np.uint32),
            sig=np.zeros((n, 64), np.uint8), sig_len=np.full(n, 64, np.uint32), txkey=self.txkeys[self.tx_of])
        chunk = 1 << 18
        for s in range(0, n, chunk):
            e = min(n, s + chunk)
            sub = VoteBatch(e - s, height=self.batch.height[s:e], txhash_arena=self.batch.txhash_arena,
                            txhash_off=self.batch.txhash_off[s:e], txhash_len=self.batch.txhash_len[s:e],
                            ts_sec=self.batch.ts_sec[s:e], ts_nanos=self.batch.ts_nanos[s:e],
                            addr=self.batch.addr[20 * s:20 * e], addr_len=self.batch.addr_len[s:e],
                            sig=self.batch.sig[64 * s:64 * e], sig_len=self.batch.sig_len[s:e])
            self.batch.sig[64 * s:64 * e] = ctx.sign_votes(sub, self.val_of[s:e], CHAIN_ID).reshape(-1)

    def head(self, m: int) -> VoteBatch:
        """the first m votes as a VoteBatch (views; the TxHash arena is shared)"""
        b = self.batch
        return VoteBatch(m, height=b.height[:m], txhash_arena=b.txhash_arena, txhash_off=b.txhash_off[:m],
                         txhash_len=b.txhash_len[:m], ts_sec=b.ts_sec[:m], ts_nanos=b.ts_nanos[:m],
                         addr=b.addr[:20 * m], addr_len=b.addr_len[:m], sig=b.sig[:64 * m], sig_len=b.sig_len[:m],
                         txkey=None if b.txkey is None else b.txkey[:32 * m])

    def vote(self, i: int) -> dict:
        """oracle-style dict of vote i"""
        return dict(height=1, txhash=self.batch.txhash(i), ts_sec=int(self.batch.ts_sec[i]),
                    ts_nanos=int(self.batch.ts_nanos[i]), addr=self.batch.addr[20 * i:20 * i + 20].tobytes(),
                    sig=self.batch.sig[64 * i:64 * i + 64].tobytes())


class StreamWorkload:
    """C5: `n_vals` validators with power 1 + (rand mod 10^6), every validator
    votes every tx, arrival order = tx index + U(0, window) so a tx's votes straddle a few
    consecutive `batch`-vote batches; the stream is cut into batches in arrival order.

    replay > 0 adds SURVEY.md Appendix C's exact replays (gossip re-deliveries): after each vote,
    with probability `replay`, a byte-identical copy of an earlier vote -- half of them from the
    last `near` votes, half from anywhere before -- so a replay meets TxVotePool's LRU while its
    key is still cached (ErrTxInCache) or after it was evicted (admitted again; TxFlow then says
    DUPLICATE).  n = stream length, n_unique = distinct votes."""

    def __init__(self, ctx: Context, n_vals: int, n_txs: int, seed: int, batch: int = 65536, window: int = 128,
                 replay: float = 0.0, near: int = 4096):
        self.rng = np.random.default_rng(seed)
        self.n_vals, self.n_txs, self.batch_size = n_vals, n_txs, batch
        self.seeds = validator_seeds(n_vals)
        self.pubs = ctx.keygen(self.seeds)
        self.powers = 1 + (self.rng.integers(0, 1 << 62, n_vals) % 1_000_000).astype(np.int64)
        ctx.set_validators(self.pubs, self.powers, CHAIN_ID)
        addrs, ok = ctx.validator_info()
        assert ok.all()
        self.addrs = np.frombuffer(b"".join(addrs), np.uint8).reshape(n_vals, 20)
        self.hashes = tx_hashes(n_txs, self.rng, 1 << 40)
        self.txkeys = tx_keys(self.hashes)
        nu = n_txs * n_vals
        tx_of = np.repeat(np.arange(n_txs, dtype=np.int64), n_vals)
        val_of = np.tile(np.arange(n_vals, dtype=np.int64), n_txs)
        order = np.argsort(tx_of + self.rng.random(nu) * window, kind="stable")
        utx, uval = tx_of[order], val_of[order]
        unanos = np.arange(nu, dtype=np.int64) % 999_999_999 + 1
        # the distinct votes, signed in chunks (arrival order)
        usig = np.zeros((nu, 64), np.uint8)
        for s in range(0, nu, batch):
            e = min(nu, s + batch)
            m = e - s
            b = VoteBatch(m, height=np.ones(m, np.int64), txhash_arena=self.hashes.reshape(-1),
                          txhash_off=(utx[s:e] * 64).astype(np.uint32), txhash_len=np.full(m, 64, np.uint32),
                          ts_sec=np.full(m, 1_700_000_000, np.int64), ts_nanos=unanos[s:e],
                          addr=self.addrs[uval[s:e]], addr_len=np.full(m, 20, np.uint32),
                          sig=usig[s:e], sig_len=np.full(m, 64, np.uint32))
            usig[s:e] = ctx.sign_votes(b, uval[s:e].astype(np.uint32), CHAIN_ID).reshape(m, 64)
        # the stream: stream slot -> distinct vote
        if replay > 0:
            flag = self.rng.random(nu) < replay
            i = np.arange(nu, dtype=np.int64)
            near_src = np.maximum(0, i - self.rng.integers(0, near, nu))
            far_src = (self.rng.random(nu) * (i + 1)).astype(np.int64)
            rsrc = np.where(self.rng.random(nu) < 0.5, near_src, far_src)
            at = i + np.cumsum(flag) - flag               # stream slot of distinct vote i
            src = np.empty(nu + int(flag.sum()), np.int64)
            src[at] = i
            src[at[flag] + 1] = rsrc[flag]
        else:
            src = np.arange(nu, dtype=np.int64)
        self.src = src
        self.tx_of, self.val_of = utx[src], uval[src]
        self.n, self.n_unique = len(src), nu
        self.batches = []
        for s in range(0, self.n, batch):
            e = min(self.n, s + batch)
            m = e - s
            q = src[s:e]
            b = VoteBatch(m, height=np.ones(m, np.int64), txhash_arena=self.hashes.reshape(-1),
                          txhash_off=(utx[q] * 64).astype(np.uint32), txhash_len=np.full(m, 64, np.uint32),
                          ts_sec=np.full(m, 1_700_000_000, np.int64), ts_nanos=unanos[q],
                          addr=self.addrs[uval[q]], addr_len=np.full(m, 20, np.uint32),
                          sig=usig[q], sig_len=np.full(m, 64, np.uint32), txkey=self.txkeys[utx[q]])
            self.batches.append(b)
        n = self.n
        first = np.full(n_txs, -1, np.int64)
        bidx = np.arange(n) // batch
        # batch index of each tx's first vote
        rev = np.arange(n)[::-1]
        first[self.tx_of[rev]] = bidx[rev]
        self.first_batch = first

"""Multi-GPU decomposition of the TxVote path, over the C-ABI's own shard rule
and packed commit state (include/txvote.h: txv_shard_of, txv_pack_commit_state,
txv_commit_state_pack_host / txv_commit_state_unpack), so a Go caller and this mirror share
one definition.

Votes are partitioned by transaction: shard(TxHash) = SHA-256(TxHash bytes)[0] mod G.  Every
TxVoteSet (types/vote_set.go:19-31) then lives on exactly one rank, so the per-(tx, validator)
dup/conflict resolution and the stake tally are rank-local and no data-path collective is
needed.  Per-vote arrival order is preserved within a shard (each rank keeps the global
arrival order of its own votes).

Ingest (txvotepool/reactor.go:170-190 -> txvotepool.go:187-261): TxVotePool is ONE
order-dependent LRU keyed by SHA-256(Signature) with one Size cap, so CheckTx cannot be split by
shard without changing which votes it admits.  It runs on one owner rank (the node's reactor
process); the votes it admits are routed to the rank owning their TxHash (route_admitted), in
arrival order, by one scatter per batch (scatter_batches) -- the path's one real data exchange
besides the commit-state all-gather.

Exchange: one all-gather per batch of the packed per-shard commit state --
[n_sets][commit bitmap][stake sums][digests] over the shard's set ids, numbered in first-seen
order, each set named by tx_digest(TxHash) = SHA-256(TxHash)[0:16] (RCCL over xGMI on GPUs, gloo
in the CPU tests) -- which gives every rank the global committed-tx set and stakes, by name, from
the gathered buffers alone (merge_states).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import VoteBatch, commit_state_unpack, shard_of as _shard_of, tx_digest


def shard_of(txhashes: Sequence[bytes], n_shards: int) -> np.ndarray:
    """shard of each TxHash (txv_shard_of)"""
    return _shard_of(list(txhashes), n_shards) if n_shards > 1 else np.zeros(len(txhashes), np.uint32)


def partition(txhashes: Sequence[bytes], n_shards: int) -> List[np.ndarray]:
    """indices of the votes owned by each shard, each in global arrival order"""
    owner = shard_of(txhashes, n_shards)
    return [np.nonzero(owner == s)[0] for s in range(n_shards)]


def merge_states(gathered: np.ndarray, n_shards: int, n_sets_cap: int) -> Tuple[set, Dict[bytes, int]]:
    """gathered: the all-gathered packed states, [n_shards * txv_commit_state_bytes(cap)] bytes.
    Returns (the global committed set, {digest: stake}), every TxVoteSet named by its
    tx_digest(TxHash) as packed by its owner -- no host-side knowledge of other ranks' sets."""
    rows = np.ascontiguousarray(gathered, np.uint8).reshape(n_shards, -1)
    committed, stakes = set(), {}
    for s in range(n_shards):
        com, sums, dig = commit_state_unpack(rows[s], n_sets_cap)
        for i in range(len(com)):
            k = dig[i].tobytes()
            stakes[k] = int(sums[i])
            if com[i]:
                committed.add(k)
    return committed, stakes


def subset(b: VoteBatch, idx: np.ndarray) -> VoteBatch:
    """the votes idx of b (in that order) as a batch with a compact TxHash arena of their own"""
    idx = np.asarray(idx, np.int64)
    n = len(idx)
    ln = b.txhash_len[idx].astype(np.int64)
    off = np.zeros(n, np.int64)
    if n:
        off[1:] = np.cumsum(ln)[:-1]
    arena = np.zeros(max(int(ln.sum()), 1), np.uint8)
    for j, i in enumerate(idx):          # TxHashes are short; the arena is rebuilt per rank
        o, l = int(b.txhash_off[i]), int(b.txhash_len[i])
        arena[off[j]:off[j] + l] = b.txhash_arena[o:o + l]
    a20 = (idx[:, None] * 20 + np.arange(20)).reshape(-1)
    a64 = (idx[:, None] * 64 + np.arange(64)).reshape(-1)
    return VoteBatch(n, height=b.height[idx], txhash_arena=arena, txhash_off=off.astype(np.uint32),
                     txhash_len=ln.astype(np.uint32), ts_sec=b.ts_sec[idx], ts_nanos=b.ts_nanos[idx],
                     addr=b.addr[a20], addr_len=b.addr_len[idx], sig=b.sig[a64], sig_len=b.sig_len[idx],
                     is_nil=None if b.is_nil is None else b.is_nil[idx],
                     txkey=None if b.txkey is None else b.txkey[(idx[:, None] * 32 + np.arange(32)).reshape(-1)])


def route_admitted(b: VoteBatch, pool_status: np.ndarray, n_shards: int, ok: int = 0) -> List[np.ndarray]:
    """CheckTx ran on the owner (pool_status per vote, TXV_POOL_*); each admitted vote goes to the
    rank owning its TxHash: per rank, the indices of its admitted votes in arrival order"""
    adm = np.nonzero(np.asarray(pool_status) == ok)[0]
    owner = shard_of([b.txhash(int(i)) for i in adm], n_shards)
    return [adm[owner == r] for r in range(n_shards)]


_COLS = (("height", np.int64, 1), ("txhash_off", np.uint32, 1), ("txhash_len", np.uint32, 1),
         ("ts_sec", np.int64, 1), ("ts_nanos", np.int32, 1), ("addr", np.uint8, 20), ("addr_len", np.uint32, 1),
         ("sig", np.uint8, 64), ("sig_len", np.uint32, 1), ("txkey", np.uint8, 32))


def pack_batch(b: VoteBatch) -> np.ndarray:
    """a batch as one byte buffer (n, arena length, then the columns): what the route sends"""
    parts = [np.array([b.n, len(b.txhash_arena), int(b.txkey is not None)], np.int64).view(np.uint8)]
    parts.append(b.txhash_arena)
    for name, dt, _ in _COLS:
        col = getattr(b, name)
        if col is None:
            continue
        parts.append(np.ascontiguousarray(col, dt).view(np.uint8).reshape(-1))
    return np.concatenate(parts)


def unpack_batch(buf: np.ndarray) -> VoteBatch:
    buf = np.ascontiguousarray(buf, np.uint8)
    n, al, has_key = (int(x) for x in buf[:24].view(np.int64))
    o = 24
    arena = buf[o:o + al].copy()
    o += al
    cols = {}
    for name, dt, w in _COLS:
        if name == "txkey" and not has_key:
            cols[name] = None
            continue
        nb = n * w * np.dtype(dt).itemsize
        cols[name] = buf[o:o + nb].view(dt).copy()
        o += nb
    return VoteBatch(n, txhash_arena=arena, **cols)


def scatter_batches(dist, batches: Optional[Sequence[VoteBatch]], src: int = 0, device: str = "cpu") -> VoteBatch:
    """the route's exchange: rank src sends batches[r] to rank r (torch.distributed scatter of the
    packed buffers, padded to the largest; gloo on the CPU, RCCL with device='cuda:k'); every
    rank returns its own batch"""
    import torch
    world, rank = dist.get_world_size(), dist.get_rank()
    size = torch.zeros(world, dtype=torch.int64, device=device)
    bufs = None
    if rank == src:
        bufs = [pack_batch(b) for b in batches]
        size = torch.tensor([len(x) for x in bufs], dtype=torch.int64, device=device)
    dist.broadcast(size, src)
    m = int(size.max().item())
    out = torch.zeros(m, dtype=torch.uint8, device=device)
    lst = None
    if rank == src:
        lst = []
        for x in bufs:
            t = torch.zeros(m, dtype=torch.uint8, device=device)
            t[:len(x)] = torch.from_numpy(x).to(device)
            lst.append(t)
    dist.scatter(out, lst, src=src)
    return unpack_batch(out[:int(size[rank].item())].cpu().numpy())


def name_sets(txhashes: Sequence[bytes]) -> Dict[bytes, bytes]:
    """{digest: TxHash} for the TxHashes a caller knows (to print a merged state by TxHash)"""
    return {tx_digest(h): bytes(h) for h in txhashes}

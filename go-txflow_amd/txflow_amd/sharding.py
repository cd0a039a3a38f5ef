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
process); the votes it admits are packed per rank on the owner's GPU by the C-ABI's
txv_route_admitted (kernels_route.hip: shard, arrival-order rank and TxHash arena offset of every
admitted vote, each rank's columns written into its own buffer) -- or on the host by
txv_route_pack_host -- sent buffer r to rank r (scatter_routed: one meta broadcast + point-to-point
sends, RCCL over xGMI), and each rank runs its TxFlow chain straight from the received buffer in
its HBM (Context.submit_routed): the path's one real data exchange besides the commit-state
all-gather.

Exchange: one all-gather per batch of the packed per-shard commit state --
[n_sets][commit bitmap][stake sums][digests] over the shard's set ids, numbered in first-seen
order, each set named by tx_digest(TxHash) = SHA-256(TxHash)[0:16] (RCCL over xGMI on GPUs, gloo
in the CPU tests) -- which gives every rank the global committed-tx set and stakes, by name, from
the gathered buffers alone (merge_states).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import ROUTE_META_DTYPE, VoteBatch, commit_state_unpack, lib, shard_of as _shard_of, tx_digest


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
    """the votes idx of b (in that order) as a batch with a compact TxHash arena of their own
    (numpy gathers, no per-vote loop)"""
    idx = np.asarray(idx, np.int64)
    n = len(idx)
    ln = b.txhash_len[idx].astype(np.int64)
    off = np.zeros(n, np.int64)
    if n:
        off[1:] = np.cumsum(ln)[:-1]
    total = int(ln.sum())
    if total:
        src = np.repeat(b.txhash_off[idx].astype(np.int64) - off, ln) + np.arange(total, dtype=np.int64)
        arena = b.txhash_arena[src]
    else:
        arena = np.zeros(1, np.uint8)
    a20 = (idx[:, None] * 20 + np.arange(20)).reshape(-1)
    a64 = (idx[:, None] * 64 + np.arange(64)).reshape(-1)
    return VoteBatch(n, height=b.height[idx], txhash_arena=arena, txhash_off=off.astype(np.uint32),
                     txhash_len=ln.astype(np.uint32), ts_sec=b.ts_sec[idx], ts_nanos=b.ts_nanos[idx],
                     addr=b.addr[a20], addr_len=b.addr_len[idx], sig=b.sig[a64], sig_len=b.sig_len[idx],
                     is_nil=None if b.is_nil is None else b.is_nil[idx],
                     txkey=None if b.txkey is None else b.txkey[(idx[:, None] * 32 + np.arange(32)).reshape(-1)])


def batch_shards(b: VoteBatch, n_shards: int) -> np.ndarray:
    """txv_shard_of of every vote of b, straight over its TxHash arena (a nil vote: the shard of
    the empty TxHash, as the route takes it)"""
    if n_shards <= 1 or b.n == 0:
        return np.zeros(b.n, np.uint32)
    ln = b.txhash_len if b.is_nil is None else np.where(b.is_nil != 0, 0, b.txhash_len).astype(np.uint32)
    ln = np.ascontiguousarray(ln, np.uint32)
    out = np.zeros(b.n, np.uint32)
    rc = lib().txv_shard_of(b.txhash_arena.ctypes.data, b.txhash_off.ctypes.data, ln.ctypes.data, b.n, n_shards,
                            out.ctypes.data)
    if rc:
        raise ValueError(f"txv_shard_of failed ({rc})")
    return out


def route_admitted(b: VoteBatch, pool_status: np.ndarray, n_shards: int, ok: int = 0) -> List[np.ndarray]:
    """CheckTx ran on the owner (pool_status per vote, TXV_POOL_*); each admitted vote goes to the
    rank owning its TxHash: per rank, the indices of its admitted votes in arrival order (the
    index view of what txv_route_admitted packs)"""
    adm = np.asarray(pool_status) == ok
    owner = batch_shards(b, n_shards)
    return [np.nonzero(adm & (owner == r))[0] for r in range(n_shards)]


def scatter_routed(dist, bufs, metas: Optional[np.ndarray], src: int = 0, device: str = "cpu"):
    """the route's exchange: rank src holds the n_shards route buffers ([n_shards, stride] uint8
    torch tensor on `device`, from txv_route_admitted / txv_route_pack_host) and their metas; one
    broadcast of the metas, then buffer r to rank r point to point, exactly meta[r].bytes of it
    (RCCL over xGMI with device='cuda:k': the buffers never leave HBM).  Every rank returns (its
    buffer as a uint8 tensor on `device`, its meta)."""
    import torch
    world, rank = dist.get_world_size(), dist.get_rank()
    mt = torch.zeros(world * 4, dtype=torch.int64, device=device)
    if rank == src:
        mt.copy_(torch.from_numpy(np.ascontiguousarray(metas, ROUTE_META_DTYPE).view(np.int64).reshape(-1)).to(device))
    dist.broadcast(mt, src)
    allm = mt.cpu().numpy().view(ROUTE_META_DTYPE)
    mine = allm[rank].copy()
    size = int(mine["bytes"])
    if rank == src:
        reqs = [dist.isend(bufs[r, :int(allm[r]["bytes"])].contiguous(), dst=r) for r in range(world) if r != src]
        for q in reqs:
            q.wait()
        return bufs[src, :size], mine
    out = torch.empty(size, dtype=torch.uint8, device=device)
    dist.recv(out, src=src)
    return out, mine


def name_sets(txhashes: Sequence[bytes]) -> Dict[bytes, bytes]:
    """{digest: TxHash} for the TxHashes a caller knows (to print a merged state by TxHash)"""
    return {tx_digest(h): bytes(h) for h in txhashes}

"""Multi-GPU decomposition of the TxVote path, over the C-ABI's own shard rule
and packed commit state (include/txvote.h: txv_shard_of, txv_pack_commit_state,
txv_commit_state_pack_host / txv_commit_state_unpack), so a Go caller and this mirror share
one definition.

Votes are partitioned by transaction: shard(TxHash) = SHA-256(TxHash bytes)[0] mod G.  Every
TxVoteSet (types/vote_set.go:19-31) then lives on exactly one rank, so the per-(tx, validator)
dup/conflict resolution and the stake tally are rank-local and no data-path collective is
needed.  Per-vote arrival order is preserved within a shard (each rank keeps the global
arrival order of its own votes).  The only exchange is one all-gather per batch of the packed
per-shard commit state -- [n_sets][commit bitmap][stake sums] over the shard's set ids, which
are numbered in first-seen order -- (RCCL over xGMI on GPUs, gloo in the CPU tests), which
gives every rank the global committed-tx set and stakes.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np

from . import commit_state_unpack, shard_of as _shard_of


def shard_of(txhashes: Sequence[bytes], n_shards: int) -> np.ndarray:
    """shard of each TxHash (txv_shard_of)"""
    return _shard_of(list(txhashes), n_shards) if n_shards > 1 else np.zeros(len(txhashes), np.uint32)


def partition(txhashes: Sequence[bytes], n_shards: int) -> List[np.ndarray]:
    """indices of the votes owned by each shard, each in global arrival order"""
    owner = shard_of(txhashes, n_shards)
    return [np.nonzero(owner == s)[0] for s in range(n_shards)]


def merge_states(gathered: np.ndarray, n_shards: int, n_sets_cap: int,
                 local_keys: Sequence[Sequence[bytes]]) -> Tuple[set, Dict[bytes, int]]:
    """gathered: the all-gathered packed states, [n_shards * txv_commit_state_bytes(cap)] bytes;
    local_keys[s][i] = TxHash of shard s's set id i.  Returns (global committed TxHash set,
    {TxHash: stake})."""
    rows = np.ascontiguousarray(gathered, np.uint8).reshape(n_shards, -1)
    committed, stakes = set(), {}
    for s in range(n_shards):
        com, sums = commit_state_unpack(rows[s], n_sets_cap)
        for i in range(min(len(com), len(local_keys[s]))):
            k = bytes(local_keys[s][i])
            stakes[k] = int(sums[i])
            if com[i]:
                committed.add(k)
    return committed, stakes

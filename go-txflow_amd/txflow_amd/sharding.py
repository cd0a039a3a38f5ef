"""Multi-GPU decomposition of the TxVote path.

Votes are partitioned by transaction: shard(TxHash) = SHA-256(TxHash bytes)[0] mod G.  Every
TxVoteSet (types/vote_set.go:19-31) then lives on exactly one rank, so the per-(tx, validator)
dup/conflict resolution and the stake tally are rank-local and no data-path collective is
needed.  Per-vote arrival order is preserved within a shard (each rank keeps the global
arrival order of its own votes).  The only exchange is one all-gather per batch of the
per-shard commit bitmaps (RCCL over xGMI on GPUs, gloo in the CPU tests), which gives every
rank the global committed-tx set.
"""
from __future__ import annotations

import hashlib
from typing import Iterable, List, Sequence

import numpy as np


def shard_of(txhash: bytes, n_shards: int) -> int:
    return hashlib.sha256(txhash).digest()[0] % n_shards if n_shards > 1 else 0


def partition(txhashes: Sequence[bytes], n_shards: int) -> List[np.ndarray]:
    """indices of the votes owned by each shard, each in global arrival order"""
    owner = np.array([shard_of(h, n_shards) for h in txhashes], dtype=np.int64)
    return [np.nonzero(owner == s)[0] for s in range(n_shards)]


def pack_bitmap(committed_ids: Iterable[int], n_bits: int) -> np.ndarray:
    words = np.zeros((n_bits + 31) // 32, dtype=np.uint32)
    for i in committed_ids:
        words[i >> 5] |= np.uint32(1 << (i & 31))
    return words


def unpack_bitmap(words: np.ndarray) -> np.ndarray:
    bits = np.unpackbits(words.view(np.uint8), bitorder="little")
    return np.nonzero(bits)[0]


def merge_gathered(gathered: np.ndarray, n_shards: int, local_keys: Sequence[Sequence[bytes]]) -> set:
    """gathered: [n_shards * words] from an all-gather of per-shard bitmaps; local_keys[s][i] is
    the TxHash of shard s's set id i.  Returns the global committed TxHash set."""
    words = gathered.reshape(n_shards, -1)
    out = set()
    for s in range(n_shards):
        for i in unpack_bitmap(words[s]):
            if i < len(local_keys[s]):
                out.add(bytes(local_keys[s][i]))
    return out

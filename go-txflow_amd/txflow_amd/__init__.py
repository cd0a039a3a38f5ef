"""Python binding of libtxvote.so (include/txvote.h) and a host-side mirror of the
reference's TxVote admission API (Fantom-foundation/go-txflow):

    TxVote            types/tx_vote.go:48-55   (SignBytes :83-89, Verify :110-119, Size :144-150)
    TxFlow            txflow/service.go:23-234 (TryAddVote :169-188, addVote :192-234)
    TxVoteSetView     types/vote_set.go:178-227 readers (Stake, HasTwoThirdsMajority, ...)
    Errors            types/tx_vote.go:30-35 sentinels + tendermint ErrVoteInvalidValidator*

All verification and tallying runs in the HIP kernels of libtxvote.so; this module only
marshals arguments.  Importing it on a machine without the built library raises, and
creating a context without a GPU raises: there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import hashlib
import weakref
import os
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "build", "libtxvote.so")
if os.environ.get("TXV_LIB_PATH"):          # experiment builds (tools/); the product default is in-tree
    LIB_PATH = os.environ["TXV_LIB_PATH"]

# status codes (include/txvote.h)
ADDED, DUPLICATE, ERR_NIL, ERR_EMPTY_ADDR, ERR_UNKNOWN_VALIDATOR, ERR_NONDETERMINISTIC, \
    ERR_INVALID_SIGNATURE, ERR_INVALID_VALIDATOR_ADDRESS, ERR_SIGNBYTES = range(9)
STATUS_FIRED = 0x80
STATUS_NAMES = {ADDED: "ADDED", DUPLICATE: "DUPLICATE", ERR_NIL: "ErrVoteNil",
                ERR_EMPTY_ADDR: "ErrVoteInvalidValidatorAddress(empty)",
                ERR_UNKNOWN_VALIDATOR: "ErrVoteInvalidValidatorIndex",
                ERR_NONDETERMINISTIC: "ErrVoteNonDeterministicSignature",
                ERR_INVALID_SIGNATURE: "ErrVoteInvalidSignature",
                ERR_INVALID_VALIDATOR_ADDRESS: "ErrVoteInvalidValidatorAddress",
                ERR_SIGNBYTES: "amino time out of range (reference panics)"}


class TxVoteError(Exception):
    """Sentinel-cause error mirroring the reference's error values."""

    def __init__(self, code: int):
        super().__init__(STATUS_NAMES.get(code & 0x7F, str(code)))
        self.code = code & 0x7F


class TxvInfraError(RuntimeError):
    pass


class _Cfg(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("max_batch", ctypes.c_uint32), ("max_txs", ctypes.c_uint32),
                ("max_validators", ctypes.c_uint32), ("max_accepted", ctypes.c_uint32),
                ("max_msg_bytes", ctypes.c_uint32), ("flags", ctypes.c_uint32),
                ("table_budget_mb", ctypes.c_uint32), ("key_arena_bytes", ctypes.c_uint64)]


class _Votes(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint32), ("is_nil", ctypes.c_void_p), ("height", ctypes.c_void_p),
                ("txhash", ctypes.c_void_p), ("txhash_off", ctypes.c_void_p), ("txhash_len", ctypes.c_void_p),
                ("ts_sec", ctypes.c_void_p), ("ts_nanos", ctypes.c_void_p), ("addr", ctypes.c_void_p),
                ("addr_len", ctypes.c_void_p), ("sig", ctypes.c_void_p), ("sig_len", ctypes.c_void_p),
                ("txkey", ctypes.c_void_p)]


class _PoolCfg(ctypes.Structure):
    _fields_ = [("size", ctypes.c_uint32), ("cache_size", ctypes.c_uint32), ("max_txs_bytes", ctypes.c_uint64),
                ("max_msg_bytes", ctypes.c_uint32), ("flags", ctypes.c_uint32)]


class _WireVotes(ctypes.Structure):
    _fields_ = [(f, ctypes.c_void_p) for f in ("status", "height", "txhash_off", "txhash_len", "txkey", "ts_sec",
                                              "ts_nanos", "addr", "addr_len", "sig", "sig_len", "sig_off")]


class _Event(ctypes.Structure):
    _fields_ = [("vote_index", ctypes.c_uint32), ("tx_index", ctypes.c_uint32), ("sum", ctypes.c_int64)]


EVENT_DTYPE = np.dtype([("vote_index", "<u4"), ("tx_index", "<u4"), ("sum", "<i8")])   # txv_commit_event
# txv_route_meta: one rank's ingest-route buffer (include/txvote.h txv_route_admitted)
ROUTE_META_DTYPE = np.dtype([("n", "<u4"), ("max_txhash_len", "<u4"), ("flags", "<u4"), ("reserved", "<u4"),
                             ("arena_bytes", "<u8"), ("bytes", "<u8")])
ROUTE_TXKEY, ROUTE_NIL = 0x1, 0x2


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise TxvInfraError(f"libtxvote.so not built at {LIB_PATH} (run __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        vp, u32, i32, i64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int32, ctypes.c_int64
        sig = {
            "txv_init": ([ctypes.POINTER(_Cfg), ctypes.POINTER(vp)], ctypes.c_int),
            "txv_destroy": ([vp], None),
            "txv_last_error": ([vp], ctypes.c_char_p),
            "txv_device_name": ([vp, ctypes.c_char_p, u32], ctypes.c_int),
            "txv_set_validators": ([vp, vp, vp, u32, ctypes.c_char_p, u32], ctypes.c_int),
            "txv_get_validator_info": ([vp, vp, vp, u32], ctypes.c_int),
            "txv_verify_batch": ([vp, ctypes.POINTER(_Votes), vp, vp], ctypes.c_int),
            "txv_verify_bytes": ([vp, vp, vp, vp, vp, vp, vp, u32, vp], ctypes.c_int),
            "txv_add_votes": ([vp, ctypes.POINTER(_Votes), vp, vp, u32, ctypes.POINTER(u32)], ctypes.c_int),
            "txv_query_tx": ([vp, ctypes.c_char_p, u32, ctypes.POINTER(i64), ctypes.POINTER(ctypes.c_uint8)],
                             ctypes.c_int),
            "txv_num_tx_sets": ([vp], u32),
            "txv_total_power": ([vp], i64),
            "txv_signbytes": ([i64, ctypes.c_char_p, u32, i64, i32, ctypes.c_char_p, u32, ctypes.c_char_p, u32],
                              ctypes.c_int),
            "txv_txvote_size": ([i64, u32, i64, i32, u32, u32], ctypes.c_int),
            "txv_keygen": ([vp, vp, u32, vp], ctypes.c_int),
            "txv_sign_votes": ([vp, ctypes.POINTER(_Votes), vp, ctypes.c_char_p, u32, vp], ctypes.c_int),
            "txv_stage": ([vp, u32, ctypes.POINTER(_Votes)], ctypes.c_int),
            "txv_run_staged": ([vp, u32, vp], ctypes.c_int),
            "txv_fetch_staged": ([vp, u32, vp, vp, u32, ctypes.POINTER(u32)], ctypes.c_int),
            "txv_commit_bitmap": ([vp, ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_uint64)], ctypes.c_int),
            "txv_reset_tally": ([vp], ctypes.c_int),
            "txv_reset_flow": ([vp], ctypes.c_int),
            "txv_sync": ([vp], ctypes.c_int),
            "txv_flow_stream": ([vp], vp),
            "txv_fe_selftest": ([vp, vp, vp, vp, u32, ctypes.c_int], ctypes.c_int),
            "txv_copy_commit_bitmap": ([vp, vp, ctypes.c_uint64], ctypes.c_int),
            "txv_valu_probe": ([vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)], ctypes.c_int),
            "txv_table_window": ([vp], ctypes.c_int),
            "txv_validator_tables_built": ([vp], ctypes.c_int),
            "txv_staged_bytes": ([vp], ctypes.c_int64),
            "txv_base_window": ([vp], ctypes.c_int),
            "txv_sig_keys": ([vp, ctypes.POINTER(_Votes), vp, vp, vp], ctypes.c_int),
            "txv_bind_host_numa": ([vp], ctypes.c_int),
            "txv_copy_set_sums": ([vp, vp, u32], ctypes.c_int),
            "txv_get_votes": ([vp, ctypes.c_char_p, u32, vp, vp, vp, u32, ctypes.POINTER(u32)], ctypes.c_int),
            "txv_submit_votes": ([vp, ctypes.POINTER(_Votes), ctypes.POINTER(ctypes.c_uint64)], ctypes.c_int),
            "txv_submit_checked": ([vp, ctypes.POINTER(_Votes), vp, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)],
                                   ctypes.c_int),
            "txv_wait_votes": ([vp, ctypes.c_uint64, vp, vp, u32, ctypes.POINTER(u32)], ctypes.c_int),
            "txv_pool_new": ([ctypes.POINTER(_PoolCfg), i64, ctypes.POINTER(vp)], ctypes.c_int),
            "txv_pool_free": ([vp], None),
            "txv_pool_check": ([vp, vp, ctypes.POINTER(_Votes), vp, vp, vp], ctypes.c_int),
            "txv_pool_check_submit": ([vp, vp, ctypes.POINTER(_Votes), vp, vp, ctypes.POINTER(ctypes.c_uint64)],
                                      ctypes.c_int),
            "txv_pool_check_wait": ([vp, ctypes.c_uint64, vp], ctypes.c_int),
            "txv_pool_check_keys": ([vp, vp, vp, vp, u32, vp], ctypes.c_int),
            "txv_pool_update": ([vp, vp, i64, ctypes.POINTER(_Votes), vp, vp], ctypes.c_int),
            "txv_pool_update_keys": ([vp, vp, i64, vp, vp, u32], ctypes.c_int),
            "txv_pool_update_submit": ([vp, vp, i64, ctypes.POINTER(_Votes), vp, vp], ctypes.c_int),
            "txv_pool_reap": ([vp, i64, vp, vp, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)], ctypes.c_int),
            "txv_pool_flush": ([vp], ctypes.c_int),
            "txv_pool_size": ([vp], i64),
            "txv_pool_txs_bytes": ([vp], i64),
            "txv_pool_height": ([vp], i64),
            "txv_pool_cache_keys": ([vp, vp, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)], ctypes.c_int),
            "txv_pool_sync": ([vp], ctypes.c_int),
            "txv_decode_msgs": ([vp, vp, ctypes.c_uint64, vp, vp, u32, u32, ctypes.POINTER(_WireVotes)], ctypes.c_int),
            "txv_decode_stage": ([vp, vp, ctypes.c_uint64, vp, vp, u32], ctypes.c_int),
            "txv_decode_run": ([vp, u32, u32, ctypes.POINTER(ctypes.c_float)], ctypes.c_int),
            "txv_decode_fetch": ([vp, ctypes.POINTER(_WireVotes)], ctypes.c_int),
            "txv_pool_receive": ([vp, vp, vp, ctypes.c_uint64, vp, vp, u32, vp, vp], ctypes.c_int),
            "txv_ingest_msgs": ([vp, vp, vp, ctypes.c_uint64, vp, vp, u32, vp, vp, vp, vp, u32, ctypes.POINTER(u32)],
                                ctypes.c_int),
            "txv_ingest_submit": ([vp, vp, vp, ctypes.c_uint64, vp, vp, u32, vp, vp, ctypes.POINTER(ctypes.c_uint64)],
                                  ctypes.c_int),
            "txv_ingest_wait": ([vp, ctypes.c_uint64, vp, vp, u32, ctypes.POINTER(u32)], ctypes.c_int),
            "txv_pool_prepare": ([vp, vp, ctypes.POINTER(_Votes), vp, vp, vp, vp], ctypes.c_int),
            "txv_ingest_decode": ([vp, vp, vp, ctypes.c_uint64, vp, vp, u32, ctypes.POINTER(ctypes.c_uint64)],
                                  ctypes.c_int),
            "txv_ingest_admit": ([vp, ctypes.c_uint64, vp, vp], ctypes.c_int),
            "txv_ingest_admit_submit": ([vp, ctypes.c_uint64, vp, vp], ctypes.c_int),
            "txv_ingest_admit_finish": ([vp, ctypes.c_uint64, vp, vp], ctypes.c_int),
            "txv_encode_msgs": ([ctypes.POINTER(_Votes), vp, vp, vp, vp, ctypes.c_uint64, vp, vp,
                                 ctypes.POINTER(ctypes.c_uint64)], ctypes.c_int),
            "txv_query_txs": ([vp, vp, vp, vp, u32, vp, vp, vp, vp], ctypes.c_int),
            "txv_make_commit": ([vp, ctypes.c_char_p, u32, vp, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)],
                                ctypes.c_int),
            "txv_save_tx_bytes": ([vp, ctypes.c_char_p, u32, vp, ctypes.c_uint64, vp], ctypes.c_int),
            "txv_host_register": ([vp, vp, ctypes.c_uint64], ctypes.c_int),
            "txv_host_unregister": ([vp, vp], ctypes.c_int),
            "txv_shard_of": ([vp, vp, vp, u32, u32, vp], ctypes.c_int),
            "txv_commit_state_bytes": ([u32], ctypes.c_uint64),
            "txv_pack_commit_state": ([vp, vp, u32], ctypes.c_int),
            "txv_set_commit_sink": ([vp, u32, vp, u32], ctypes.c_int),
            "txv_slot_kernel_ms": ([vp, u32, ctypes.POINTER(ctypes.c_float)], ctypes.c_int),
            "txv_slot_verify_ms": ([vp, u32, ctypes.POINTER(ctypes.c_float)], ctypes.c_int),
            "txv_read_commit_state": ([vp, vp, u32], ctypes.c_int),
            "txv_commit_state_pack_host": ([u32, vp, vp, vp, u32, vp], ctypes.c_int),
            "txv_commit_state_unpack": ([vp, u32, ctypes.POINTER(u32), vp, vp, vp, u32], ctypes.c_int),
            "txv_route_bytes": ([u32, ctypes.c_uint64, u32], ctypes.c_uint64),
            "txv_route_admitted": ([vp, ctypes.POINTER(_Votes), vp, u32, vp, ctypes.c_uint64, vp], ctypes.c_int),
            "txv_route_checked": ([vp, ctypes.POINTER(_Votes), vp, ctypes.c_uint64, u32, vp, ctypes.c_uint64, vp],
                                  ctypes.c_int),
            "txv_route_pack_host": ([ctypes.POINTER(_Votes), vp, u32, vp, ctypes.c_uint64, vp], ctypes.c_int),
            "txv_route_view": ([vp, ctypes.c_uint64, ctypes.POINTER(_Votes)], ctypes.c_int),
            "txv_submit_routed": ([vp, vp, vp, ctypes.POINTER(ctypes.c_uint64)], ctypes.c_int),
        }
        for name, (args, res) in sig.items():
            if os.environ.get("TXV_LIB_PATH") and not hasattr(L, name):
                continue            # an experiment build of an older ABI (A/B runs of tools/)
            f = getattr(L, name)
            f.argtypes = args
            f.restype = res
        _lib = L
    return _lib


EXPORTED_SYMBOLS = [
    "txv_init", "txv_destroy", "txv_last_error", "txv_device_name", "txv_set_validators",
    "txv_get_validator_info", "txv_verify_batch", "txv_verify_bytes", "txv_add_votes", "txv_query_tx", "txv_num_tx_sets",
    "txv_total_power", "txv_signbytes", "txv_txvote_size", "txv_keygen", "txv_sign_votes", "txv_stage",
    "txv_run_staged", "txv_fetch_staged", "txv_commit_bitmap", "txv_reset_tally", "txv_reset_flow", "txv_sync", "txv_fe_selftest",
    "txv_copy_commit_bitmap", "txv_valu_probe", "txv_table_window", "txv_validator_tables_built", "txv_staged_bytes", "txv_base_window", "txv_sig_keys",
    "txv_submit_votes", "txv_submit_checked", "txv_wait_votes", "txv_bind_host_numa", "txv_get_votes", "txv_copy_set_sums",
    "txv_pool_new", "txv_pool_free", "txv_pool_check", "txv_pool_check_keys", "txv_pool_update", "txv_pool_update_keys", "txv_pool_reap", "txv_pool_flush",
    "txv_pool_size", "txv_pool_txs_bytes", "txv_pool_height", "txv_pool_cache_keys", "txv_pool_sync",
    "txv_pool_check_submit", "txv_pool_check_wait", "txv_pool_update_submit",
    "txv_decode_msgs", "txv_decode_stage", "txv_decode_run", "txv_decode_fetch", "txv_pool_receive", "txv_encode_msgs",
    "txv_query_txs", "txv_make_commit", "txv_save_tx_bytes", "txv_host_register", "txv_host_unregister",
    "txv_shard_of", "txv_commit_state_bytes", "txv_pack_commit_state", "txv_read_commit_state", "txv_commit_state_pack_host",
    "txv_commit_state_unpack", "txv_set_commit_sink", "txv_slot_kernel_ms", "txv_slot_verify_ms", "txv_flow_stream",
    "txv_ingest_msgs", "txv_ingest_submit", "txv_ingest_wait", "txv_pool_prepare",
    "txv_ingest_decode", "txv_ingest_admit", "txv_route_bytes", "txv_route_admitted", "txv_route_checked", "txv_route_pack_host",
    "txv_route_view", "txv_submit_routed", "txv_ingest_admit_submit", "txv_ingest_admit_finish"]


# ------------------------------------------------------------------ host-only helpers
def sign_bytes(height: int, txhash: bytes, ts_sec: int, ts_nanos: int, chain_id: str) -> bytes:
    """TxVote.SignBytes(chainID) — types/tx_vote.go:83-89 (amino restatement, host C++)."""
    out = ctypes.create_string_buffer(2048)
    cid = chain_id.encode() if isinstance(chain_id, str) else chain_id
    n = lib().txv_signbytes(height, txhash, len(txhash), ts_sec, ts_nanos, cid, len(cid), out, 2048)
    if n < 0:
        raise ValueError("amino: timestamp out of range (reference panics)")
    return out.raw[:n]


def txvote_size(height: int, txhash_len: int, ts_sec: int, ts_nanos: int, addr_len: int, sig_len: int) -> int:
    """TxVote.Size() — types/tx_vote.go:144-150."""
    return lib().txv_txvote_size(height, txhash_len, ts_sec, ts_nanos, addr_len, sig_len)


# ------------------------------------------------------------------ vote batches
@dataclass
class TxVote:
    """types/tx_vote.go:48-55.  Timestamp as (Unix seconds, nanoseconds)."""
    Height: int = 0
    TxHash: str = ""
    TxKey: bytes = b"\0" * 32
    Timestamp: tuple = (0, 0)
    ValidatorAddress: bytes = b""
    Signature: Optional[bytes] = None

    def SignBytes(self, chain_id: str) -> bytes:
        return sign_bytes(self.Height, self.TxHash.encode(), self.Timestamp[0], self.Timestamp[1], chain_id)

    def Size(self) -> int:
        return txvote_size(self.Height, len(self.TxHash), self.Timestamp[0], self.Timestamp[1],
                           len(self.ValidatorAddress), len(self.Signature or b""))


class VoteBatch:
    """Structure-of-arrays TxVote batch matching txv_votes (include/txvote.h)."""

    def __init__(self, n: int, *, height, txhash_arena, txhash_off, txhash_len, ts_sec, ts_nanos,
                 addr, addr_len, sig, sig_len, is_nil=None, txkey=None):
        self.n = int(n)
        c = np.ascontiguousarray
        self.height = c(height, dtype=np.int64)
        self.txhash_arena = c(np.frombuffer(txhash_arena, np.uint8) if isinstance(txhash_arena, (bytes, bytearray))
                              else txhash_arena, dtype=np.uint8)
        if self.txhash_arena.size == 0:
            self.txhash_arena = np.zeros(1, np.uint8)
        self.txhash_off = c(txhash_off, dtype=np.uint32)
        self.txhash_len = c(txhash_len, dtype=np.uint32)
        self.ts_sec = c(ts_sec, dtype=np.int64)
        self.ts_nanos = c(ts_nanos, dtype=np.int32)
        self.addr = c(addr, dtype=np.uint8).reshape(-1)
        self.addr_len = c(addr_len, dtype=np.uint32)
        self.sig = c(sig, dtype=np.uint8).reshape(-1)
        self.sig_len = c(sig_len, dtype=np.uint32)
        self.is_nil = None if is_nil is None else c(is_nil, dtype=np.uint8)
        self.txkey = None if txkey is None else c(txkey, dtype=np.uint8).reshape(-1)
        assert self.addr.size == 20 * self.n and self.sig.size == 64 * self.n
        assert self.txkey is None or self.txkey.size == 32 * self.n

    @classmethod
    def from_votes(cls, votes: Sequence[Optional[TxVote]]) -> "VoteBatch":
        n = len(votes)
        arena = bytearray()
        off = np.zeros(n, np.uint32); ln = np.zeros(n, np.uint32)
        h = np.zeros(n, np.int64); ts = np.zeros(n, np.int64); tn = np.zeros(n, np.int32)
        addr = np.zeros((n, 20), np.uint8); al = np.zeros(n, np.uint32)
        sig = np.zeros((n, 64), np.uint8); sl = np.zeros(n, np.uint32)
        nil = np.zeros(n, np.uint8)
        tk = np.zeros((n, 32), np.uint8)
        for i, v in enumerate(votes):
            if v is None:
                nil[i] = 1
                continue
            tk[i] = np.frombuffer(bytes(v.TxKey)[:32].ljust(32, b"\0"), np.uint8)
            th = v.TxHash.encode() if isinstance(v.TxHash, str) else v.TxHash
            off[i] = len(arena); ln[i] = len(th); arena += th
            h[i] = v.Height; ts[i], tn[i] = v.Timestamp
            a = v.ValidatorAddress or b""
            al[i] = len(a); addr[i, :min(20, len(a))] = np.frombuffer(a[:20], np.uint8)
            s = v.Signature or b""
            sl[i] = len(s); sig[i, :min(64, len(s))] = np.frombuffer(s[:64], np.uint8)
        return cls(n, height=h, txhash_arena=bytes(arena), txhash_off=off, txhash_len=ln, ts_sec=ts,
                   ts_nanos=tn, addr=addr, addr_len=al, sig=sig, sig_len=sl, is_nil=nil, txkey=tk)

    def c_struct(self) -> _Votes:
        v = _Votes()
        v.n = self.n
        v.is_nil = None if self.is_nil is None else self.is_nil.ctypes.data
        v.height = self.height.ctypes.data
        v.txhash = self.txhash_arena.ctypes.data
        v.txhash_off = self.txhash_off.ctypes.data
        v.txhash_len = self.txhash_len.ctypes.data
        v.ts_sec = self.ts_sec.ctypes.data
        v.ts_nanos = self.ts_nanos.ctypes.data
        v.addr = self.addr.ctypes.data
        v.addr_len = self.addr_len.ctypes.data
        v.sig = self.sig.ctypes.data
        v.sig_len = self.sig_len.ctypes.data
        v.txkey = None if self.txkey is None else self.txkey.ctypes.data
        return v

    def txhash(self, i: int) -> bytes:
        o, l = int(self.txhash_off[i]), int(self.txhash_len[i])
        return self.txhash_arena[o:o + l].tobytes()


def route_flags(batch: VoteBatch) -> int:
    return (ROUTE_TXKEY if batch.txkey is not None else 0) | (ROUTE_NIL if batch.is_nil is not None else 0)


def route_stride(batch: VoteBatch) -> int:
    """bytes every rank's route buffer needs for this batch whatever the split
    (txv_route_bytes of all n votes and the whole TxHash arena extent)"""
    live = np.ones(batch.n, bool) if batch.is_nil is None else batch.is_nil == 0
    ext = int((batch.txhash_off[live].astype(np.int64) + batch.txhash_len[live]).max()) if live.any() else 0
    return int(lib().txv_route_bytes(batch.n, ext, route_flags(batch)))


def route_pack_host(batch: VoteBatch, pool_status=None, n_shards: int = 1):
    """txv_route_pack_host: the votes pool_status admits (TXV_POOL_OK; None = all), each rank's
    in arrival order, as [n_shards, stride] route buffers built on the host, and their metas"""
    stride = route_stride(batch)
    out = np.zeros((n_shards, stride), np.uint8)
    meta = np.zeros(n_shards, ROUTE_META_DTYPE)
    st = None if pool_status is None else np.ascontiguousarray(pool_status, np.uint8)
    vs = batch.c_struct()
    r = lib().txv_route_pack_host(ctypes.byref(vs), None if st is None else st.ctypes.data, n_shards, out.ctypes.data,
                                  stride, meta.ctypes.data)
    if r:
        raise ValueError(f"txv_route_pack_host: {r}")
    return out, meta


def route_view(buf) -> VoteBatch:
    """a route buffer (host bytes) as a VoteBatch (copies; txv_route_view)"""
    b = np.ascontiguousarray(buf, np.uint8)
    v = _Votes()
    r = lib().txv_route_view(b.ctypes.data, b.size, ctypes.byref(v))
    if r:
        raise ValueError(f"txv_route_view: {r}")
    n = v.n

    def col(ptr, dt, count):
        if not ptr or not count:
            return np.zeros(count, dt)
        return np.frombuffer((ctypes.c_uint8 * (count * np.dtype(dt).itemsize)).from_address(ptr), dt).copy()
    off = col(v.txhash_off, np.uint32, n)
    ln = col(v.txhash_len, np.uint32, n)
    ab = int((off.astype(np.int64) + ln).max()) if n else 0
    return VoteBatch(n, height=col(v.height, np.int64, n), txhash_arena=col(v.txhash, np.uint8, ab), txhash_off=off,
                     txhash_len=ln, ts_sec=col(v.ts_sec, np.int64, n), ts_nanos=col(v.ts_nanos, np.int32, n),
                     addr=col(v.addr, np.uint8, 20 * n), addr_len=col(v.addr_len, np.uint32, n),
                     sig=col(v.sig, np.uint8, 64 * n), sig_len=col(v.sig_len, np.uint32, n),
                     is_nil=col(v.is_nil, np.uint8, n) if v.is_nil else None,
                     txkey=col(v.txkey, np.uint8, 32 * n) if v.txkey else None)


# ------------------------------------------------------------------ received wire messages
WIRE_OK, WIRE_TOO_LARGE, WIRE_ERR_DECODE, WIRE_NIL = range(4)   # TXV_WIRE_*
POOL_NOT_CHECKED = 0xFF


class WireBatch:
    """n received TxVoteMessage wire messages (Reactor.Receive msgBytes) packed in one buffer."""

    def __init__(self, msgs: Sequence[bytes] = (), *, wire=None, off=None, length=None):
        if wire is None:
            lens = np.array([len(m) for m in msgs], np.uint32)
            off = np.zeros(len(msgs), np.uint64)
            if len(msgs) > 1:
                off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
            # a writable buffer (txv_host_register pins it for DMA)
            wire = np.frombuffer(bytearray(b"".join(msgs)), np.uint8) if msgs else np.zeros(0, np.uint8)
            length = lens
        self.wire = np.ascontiguousarray(wire, dtype=np.uint8)
        if self.wire.size == 0:
            self.wire = np.zeros(1, np.uint8)
            self.nbytes = 0
        else:
            self.nbytes = int(self.wire.size)
        self.off = np.ascontiguousarray(off, dtype=np.uint64)
        self.len = np.ascontiguousarray(length, dtype=np.uint32)
        self.n = int(self.off.size)

    def msg(self, i: int) -> bytes:
        o, l = int(self.off[i]), int(self.len[i])
        return self.wire[o:o + l].tobytes()


def encode_msgs(batch: "VoteBatch", txkey: Optional[np.ndarray] = None) -> WireBatch:
    """cdc.MustMarshalBinaryBare(&TxVoteMessage{tx}) for every vote of `batch` (txv_encode_msgs)."""
    vs = batch.c_struct()
    n = batch.n
    off = np.zeros(max(n, 1), np.uint64)
    ln = np.zeros(max(n, 1), np.uint32)
    total = ctypes.c_uint64()
    tk = None if txkey is None else np.ascontiguousarray(txkey, np.uint8).ctypes.data
    rc = lib().txv_encode_msgs(ctypes.byref(vs), tk, None, None, None, 0, off.ctypes.data, ln.ctypes.data,
                               ctypes.byref(total))
    if rc not in (0, -28):
        raise TxvInfraError(f"txv_encode_msgs failed ({rc})")
    wire = np.zeros(max(total.value, 1), np.uint8)
    rc = lib().txv_encode_msgs(ctypes.byref(vs), tk, None, None, wire.ctypes.data, total.value, off.ctypes.data,
                               ln.ctypes.data, ctypes.byref(total))
    if rc != 0:
        raise TxvInfraError(f"txv_encode_msgs failed ({rc})")
    return WireBatch(wire=wire[:total.value], off=off[:n], length=ln[:n])


class DecodedMsgs:
    """txv_wire_votes results: status, the votes as a VoteBatch over the wire buffer, TxKey, sig offsets"""

    def __init__(self, wb: WireBatch):
        n = max(wb.n, 1)
        self.status = np.zeros(n, np.uint8)
        self.height = np.zeros(n, np.int64)
        self.txhash_off = np.zeros(n, np.uint32)
        self.txhash_len = np.zeros(n, np.uint32)
        self.txkey = np.zeros((n, 32), np.uint8)
        self.ts_sec = np.zeros(n, np.int64)
        self.ts_nanos = np.zeros(n, np.int32)
        self.addr = np.zeros((n, 20), np.uint8)
        self.addr_len = np.zeros(n, np.uint32)
        self.sig = np.zeros((n, 64), np.uint8)
        self.sig_len = np.zeros(n, np.uint32)
        self.sig_off = np.zeros(n, np.uint64)
        self.n = wb.n
        self.wb = wb

    def c_struct(self) -> _WireVotes:
        w = _WireVotes()
        for f, _ in _WireVotes._fields_:
            setattr(w, f, getattr(self, f).ctypes.data)
        return w

    def batch(self) -> VoteBatch:
        """all n messages as a VoteBatch (fields zero where status != WIRE_OK); TxHash arena = the wire"""
        n = self.n
        return VoteBatch(n, height=self.height[:n], txhash_arena=self.wb.wire, txhash_off=self.txhash_off[:n],
                         txhash_len=self.txhash_len[:n], ts_sec=self.ts_sec[:n], ts_nanos=self.ts_nanos[:n],
                         addr=self.addr[:n], addr_len=self.addr_len[:n], sig=self.sig[:n], sig_len=self.sig_len[:n],
                         txkey=self.txkey[:n])

    def vote(self, i: int) -> Optional[TxVote]:
        if self.status[i] != WIRE_OK:
            return None
        w = self.wb.wire
        o, l = int(self.txhash_off[i]), int(self.txhash_len[i])
        so, sl = int(self.sig_off[i]), int(self.sig_len[i])
        al = int(self.addr_len[i])
        return TxVote(Height=int(self.height[i]), TxHash=w[o:o + l].tobytes().decode("latin-1"),
                      TxKey=self.txkey[i].tobytes(), Timestamp=(int(self.ts_sec[i]), int(self.ts_nanos[i])),
                      ValidatorAddress=self.addr[i, :min(al, 20)].tobytes() if al <= 20 else b"?" * al,
                      Signature=w[so:so + sl].tobytes() if sl else None)


# ------------------------------------------------------------------ context
class Context:
    """Owns a txv_ctx (one GPU).  Thin wrapper; every call raises on infrastructure errors."""

    def __init__(self, device: int = -1, max_batch: int = 1 << 20, max_txs: int = 1 << 20,
                 max_validators: int = 1024, max_accepted: int = 0, max_msg_bytes: int = 256,
                 table_w: int | None = None, table_budget_mb: int = 0, lane_votes: int = 0,
                 base_w: int = 0, key_arena_bytes: int = 0):
        """table_w: fixed-base window (4, 8, 10, 12, 14, 16, 18, 20, 21) or None = the largest
        whose per-validator tables fit ``table_budget_mb`` (0 = library default, 112 GiB); 21 (the
        12-position layout, 1.70 GB per validator, one table addition per vote fewer than 20) is
        only taken on request and runs against the radix-2^26 base table."""
        if table_w not in (None, 4, 8, 10, 12, 14, 16, 18, 20, 21):
            raise ValueError("table_w must be None or one of 4, 8, 10, 12, 14, 16, 18, 20, 21")
        if lane_votes not in (0, 1, 2, 4, 8):
            raise ValueError("lane_votes must be 0 (default), 1 (split K1b/K1c), 2, 4 or 8")
        cfg = _Cfg(device, max_batch, max_txs, max_validators, max_accepted, max_msg_bytes,
                   (((table_w or 0) & 0xFF) << 8) | ((lane_votes & 0xF) << 16) | ((base_w & 0xFF) << 20),
                   table_budget_mb, key_arena_bytes)
        h = ctypes.c_void_p()
        rc = lib().txv_init(ctypes.byref(cfg), ctypes.byref(h))
        if rc != 0:
            raise TxvInfraError(f"txv_init failed ({rc}): no usable HIP device")
        self._h = h
        self.n_vals = 0

    def close(self):
        if getattr(self, "_h", None):
            for pool in list(getattr(self, "_pools", ())):   # their queued appends use this context's workers
                pool.sync()
            lib().txv_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def _chk(self, rc: int, what: str):
        if rc < 0:
            raise TxvInfraError(f"{what} failed ({rc}): {lib().txv_last_error(self._h).decode()}")
        return rc

    def device_name(self) -> str:
        buf = ctypes.create_string_buffer(256)
        self._chk(lib().txv_device_name(self._h, buf, 256), "txv_device_name")
        return buf.value.decode()

    def set_validators(self, pubs: Sequence[bytes], powers: Sequence[int], chain_id: str):
        pubs_b = b"".join(pubs)
        pw = np.ascontiguousarray(np.asarray(powers, dtype=np.int64))
        cid = chain_id.encode()
        self._chk(lib().txv_set_validators(self._h, pubs_b, pw.ctypes.data if len(pw) else None, len(pubs),
                                           cid, len(cid)), "txv_set_validators")
        self.n_vals = len(pubs)

    def validator_info(self):
        n = self.n_vals
        addr = np.zeros((max(n, 1), 20), np.uint8)
        ok = np.zeros(max(n, 1), np.uint8)
        self._chk(lib().txv_get_validator_info(self._h, addr.ctypes.data, ok.ctypes.data, n), "info")
        return [addr[i].tobytes() for i in range(n)], ok[:n].astype(bool)

    def verify_batch(self, batch: VoteBatch, pubs: Optional[np.ndarray] = None) -> np.ndarray:
        out = np.zeros(max(batch.n, 1), np.uint8)
        vs = batch.c_struct()
        pp = None
        if pubs is not None:
            pubs = np.ascontiguousarray(pubs, dtype=np.uint8).reshape(-1)
            assert pubs.size == 32 * batch.n
            pp = pubs.ctypes.data
        self._chk(lib().txv_verify_batch(self._h, ctypes.byref(vs), pp, out.ctypes.data), "txv_verify_batch")
        return out[:batch.n]

    def verify_bytes(self, pubs: Sequence[bytes], msgs: Sequence[bytes], sigs: Sequence[bytes]) -> np.ndarray:
        """PubKeyEd25519.VerifyBytes(msg, sig) per (pub, msg, sig) triple (the call at
        types/tx_vote.go:115); signatures of any length (only len 64 can verify)."""
        n = len(pubs)
        assert len(msgs) == n and len(sigs) == n
        pk = np.frombuffer(b"".join(pubs), np.uint8) if n else np.zeros(32, np.uint8)
        assert pk.size == 32 * max(n, 1) or n == 0
        arena = np.frombuffer(b"".join(msgs) or b"\0", np.uint8)
        ln = np.array([len(m) for m in msgs] or [0], np.uint32)
        off = np.concatenate([[0], np.cumsum(ln[:-1], dtype=np.uint64)]).astype(np.uint32)
        sg = np.zeros((max(n, 1), 64), np.uint8)
        sl = np.zeros(max(n, 1), np.uint32)
        for i, s in enumerate(sigs):
            sl[i] = len(s)
            sg[i, :min(64, len(s))] = np.frombuffer(s[:64], np.uint8)
        out = np.zeros(max(n, 1), np.uint8)
        self._chk(lib().txv_verify_bytes(self._h, pk.ctypes.data, arena.ctypes.data, off.ctypes.data, ln.ctypes.data,
                                         sg.ctypes.data, sl.ctypes.data, n, out.ctypes.data), "txv_verify_bytes")
        return out[:n].astype(bool)

    def sig_keys(self, batch: VoteBatch, long_sigs: Optional[dict] = None) -> np.ndarray:
        """txVoteKey = SHA-256(Signature) per vote ([n, 32] u8), hashed on the GPU;
        long_sigs: {index: full signature bytes} for votes with sig_len > 64."""
        out = np.zeros((max(batch.n, 1), 32), np.uint8)
        full, off = _long_sig_arena(batch, long_sigs)
        vs = batch.c_struct()
        self._chk(lib().txv_sig_keys(self._h, ctypes.byref(vs), full, off, out.ctypes.data), "txv_sig_keys")
        return out[:batch.n]

    def add_votes(self, batch: VoteBatch, ev_cap: int = 0):
        out = np.zeros(max(batch.n, 1), np.uint8)
        ev_cap = ev_cap or max(batch.n, 1)
        evs = np.zeros(ev_cap, EVENT_DTYPE)
        nev = ctypes.c_uint32()
        vs = batch.c_struct()
        self._chk(lib().txv_add_votes(self._h, ctypes.byref(vs), out.ctypes.data, evs.ctypes.data, ev_cap,
                                      ctypes.byref(nev)), "txv_add_votes")
        return out[:batch.n], evs[:min(nev.value, ev_cap)]

    def route_admitted(self, batch: VoteBatch, pool_status, n_shards: int, dst_ptr: int, stride: int) -> np.ndarray:
        """txv_route_admitted: the admitted votes packed on this context's GPU into rank r's buffer at
        device address dst_ptr + r * stride (>= route_stride(batch)); returns the metas"""
        meta = np.zeros(n_shards, ROUTE_META_DTYPE)
        st = None if pool_status is None else np.ascontiguousarray(pool_status, np.uint8)
        vs = batch.c_struct()
        self._chk(lib().txv_route_admitted(self._h, ctypes.byref(vs), None if st is None else st.ctypes.data, n_shards,
                                           ctypes.c_void_p(dst_ptr), stride, meta.ctypes.data), "txv_route_admitted")
        return meta

    def route_checked(self, batch: VoteBatch, pool, pool_ticket: int, n_shards: int, dst_ptr: int, stride: int) -> np.ndarray:
        """txv_route_checked: route_admitted for the batch TxVotePool.check_submit(batch) returned
        pool_ticket for, its statuses and signatures read in HBM behind the pool's decisions"""
        meta = np.zeros(n_shards, ROUTE_META_DTYPE)
        vs = batch.c_struct()
        self._chk(lib().txv_route_checked(self._h, ctypes.byref(vs), pool._h, pool_ticket, n_shards,
                                          ctypes.c_void_p(dst_ptr), stride, meta.ctypes.data), "txv_route_checked")
        return meta

    def submit_routed(self, buf_ptr: int, meta) -> int:
        """txv_submit_routed: TryAddVote for a route buffer already in this context's HBM (at device
        address buf_ptr, e.g. what the node's RCCL scatter delivered); a ticket for wait_votes"""
        m = np.ascontiguousarray(np.asarray(meta, ROUTE_META_DTYPE).reshape(1))
        t = ctypes.c_uint64()
        self._chk(lib().txv_submit_routed(self._h, ctypes.c_void_p(buf_ptr), m.ctypes.data, ctypes.byref(t)),
                  "txv_submit_routed")
        self._inflight = getattr(self, "_inflight", {})
        self._inflight[t.value] = int(m[0]["n"])
        return t.value

    def submit_votes(self, batch: VoteBatch) -> int:
        """asynchronous TryAddVote batch (txv_submit_votes): returns a ticket for wait_votes"""
        t = ctypes.c_uint64()
        vs = batch.c_struct()
        self._chk(lib().txv_submit_votes(self._h, ctypes.byref(vs), ctypes.byref(t)), "txv_submit_votes")
        self._inflight = getattr(self, "_inflight", {})
        self._inflight[t.value] = batch.n
        return t.value

    def submit_checked(self, batch: VoteBatch, pool, pool_ticket: int) -> int:
        """txv_submit_checked: TryAddVote for the batch TxVotePool.check_submit(batch) returned
        pool_ticket for -- the votes the pool did not admit as nil entries, decided on the device
        behind the pool's decisions (no wait for its statuses); a ticket for wait_votes"""
        t = ctypes.c_uint64()
        vs = batch.c_struct()
        self._chk(lib().txv_submit_checked(self._h, ctypes.byref(vs), pool._h, pool_ticket, ctypes.byref(t)),
                  "txv_submit_checked")
        self._inflight = getattr(self, "_inflight", {})
        self._inflight[t.value] = batch.n
        return t.value

    def wait_votes(self, ticket: int, ev_cap: int = 0):
        n = getattr(self, "_inflight", {}).get(ticket, 0)   # kept until the library took the ticket
        out = np.zeros(max(n, 1), np.uint8)
        ev_cap = ev_cap or max(n, 1)
        evs = np.zeros(ev_cap, EVENT_DTYPE)
        nev = ctypes.c_uint32()
        self._chk(lib().txv_wait_votes(self._h, ticket, out.ctypes.data, evs.ctypes.data, ev_cap, ctypes.byref(nev)),
                  "txv_wait_votes")
        self._inflight.pop(ticket, None)
        return out[:n], evs[:min(nev.value, ev_cap)]

    def get_votes(self, txhash: bytes):
        """TxVoteSet.GetVotes: [(validator index, vote sequence number, signature bytes)] in
        validator order"""
        n = ctypes.c_uint32()
        self._chk(lib().txv_get_votes(self._h, txhash, len(txhash), None, None, None, 0, ctypes.byref(n)), "get_votes")
        k = n.value
        vals = np.zeros(max(k, 1), np.uint32); seqs = np.zeros(max(k, 1), np.uint64)
        sigs = np.zeros((max(k, 1), 64), np.uint8)
        self._chk(lib().txv_get_votes(self._h, txhash, len(txhash), vals.ctypes.data, seqs.ctypes.data,
                                      sigs.ctypes.data, k, ctypes.byref(n)), "get_votes")
        return [(int(vals[j]), int(seqs[j]), sigs[j].tobytes()) for j in range(k)]

    def query_tx(self, txhash: bytes):
        s = ctypes.c_int64(); m = ctypes.c_uint8()
        r = self._chk(lib().txv_query_tx(self._h, txhash, len(txhash), ctypes.byref(s), ctypes.byref(m)), "query")
        return (s.value, bool(m.value)) if r == 1 else None

    def query_txs(self, hashes: Sequence[bytes]):
        """batched readers: (exists [n] bool, sum [n] i64, maj23 [n] bool, TxKey [n, 32] u8)"""
        n = len(hashes)
        arena = np.frombuffer(b"".join(hashes) or b"\0", np.uint8)
        ln = np.array([len(h) for h in hashes] or [0], np.uint32)
        off = np.concatenate([[0], np.cumsum(ln[:-1], dtype=np.uint64)]).astype(np.uint32)
        ex = np.zeros(max(n, 1), np.uint8); sm = np.zeros(max(n, 1), np.int64); mj = np.zeros(max(n, 1), np.uint8)
        tk = np.zeros((max(n, 1), 32), np.uint8)
        self._chk(lib().txv_query_txs(self._h, arena.ctypes.data, off.ctypes.data, ln.ctypes.data, n, ex.ctypes.data,
                                      sm.ctypes.data, mj.ctypes.data, tk.ctypes.data), "txv_query_txs")
        return ex[:n].astype(bool), sm[:n], mj[:n].astype(bool), tk[:n]

    def make_commit(self, txhash: bytes) -> bytes:
        """TxVoteSet.MakeCommit amino bytes (CommitSigs in validator order)"""
        ln = ctypes.c_uint64()
        rc = lib().txv_make_commit(self._h, txhash, len(txhash), None, 0, ctypes.byref(ln))
        if rc not in (0, -28):
            self._chk(rc, "txv_make_commit")
        out = ctypes.create_string_buffer(max(ln.value, 1))
        self._chk(lib().txv_make_commit(self._h, txhash, len(txhash), out, ln.value, ctypes.byref(ln)), "txv_make_commit")
        return out.raw[:ln.value]

    def save_tx_bytes(self, txhash: bytes):
        """TxStore.SaveTx's two db.Set calls: (H-key, TxVoteSet bytes, C-key, Commit bytes)"""
        lens = np.zeros(4, np.uint64)
        rc = lib().txv_save_tx_bytes(self._h, txhash, len(txhash), None, 0, lens.ctypes.data)
        if rc not in (0, -28):
            self._chk(rc, "txv_save_tx_bytes")
        out = ctypes.create_string_buffer(max(int(lens.sum()), 1))
        self._chk(lib().txv_save_tx_bytes(self._h, txhash, len(txhash), out, int(lens.sum()), lens.ctypes.data),
                  "txv_save_tx_bytes")
        parts, at = [], 0
        for L in lens.tolist():
            parts.append(out.raw[at:at + int(L)])
            at += int(L)
        return tuple(parts)

    def host_register(self, arr: np.ndarray):
        """pin a host array so batch columns inside it are DMA'd without a staging copy"""
        self._chk(lib().txv_host_register(self._h, arr.ctypes.data, arr.nbytes), "txv_host_register")

    def host_unregister(self, arr: np.ndarray):
        self._chk(lib().txv_host_unregister(self._h, arr.ctypes.data), "txv_host_unregister")

    def pack_commit_state(self, dst_dev_ptr: int, n_sets_cap: int):
        self._chk(lib().txv_pack_commit_state(self._h, ctypes.c_void_p(dst_dev_ptr), n_sets_cap), "pack state")

    def set_commit_sink(self, slot: int, dst_dev_ptr: int | None, n_sets_cap: int = 0):
        """txv_set_commit_sink: the packed commit state written into dst_dev_ptr (device memory)
        at the end of every batch run in `slot` (staged slot / submit-ticket slot); None removes it"""
        self._chk(lib().txv_set_commit_sink(self._h, slot, ctypes.c_void_p(dst_dev_ptr or 0), n_sets_cap if dst_dev_ptr else 0),
                  "commit sink")

    def slot_kernel_ms(self, slot: int):
        """(prep + SignBytes, verify, tally after verify, total) device ms of the slot's last run"""
        ms = (ctypes.c_float * 4)()
        self._chk(lib().txv_slot_kernel_ms(self._h, slot, ms), "txv_slot_kernel_ms")
        return (ms[0], ms[1], ms[2], ms[3])

    def slot_verify_ms(self, slot: int):
        """(K1a, K1b) device ms of the slot's last run (the verify time split in two)"""
        ms = (ctypes.c_float * 2)()
        self._chk(lib().txv_slot_verify_ms(self._h, slot, ms), "txv_slot_verify_ms")
        return (ms[0], ms[1])

    def read_commit_state(self, n_sets_cap: int) -> np.ndarray:
        """the device-packed commit state (txv_read_commit_state) as host bytes"""
        out = np.zeros(commit_state_bytes(n_sets_cap), np.uint8)
        self._chk(lib().txv_read_commit_state(self._h, out.ctypes.data, n_sets_cap), "read state")
        return out

    def num_tx_sets(self) -> int:
        return lib().txv_num_tx_sets(self._h)

    def total_power(self) -> int:
        return lib().txv_total_power(self._h)

    def keygen(self, seeds: Sequence[bytes]) -> List[bytes]:
        sb = b"".join(seeds)
        out = ctypes.create_string_buffer(32 * max(len(seeds), 1))
        self._chk(lib().txv_keygen(self._h, sb, len(seeds), out), "txv_keygen")
        return [out.raw[32 * i:32 * i + 32] for i in range(len(seeds))]

    def sign_votes(self, batch: VoteBatch, signer: np.ndarray, chain_id: str) -> np.ndarray:
        signer = np.ascontiguousarray(signer, dtype=np.uint32)
        out = np.zeros((max(batch.n, 1), 64), np.uint8)
        vs = batch.c_struct()
        cid = chain_id.encode()
        self._chk(lib().txv_sign_votes(self._h, ctypes.byref(vs), signer.ctypes.data, cid, len(cid), out.ctypes.data),
                  "txv_sign_votes")
        return out[:batch.n]

    def stage(self, slot: int, batch: VoteBatch):
        vs = batch.c_struct()
        self._chk(lib().txv_stage(self._h, slot, ctypes.byref(vs)), "txv_stage")

    def run_staged(self, slot: int, timed: bool = False):
        """timed: (route, verify, tally, total) device ms of this run"""
        ms = (ctypes.c_float * 4)()
        self._chk(lib().txv_run_staged(self._h, slot, ms if timed else None), "txv_run_staged")
        return (ms[0], ms[1], ms[2], ms[3]) if timed else None

    def fetch_staged(self, slot: int, n: int, ev_cap: int = 0, out: np.ndarray | None = None,
                     evs: np.ndarray | None = None):
        """statuses and commit events of a staged run; `out` / `evs` may be caller-owned buffers
        (reused across calls: no fresh pages to fault in on the hot path)"""
        if out is None or out.size < max(n, 1) or out.dtype != np.uint8 or not out.flags.c_contiguous:
            out = np.zeros(max(n, 1), np.uint8)
        ev_cap = ev_cap or max(n, 1)
        if evs is None or evs.size < ev_cap or evs.dtype != EVENT_DTYPE:
            evs = np.zeros(ev_cap, EVENT_DTYPE)
        nev = ctypes.c_uint32()
        self._chk(lib().txv_fetch_staged(self._h, slot, out.ctypes.data, evs.ctypes.data, ev_cap, ctypes.byref(nev)),
                  "fetch")
        return out[:n], evs[:min(nev.value, ev_cap)]

    def commit_bitmap(self):
        p = ctypes.c_void_p(); nb = ctypes.c_uint64()
        self._chk(lib().txv_commit_bitmap(self._h, ctypes.byref(p), ctypes.byref(nb)), "bitmap")
        return p.value, nb.value

    def copy_commit_bitmap(self, dst_dev_ptr: int, nbytes: int):
        self._chk(lib().txv_copy_commit_bitmap(self._h, ctypes.c_void_p(dst_dev_ptr), nbytes), "bitmap copy")

    def copy_set_sums(self, dst_dev_ptr: int, n_sets: int):
        self._chk(lib().txv_copy_set_sums(self._h, ctypes.c_void_p(dst_dev_ptr), n_sets), "set sums copy")

    def valu_probe(self):
        """(v_add_u32, v_mad_u64_u32) lane-ops/s measured on this device"""
        a = ctypes.c_double(); m = ctypes.c_double()
        self._chk(lib().txv_valu_probe(self._h, ctypes.byref(a), ctypes.byref(m)), "valu probe")
        return a.value, m.value

    @property
    def base_w(self) -> int:
        """window of the base-point table used by the verify kernel"""
        return int(lib().txv_base_window(self._h))

    @property
    def table_w(self) -> int:
        """fixed-base window of the validator tables in use (0 before set_validators)"""
        return int(lib().txv_table_window(self._h))

    def staged_bytes(self) -> int:
        """host bytes the last staged batch sent over PCIe (uniform columns and a TxKey column
        its TxHashes spell are produced on the device instead)"""
        return int(lib().txv_staged_bytes(self._h))

    @property
    def tables_built(self) -> int:
        """keys whose fixed-base tables the last set_validators built (the rest were kept)"""
        return int(lib().txv_validator_tables_built(self._h))

    def reset_tally(self):
        self._chk(lib().txv_reset_tally(self._h), "txv_reset_tally")

    def bind_host_numa(self) -> bool:
        """pin this thread and the library's pack threads to the GPU-local NUMA node (True on success;
        TXV_NUMA_BIND=0 leaves the affinity alone, experiment)"""
        if os.environ.get("TXV_NUMA_BIND") == "0":
            return False
        return lib().txv_bind_host_numa(self._h) == 0

    def reset_flow(self):
        """forget every TxVoteSet (a fresh TxFlow, txflow/service.go:71); validators stay"""
        self._chk(lib().txv_reset_flow(self._h), "txv_reset_flow")

    def flow_stream(self) -> int:
        """hipStream_t of the context's flow stream (txv_flow_stream), for torch.cuda.ExternalStream"""
        return lib().txv_flow_stream(self._h)

    def sync(self):
        self._chk(lib().txv_sync(self._h), "txv_sync")

    def decode_msgs(self, wb: WireBatch, max_msg_bytes: int = 1 << 20) -> DecodedMsgs:
        """Reactor.decodeMsg for a batch of received messages, on the GPU (txv_decode_msgs)."""
        d = DecodedMsgs(wb)
        ws = d.c_struct()
        self._chk(lib().txv_decode_msgs(self._h, wb.wire.ctypes.data, wb.nbytes, wb.off.ctypes.data,
                                        wb.len.ctypes.data, wb.n, max_msg_bytes, ctypes.byref(ws)), "txv_decode_msgs")
        return d

    def decode_stage(self, wb: WireBatch):
        self._chk(lib().txv_decode_stage(self._h, wb.wire.ctypes.data, wb.nbytes, wb.off.ctypes.data,
                                         wb.len.ctypes.data, wb.n), "txv_decode_stage")

    def decode_run(self, max_msg_bytes: int = 1 << 20, reps: int = 1) -> float:
        ms = ctypes.c_float()
        self._chk(lib().txv_decode_run(self._h, max_msg_bytes, reps, ctypes.byref(ms)), "txv_decode_run")
        return ms.value

    def decode_fetch(self, wb: WireBatch) -> DecodedMsgs:
        d = DecodedMsgs(wb)
        ws = d.c_struct()
        self._chk(lib().txv_decode_fetch(self._h, ctypes.byref(ws)), "txv_decode_fetch")
        return d

    def fe_selftest(self, a: np.ndarray, b: np.ndarray, op: int) -> np.ndarray:
        a = np.ascontiguousarray(a, dtype=np.uint32); b = np.ascontiguousarray(b, dtype=np.uint32)
        n = a.shape[0]
        out = np.zeros((n, 8), np.uint32)
        self._chk(lib().txv_fe_selftest(self._h, a.ctypes.data, b.ctypes.data, out.ctypes.data, n, op), "selftest")
        return out


def shard_of(hashes: Sequence[bytes], n_shards: int) -> np.ndarray:
    """SHA-256(TxHash)[0] mod n_shards per TxHash (txv_shard_of)"""
    n = len(hashes)
    arena = np.frombuffer(b"".join(hashes) or b"\0", np.uint8)
    ln = np.array([len(h) for h in hashes] or [0], np.uint32)
    off = np.concatenate([[0], np.cumsum(ln[:-1], dtype=np.uint64)]).astype(np.uint32)
    out = np.zeros(max(n, 1), np.uint32)
    rc = lib().txv_shard_of(arena.ctypes.data, off.ctypes.data, ln.ctypes.data, n, n_shards, out.ctypes.data)
    if rc:
        raise TxvInfraError(f"txv_shard_of failed ({rc})")
    return out[:n]


def commit_state_bytes(n_sets_cap: int) -> int:
    return int(lib().txv_commit_state_bytes(n_sets_cap))


def tx_digest(txhash: bytes) -> bytes:
    """a TxVoteSet's name in the multi-GPU exchange: SHA-256(TxHash bytes)[0:16] (byte 0 mod G is
    its shard, txv_shard_of)"""
    return hashlib.sha256(bytes(txhash)).digest()[:16]


def commit_state_pack_host(committed: np.ndarray, sums: np.ndarray, n_sets_cap: int, digests=None) -> np.ndarray:
    """the packed per-shard commit state (txv_pack_commit_state's layout) from host arrays;
    digests: [n_sets, 16] u8 (tx_digest of each set's TxHash) or None (zeros)"""
    committed = np.ascontiguousarray(committed, np.uint8)
    sums = np.ascontiguousarray(sums, np.int64)
    dg = None if digests is None else np.ascontiguousarray(digests, np.uint8).reshape(-1, 16)
    assert dg is None or len(dg) == len(sums)
    out = np.zeros(commit_state_bytes(n_sets_cap), np.uint8)
    rc = lib().txv_commit_state_pack_host(len(sums), committed.ctypes.data if len(sums) else None,
                                          sums.ctypes.data if len(sums) else None,
                                          dg.ctypes.data if dg is not None and len(dg) else None, n_sets_cap,
                                          out.ctypes.data)
    if rc:
        raise TxvInfraError(f"txv_commit_state_pack_host failed ({rc})")
    return out


def commit_state_unpack(buf: np.ndarray, n_sets_cap: int):
    """(committed [n_sets] bool, sums [n_sets] i64, digests [n_sets, 16] u8) of one packed shard state"""
    buf = np.ascontiguousarray(buf, np.uint8)
    ns = ctypes.c_uint32()
    committed = np.zeros(max(n_sets_cap, 1), np.uint8)
    sums = np.zeros(max(n_sets_cap, 1), np.int64)
    digests = np.zeros((max(n_sets_cap, 1), 16), np.uint8)
    rc = lib().txv_commit_state_unpack(buf.ctypes.data, n_sets_cap, ctypes.byref(ns), committed.ctypes.data,
                                       sums.ctypes.data, digests.ctypes.data, n_sets_cap)
    if rc:
        raise TxvInfraError(f"txv_commit_state_unpack failed ({rc})")
    return committed[:ns.value].astype(bool), sums[:ns.value], digests[:ns.value]


def _long_sig_arena(batch: VoteBatch, long_sigs: Optional[dict]):
    """(arena ptr, offsets ptr) for txv_* calls taking sig_full / sig_full_off, or (None, None)"""
    if not long_sigs:
        return None, None
    arena = bytearray()
    off = np.zeros(max(batch.n, 1), np.uint64)
    for i, s in long_sigs.items():
        assert len(s) == int(batch.sig_len[i]), "long_sigs entry does not match sig_len"
        off[i] = len(arena)
        arena += s
    a = np.frombuffer(bytes(arena) or b"\0", np.uint8)
    _long_sig_arena.keep = (a, off)     # alive for the duration of the call
    return a.ctypes.data, off.ctypes.data


POOL_OK, POOL_ERR_FULL, POOL_ERR_TOO_LARGE, POOL_ERR_IN_CACHE, POOL_ERR_ENCODING = range(5)
FLOW_NOT_ADDED = 0xFE   # TXV_FLOW_NOT_ADDED: a message the pool did not admit (txv_ingest_msgs)
FLOW_NOT_RUN = 0xFD     # TXV_FLOW_NOT_RUN: admitted by the pool, but the TxFlow stage failed (error returned)


class IngestError(TxvInfraError):
    """txv_ingest_wait / txv_ingest_msgs failed after the pool stage: `result` holds the
    (wire status, pool status, flow status, events) the call reported -- the pool-admitted votes
    carry FLOW_NOT_RUN (they are in the pool, not in TxFlow) -- and `rc` the return code."""

    def __init__(self, msg, rc, result):
        super().__init__(msg)
        self.rc = rc
        self.result = result


class IngestTicket:
    """one txv_ingest_submit batch in flight: wire / pool statuses are final at submit"""

    def __init__(self, ticket: int, n: int, ws: np.ndarray, ps: np.ndarray):
        self.ticket, self.n, self.wire_status, self.pool_status = ticket, n, ws, ps
POOL_NO_CACHE = 0xFFFFFFFF
POOL_WAL = 0x1      # TXV_POOL_WAL
SUBMIT_RING = 4         # txv_submit_votes batches in flight (staged slots 0 .. 3)
POOL_DEVICE_CACHE = 0x2   # TXV_POOL_DEVICE_CACHE: the LRU cache in HBM, CheckTx decisions on the GPU


class TxVotePool:
    """TxVotePool (txvotepool/txvotepool.go) over libtxvote.so: CheckTx (:180-261) per vote in
    arrival order with the txVoteKey = SHA-256(Signature) keys computed on the GPU of `ctx`,
    Update (:329-359), ReapMaxTxs (:310-324), Flush (:146-159), Size (:136), TxsBytes (:141).
    cache_size POOL_NO_CACHE selects nopTxCache; 0 fields take tendermint's defaults.
    device_cache: TXV_POOL_DEVICE_CACHE (include/txvote.h) -- the cache lives in the HBM of
    ctx's GPU and each batch's CheckTx decisions are made there."""

    def __init__(self, ctx: Optional[Context], size: int = 0, cache_size: int = 0, max_txs_bytes: int = 0,
                 max_msg_bytes: int = 0, height: int = 0, wal: bool = False, device_cache: bool = False):
        self.ctx = ctx
        if ctx is not None:
            if not hasattr(ctx, "_pools"):
                ctx._pools = weakref.WeakSet()
            ctx._pools.add(self)
        cfg = _PoolCfg(size, cache_size, max_txs_bytes, max_msg_bytes,
                       (POOL_WAL if wal else 0) | (POOL_DEVICE_CACHE if device_cache else 0))
        h = ctypes.c_void_p()
        rc = lib().txv_pool_new(ctypes.byref(cfg), height, ctypes.byref(h))
        if rc != 0:
            raise TxvInfraError(f"txv_pool_new failed ({rc})")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().txv_pool_free(self._h)
            self._h = None

    def sync(self):
        """txv_pool_sync: the queued appends of device batches done"""
        if getattr(self, "_h", None):
            lib().txv_pool_sync(self._h)

    def __del__(self):
        self.close()

    def check_batch(self, batch: VoteBatch, long_sigs: Optional[dict] = None) -> np.ndarray:
        out = np.zeros(max(batch.n, 1), np.uint8)
        full, off = _long_sig_arena(batch, long_sigs)
        vs = batch.c_struct()
        ctx = self._ctx_or_raise("check_batch")
        ctx._chk(lib().txv_pool_check(self._h, ctx._h, ctypes.byref(vs), full, off, out.ctypes.data), "txv_pool_check")
        return out[:batch.n]

    def check_submit(self, batch: VoteBatch, long_sigs: Optional[dict] = None) -> int:
        """txv_pool_check_submit: the batch is CheckTx'd in submission order; with the device cache
        its decisions are enqueued on the GPU and the call returns (check_wait(ticket) gives the
        statuses).  The batch's columns are kept referenced until the wait."""
        ctx = self._ctx_or_raise("check_submit")
        full, off = _long_sig_arena(batch, long_sigs)
        vs = batch.c_struct()
        t = ctypes.c_uint64(0)
        ctx._chk(lib().txv_pool_check_submit(self._h, ctx._h, ctypes.byref(vs), full, off, ctypes.byref(t)),
                 "txv_pool_check_submit")
        if not hasattr(self, "_inflight"):
            self._inflight = {}
        self._inflight[t.value] = (batch, vs, full, off)
        return t.value

    def check_wait(self, ticket: int) -> np.ndarray:
        """txv_pool_check_wait: the statuses of a submitted batch"""
        batch = self._inflight[ticket][0]
        out = np.zeros(max(batch.n, 1), np.uint8)
        rc = lib().txv_pool_check_wait(self._h, ticket, out.ctypes.data)
        del self._inflight[ticket]
        if rc != 0:
            raise TxvInfraError(f"txv_pool_check_wait failed ({rc})")
        return out[:batch.n]

    def prepare(self, batch: VoteBatch, long_sigs: Optional[dict] = None):
        """txv_pool_prepare: (keys [n, 32] u8, TxVote.Size() [n] u32) of a batch -- the
        order-independent half of check_batch; check_keys(keys, sizes) is the other half"""
        ctx = self._ctx_or_raise("prepare")
        n = batch.n
        keys = np.zeros((max(n, 1), 32), np.uint8)
        sizes = np.zeros(max(n, 1), np.uint32)
        full, off = _long_sig_arena(batch, long_sigs)
        vs = batch.c_struct()
        ctx._chk(lib().txv_pool_prepare(self._h, ctx._h, ctypes.byref(vs), full, off, keys.ctypes.data,
                                        sizes.ctypes.data), "txv_pool_prepare")
        return keys[:n], sizes[:n]

    def check_keys(self, keys: np.ndarray, sizes: np.ndarray) -> np.ndarray:
        """CheckTxWithInfo over (txVoteKey [n, 32] u8, TxVote.Size() [n] u32) pairs in arrival order
        (txv_pool_check_keys); needs no GPU when the pool was made with ctx=None"""
        keys = np.ascontiguousarray(keys, np.uint8)
        sizes = np.ascontiguousarray(sizes, np.uint32)
        n = len(sizes)
        out = np.zeros(max(n, 1), np.uint8)
        rc = lib().txv_pool_check_keys(self._h, self.ctx._h if self.ctx is not None else None, keys.ctypes.data,
                                       sizes.ctypes.data, n, out.ctypes.data)
        if rc != 0:
            raise TxvInfraError(f"txv_pool_check_keys failed ({rc})")
        return out[:n]

    def receive(self, wb: WireBatch):
        """Reactor.Receive (txvotepool/reactor.go:170-190) for a batch of messages in arrival order:
        (wire status TXV_WIRE_*, pool status TXV_POOL_* or POOL_NOT_CHECKED) per message."""
        ws = np.zeros(max(wb.n, 1), np.uint8)
        ps = np.zeros(max(wb.n, 1), np.uint8)
        ctx = self._ctx_or_raise("receive")
        ctx._chk(lib().txv_pool_receive(self._h, ctx._h, wb.wire.ctypes.data, wb.nbytes, wb.off.ctypes.data,
                                        wb.len.ctypes.data, wb.n, ws.ctypes.data, ps.ctypes.data), "txv_pool_receive")
        return ws[:wb.n], ps[:wb.n]

    def _ctx_or_raise(self, what: str):
        if self.ctx is None:
            raise ValueError(f"TxVotePool.{what} needs a Context (this pool was made with ctx=None: only "
                             "check_keys runs without one)")
        return self.ctx

    def ingest(self, wb: WireBatch, ev_cap: int = 0):
        """txv_ingest_msgs: Reactor.Receive -> CheckTxWithInfo -> TxFlow.TryAddVote for a batch of
        received messages with the decoded votes kept on the device.  Returns (wire status, pool
        status, flow status (FLOW_NOT_ADDED unless admitted), commit events by message index).
        After the pool stage a failure raises IngestError carrying those arrays (FLOW_NOT_RUN for
        the admitted votes)."""
        ctx = self._ctx_or_raise("ingest")
        n = wb.n
        ws = np.zeros(max(n, 1), np.uint8)
        ps = np.zeros(max(n, 1), np.uint8)
        fs = np.zeros(max(n, 1), np.uint8)
        ev_cap = ev_cap or max(n, 1)
        evs = np.zeros(ev_cap, EVENT_DTYPE)
        nev = ctypes.c_uint32()
        rc = lib().txv_ingest_msgs(ctx._h, self._h, wb.wire.ctypes.data, wb.nbytes, wb.off.ctypes.data,
                                   wb.len.ctypes.data, n, ws.ctypes.data, ps.ctypes.data, fs.ctypes.data,
                                   evs.ctypes.data, ev_cap, ctypes.byref(nev))
        res = (ws[:n], ps[:n], fs[:n], evs[:min(nev.value, ev_cap)])
        if rc < 0:
            msg = f"txv_ingest_msgs failed ({rc}): {lib().txv_last_error(ctx._h).decode()}"
            if (fs[:n] == FLOW_NOT_RUN).any():
                raise IngestError(msg, rc, res)
            raise TxvInfraError(msg)
        return res

    def ingest_submit(self, wb: WireBatch) -> IngestTicket:
        """txv_ingest_submit: decode + CheckTxWithInfo now, the admitted votes' TxFlow chain
        enqueued (up to three batches in flight; ingest_wait in submission order)"""
        ctx = self._ctx_or_raise("ingest_submit")
        n = wb.n
        ws = np.zeros(max(n, 1), np.uint8)
        ps = np.zeros(max(n, 1), np.uint8)
        t = ctypes.c_uint64()
        ctx._chk(lib().txv_ingest_submit(ctx._h, self._h, wb.wire.ctypes.data, wb.nbytes, wb.off.ctypes.data,
                                         wb.len.ctypes.data, n, ws.ctypes.data, ps.ctypes.data, ctypes.byref(t)),
                 "txv_ingest_submit")
        return IngestTicket(t.value, n, ws[:n], ps[:n])

    def ingest_decode(self, wb: WireBatch) -> IngestTicket:
        """txv_ingest_decode: upload + decode + keys enqueued (returns at once); ingest_admit next"""
        ctx = self._ctx_or_raise("ingest_decode")
        t = ctypes.c_uint64()
        ctx._chk(lib().txv_ingest_decode(ctx._h, self._h, wb.wire.ctypes.data, wb.nbytes, wb.off.ctypes.data,
                                         wb.len.ctypes.data, wb.n, ctypes.byref(t)), "txv_ingest_decode")
        n = wb.n
        return IngestTicket(t.value, n, np.zeros(n, np.uint8), np.zeros(n, np.uint8))

    def ingest_admit(self, tk: IngestTicket) -> IngestTicket:
        """txv_ingest_admit: CheckTxWithInfo of a decoded batch + its TxFlow chain enqueued; fills
        the ticket's wire / pool statuses"""
        ctx = self._ctx_or_raise("ingest_admit")
        ws = np.zeros(max(tk.n, 1), np.uint8)
        ps = np.zeros(max(tk.n, 1), np.uint8)
        ctx._chk(lib().txv_ingest_admit(ctx._h, tk.ticket, ws.ctypes.data, ps.ctypes.data), "txv_ingest_admit")
        tk.wire_status, tk.pool_status = ws[:tk.n], ps[:tk.n]
        return tk

    def ingest_admit_submit(self, tk: IngestTicket) -> IngestTicket:
        """txv_ingest_admit_submit: the batch's CheckTx handed to the device (returns at once), or
        the whole admission on the host path; ingest_admit_finish next"""
        ctx = self._ctx_or_raise("ingest_admit_submit")
        tk.wire_status = np.zeros(max(tk.n, 1), np.uint8)
        tk.pool_status = np.zeros(max(tk.n, 1), np.uint8)
        ctx._chk(lib().txv_ingest_admit_submit(ctx._h, tk.ticket, tk.wire_status.ctypes.data, tk.pool_status.ctypes.data),
                 "txv_ingest_admit_submit")
        return tk

    def ingest_admit_finish(self, tk: IngestTicket) -> IngestTicket:
        """txv_ingest_admit_finish: the submitted CheckTx's statuses in, the admitted votes' TxFlow
        chain enqueued; fills the ticket's wire / pool statuses"""
        ctx = self._ctx_or_raise("ingest_admit_finish")
        ws, ps = tk.wire_status, tk.pool_status
        ctx._chk(lib().txv_ingest_admit_finish(ctx._h, tk.ticket, ws.ctypes.data, ps.ctypes.data), "txv_ingest_admit_finish")
        tk.wire_status, tk.pool_status = ws[:tk.n], ps[:tk.n]
        return tk

    def ingest_wait(self, tk: IngestTicket, ev_cap: int = 0):
        """txv_ingest_wait: (wire status, pool status, flow status, commit events) of the batch"""
        ctx = self._ctx_or_raise("ingest_wait")
        n = tk.n
        fs = np.zeros(max(n, 1), np.uint8)
        ev_cap = ev_cap or max(n, 1)
        evs = np.zeros(ev_cap, EVENT_DTYPE)
        nev = ctypes.c_uint32()
        rc = lib().txv_ingest_wait(ctx._h, tk.ticket, fs.ctypes.data, evs.ctypes.data, ev_cap, ctypes.byref(nev))
        res = (tk.wire_status, tk.pool_status, fs[:n], evs[:min(nev.value, ev_cap)])
        if rc < 0:
            msg = f"txv_ingest_wait failed ({rc}): {lib().txv_last_error(ctx._h).decode()}"
            if (fs[:n] == FLOW_NOT_RUN).any():
                raise IngestError(msg, rc, res)
            raise TxvInfraError(msg)
        return res

    def update(self, height: int, batch: VoteBatch, long_sigs: Optional[dict] = None):
        full, off = _long_sig_arena(batch, long_sigs)
        vs = batch.c_struct()
        ctx = self._ctx_or_raise("update")
        ctx._chk(lib().txv_pool_update(self._h, ctx._h, height, ctypes.byref(vs), full, off), "txv_pool_update")

    def update_keys(self, height: int, keys: np.ndarray, sizes: np.ndarray):
        """Update over (txVoteKey [n, 32] u8, TxVote.Size() [n] u32) pairs (txv_pool_update_keys);
        needs no GPU when the pool was made with ctx=None"""
        keys = np.ascontiguousarray(keys, np.uint8)
        sizes = np.ascontiguousarray(sizes, np.uint32)
        rc = lib().txv_pool_update_keys(self._h, self.ctx._h if self.ctx is not None else None, height,
                                        keys.ctypes.data, sizes.ctypes.data, len(sizes))
        if rc != 0:
            raise TxvInfraError(f"txv_pool_update_keys failed ({rc})")

    def update_submit(self, height: int, batch: VoteBatch, long_sigs: Optional[dict] = None):
        """txv_pool_update_submit: Update enqueued behind the submitted CheckTx batches (device
        cache: no wait; applied once the batches before it are waited, or at sync())"""
        full, off = _long_sig_arena(batch, long_sigs)
        vs = batch.c_struct()
        ctx = self._ctx_or_raise("update_submit")
        ctx._chk(lib().txv_pool_update_submit(self._h, ctx._h, height, ctypes.byref(vs), full, off),
                 "txv_pool_update_submit")
        # registered columns are DMA'd by the engine after the call returns: keep them referenced
        # while the submission can still be unfinished (the engine has four flight slots)
        refs = self.__dict__.setdefault("_upd_refs", [])
        refs.append((batch, full, off, vs))
        del refs[:-5]

    def reap(self, max_txs: int = -1):
        """ReapMaxTxs: ([k, 32] keys, [k] sizes) in pool order"""
        n = ctypes.c_uint64()
        lib().txv_pool_reap(self._h, max_txs, None, None, 0, ctypes.byref(n))
        k = n.value
        keys = np.zeros((max(k, 1), 32), np.uint8)
        sizes = np.zeros(max(k, 1), np.uint32)
        lib().txv_pool_reap(self._h, max_txs, keys.ctypes.data, sizes.ctypes.data, k, ctypes.byref(n))
        return keys[:k], sizes[:k]

    def cache_keys(self) -> np.ndarray:
        n = ctypes.c_uint64()
        lib().txv_pool_cache_keys(self._h, None, 0, ctypes.byref(n))
        keys = np.zeros((max(n.value, 1), 32), np.uint8)
        lib().txv_pool_cache_keys(self._h, keys.ctypes.data, n.value, ctypes.byref(n))
        return keys[:n.value]

    def flush(self):
        lib().txv_pool_flush(self._h)

    def Size(self) -> int:
        return int(lib().txv_pool_size(self._h))

    def TxsBytes(self) -> int:
        return int(lib().txv_pool_txs_bytes(self._h))

    def Height(self) -> int:
        return int(lib().txv_pool_height(self._h))


# ------------------------------------------------------------------ reference-shaped API
class TxVoteSetView:
    """Readers of a TxVoteSet (types/vote_set.go:178-227) backed by the device tally."""

    def __init__(self, flow: "TxFlow", txhash: str):
        self._flow, self.TxHash = flow, txhash

    def _q(self):
        return self._flow.ctx.query_tx(self.TxHash.encode())

    def Stake(self) -> int:
        q = self._q()
        return -1 if q is None else q[0]

    def HasTwoThirdsMajority(self) -> bool:
        q = self._q()
        return bool(q and q[1])

    IsCommit = HasTwoThirdsMajority

    def HasTwoThirdsAny(self) -> bool:
        q = self._q()
        return bool(q) and q[0] > self._flow.ctx.total_power() * 2 // 3

    def TotalStake(self) -> int:
        return self._flow.ctx.total_power() * 2 // 3

    def HasAll(self) -> bool:
        q = self._q()
        return bool(q) and q[0] == self._flow.ctx.total_power()


class TxFlow:
    """txflow/service.go: TryAddVote/addVote over the GPU tally.  AddVotes is the batched
    form the single-goroutine checkMaj23Routine (service.go:123-166) becomes."""

    def __init__(self, ctx: Context, pubs: Sequence[bytes], powers: Sequence[int], chain_id: str):
        self.ctx = ctx
        self.chain_id = chain_id
        ctx.set_validators(pubs, powers, chain_id)
        self.commits: List[tuple] = []

    def AddVotes(self, votes: Sequence[Optional[TxVote]]):
        batch = VoteBatch.from_votes(votes)
        status, events = self.ctx.add_votes(batch)
        for e in events:
            self.commits.append((votes[int(e["vote_index"])].TxHash, int(e["sum"])))
        return status

    def TryAddVote(self, vote: TxVote):
        """(added, err) like service.go:169-188 (err carries the sentinel cause)."""
        st = int(self.AddVotes([vote])[0])
        code = st & 0x7F
        if code in (ADDED,):
            return True, None
        if code == DUPLICATE:
            return False, None
        return False, TxVoteError(code)

    def TxVoteSet(self, txhash: str) -> Optional[TxVoteSetView]:
        return TxVoteSetView(self, txhash) if self.ctx.query_tx(txhash.encode()) is not None else None


def verify(ctx: Context, vote: TxVote, chain_id_unused: str, pub: bytes):
    """TxVote.Verify(chainID, pubKey) (types/tx_vote.go:110-119) for one vote; the chain id of
    the context is used.  Returns None or a TxVoteError."""
    b = VoteBatch.from_votes([vote])
    st = int(ctx.verify_batch(b, np.frombuffer(pub, np.uint8).reshape(1, 32))[0])
    return None if st == ADDED else TxVoteError(st)

"""ctypes binding to the CPU oracle (oracle/build/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, always as the checker.  The product (go-txflow_amd/) never imports it.
See oracle.h for the reference file:line each function restates.
"""
import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")

ADDED, DUPLICATE, ERR_NIL, ERR_EMPTY_ADDR, ERR_UNKNOWN_VALIDATOR, ERR_NONDETERMINISTIC, \
    ERR_INVALID_SIGNATURE, ERR_INVALID_VALIDATOR_ADDRESS, ERR_SIGNBYTES = range(9)

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        c_u8p = ctypes.c_char_p
        L.orc_sha512.argtypes = [c_u8p, ctypes.c_size_t, ctypes.c_char_p]
        L.orc_sha256.argtypes = [c_u8p, ctypes.c_size_t, ctypes.c_char_p]
        L.orc_ed25519_verify.argtypes = [c_u8p, c_u8p, ctypes.c_size_t, c_u8p, ctypes.c_size_t]
        L.orc_ed25519_verify.restype = ctypes.c_int
        L.orc_ed25519_pubkey.argtypes = [c_u8p, ctypes.c_char_p]
        L.orc_ed25519_sign.argtypes = [c_u8p, c_u8p, ctypes.c_size_t, ctypes.c_char_p]
        L.orc_ed25519_decode_ok.argtypes = [c_u8p]
        L.orc_sc_reduce64.argtypes = [c_u8p, ctypes.c_char_p]
        L.orc_sc_minimal.argtypes = [c_u8p]
        L.orc_scalarmult.argtypes = [c_u8p, c_u8p, ctypes.c_char_p]
        L.orc_scalarmult_base.argtypes = [c_u8p, ctypes.c_char_p]
        L.orc_point_canonical.argtypes = [c_u8p, ctypes.c_char_p]
        L.orc_signbytes.argtypes = [ctypes.c_int64, c_u8p, ctypes.c_size_t, ctypes.c_int64, ctypes.c_int32,
                                    c_u8p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t]
        L.orc_txvote_size.argtypes = [ctypes.c_int64, ctypes.c_size_t, ctypes.c_int64, ctypes.c_int32,
                                      ctypes.c_size_t, ctypes.c_size_t]
        L.orc_flow_new.restype = ctypes.c_void_p
        L.orc_flow_new.argtypes = [c_u8p, ctypes.c_void_p, ctypes.c_uint32, c_u8p, ctypes.c_size_t]
        L.orc_flow_free.argtypes = [ctypes.c_void_p]
        L.orc_flow_add_votes.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.orc_flow_add_votes_soa.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_void_p]
        L.orc_txvote_verify_soa.argtypes = [ctypes.c_void_p, ctypes.c_void_p, c_u8p, ctypes.c_size_t, ctypes.c_int,
                                            ctypes.c_void_p]
        L.orc_pool_new.restype = ctypes.c_void_p
        L.orc_pool_new.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int64,
                                   ctypes.c_int]
        L.orc_pool_free.argtypes = [ctypes.c_void_p]
        L.orc_pool_check.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.orc_pool_check_keys.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
        L.orc_pool_check_soa.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p]
        L.orc_pool_update.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_uint32]
        L.orc_pool_update_keys.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_uint32]
        L.orc_pool_update_soa.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p]
        L.orc_pool_reap.restype = ctypes.c_uint64
        L.orc_pool_reap.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
        L.orc_pool_flush.argtypes = [ctypes.c_void_p]
        L.orc_pool_size.restype = ctypes.c_int64
        L.orc_pool_size.argtypes = [ctypes.c_void_p]
        L.orc_pool_txs_bytes.restype = ctypes.c_int64
        L.orc_pool_txs_bytes.argtypes = [ctypes.c_void_p]
        L.orc_pool_cache_keys.restype = ctypes.c_uint64
        L.orc_pool_cache_keys.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
        L.orc_flow_get_votes.restype = ctypes.c_uint32
        L.orc_flow_get_votes.argtypes = [ctypes.c_void_p, c_u8p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_uint32]
        L.orc_flow_query.argtypes = [ctypes.c_void_p, c_u8p, ctypes.c_uint32,
                                     ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int32)]
        L.orc_flow_num_sets.argtypes = [ctypes.c_void_p]
        L.orc_flow_num_sets.restype = ctypes.c_uint32
        L.orc_flow_num_verifies.argtypes = [ctypes.c_void_p]
        L.orc_flow_num_verifies.restype = ctypes.c_uint64
        L.orc_verify_many.restype = ctypes.c_double
        L.orc_verify_many.argtypes = [ctypes.c_void_p] * 6 + [ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p]
        L.orc_wire_decode.argtypes = [c_u8p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_void_p]
        L.orc_txvote_encode.argtypes = [ctypes.c_int64, c_u8p, ctypes.c_size_t, c_u8p, ctypes.c_int64, ctypes.c_int32,
                                         c_u8p, ctypes.c_size_t, c_u8p, ctypes.c_size_t, ctypes.c_char_p]
        L.orc_wire_encode.argtypes = [ctypes.c_int64, c_u8p, ctypes.c_size_t, c_u8p, ctypes.c_int64, ctypes.c_int32,
                                      c_u8p, ctypes.c_size_t, c_u8p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t]
        L.orc_wire_prefix.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        L.orc_wire_decode_many.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                                                  ctypes.c_void_p]
        L.orc_wire_decode_many.restype = ctypes.c_double
        _lib = L
    return _lib


def sha512(b: bytes) -> bytes:
    out = ctypes.create_string_buffer(64)
    lib().orc_sha512(b, len(b), out)
    return out.raw


def sha256(b: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().orc_sha256(b, len(b), out)
    return out.raw


def verify(pub: bytes, msg: bytes, sig: bytes) -> bool:
    assert len(pub) == 32
    return bool(lib().orc_ed25519_verify(pub, msg, len(msg), sig, len(sig)))


def pubkey(seed: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().orc_ed25519_pubkey(seed, out)
    return out.raw


def sign(seed: bytes, msg: bytes) -> bytes:
    out = ctypes.create_string_buffer(64)
    lib().orc_ed25519_sign(seed, msg, len(msg), out)
    return out.raw


def decode_ok(pub: bytes) -> bool:
    return bool(lib().orc_ed25519_decode_ok(pub))


def sc_reduce64(h: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().orc_sc_reduce64(h, out)
    return out.raw


def sc_minimal(s: bytes) -> bool:
    return bool(lib().orc_sc_minimal(s))


def scalarmult(k: bytes, p: bytes):
    out = ctypes.create_string_buffer(32)
    return out.raw if lib().orc_scalarmult(k, p, out) else None


def scalarmult_base(k: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().orc_scalarmult_base(k, out)
    return out.raw


def point_canonical(p: bytes):
    out = ctypes.create_string_buffer(32)
    return out.raw if lib().orc_point_canonical(p, out) else None


def signbytes(height: int, txhash: bytes, ts_sec: int, ts_nanos: int, chain_id: bytes):
    out = ctypes.create_string_buffer(2048)
    n = lib().orc_signbytes(height, txhash, len(txhash), ts_sec, ts_nanos, chain_id, len(chain_id), out, 2048)
    return None if n < 0 else out.raw[:n]


def txvote_size(height, txhash_len, ts_sec, ts_nanos, addr_len, sig_len) -> int:
    return lib().orc_txvote_size(height, txhash_len, ts_sec, ts_nanos, addr_len, sig_len)


class _Vote(ctypes.Structure):
    _fields_ = [("is_nil", ctypes.c_int32), ("height", ctypes.c_int64),
                ("txhash", ctypes.c_void_p), ("txhash_len", ctypes.c_uint32),
                ("ts_sec", ctypes.c_int64), ("ts_nanos", ctypes.c_int32),
                ("addr", ctypes.c_void_p), ("addr_len", ctypes.c_uint32),
                ("sig", ctypes.c_void_p), ("sig_len", ctypes.c_uint32)]


class _Soa(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint32)] + [(k, ctypes.c_void_p) for k in (
        "is_nil", "height", "txhash", "txhash_off", "txhash_len", "ts_sec", "ts_nanos", "addr", "addr_len",
        "sig", "sig_len")]


def _soa(b) -> _Soa:
    return _Soa(b.n, None if b.is_nil is None else b.is_nil.ctypes.data, b.height.ctypes.data,
                b.txhash_arena.ctypes.data, b.txhash_off.ctypes.data, b.txhash_len.ctypes.data,
                b.ts_sec.ctypes.data, b.ts_nanos.ctypes.data, b.addr.ctypes.data, b.addr_len.ctypes.data,
                b.sig.ctypes.data, b.sig_len.ctypes.data)


def txvote_verify_batch(b, pubs32, chain_id: bytes, threads: int = 1):
    """TxVote.Verify(chainID, pubs32[i]) for every vote of a VoteBatch-shaped object
    (types/tx_vote.go:110-119); returns the status codes (ADDED = nil error)."""
    import numpy as np
    pk = np.ascontiguousarray(np.asarray(pubs32, np.uint8).reshape(-1, 32))
    assert pk.shape[0] >= b.n
    out = np.zeros(max(b.n, 1), np.uint8)
    soa = _soa(b)
    lib().orc_txvote_verify_soa(ctypes.addressof(soa), pk.ctypes.data, chain_id, len(chain_id), threads,
                                out.ctypes.data)
    return out[:b.n]


class Flow:
    """Sequential TxFlow.addVote/TxVoteSet.AddVote restatement (txflow/service.go:192-234,
    types/vote_set.go:81-166).  votes: list of dicts with keys
    nil, height, txhash (bytes), ts_sec, ts_nanos, addr (bytes), sig (bytes)."""

    def __init__(self, pubs, powers, chain_id: bytes):
        import numpy as np
        self._np = np
        L = lib()
        pw = np.ascontiguousarray(np.asarray(powers, dtype=np.int64))
        self._h = L.orc_flow_new(b"".join(pubs), pw.ctypes.data, len(pubs), chain_id, len(chain_id))

    def __del__(self):
        if getattr(self, "_h", None):
            lib().orc_flow_free(self._h)
            self._h = None

    def add_votes(self, votes, verdicts=None):
        np = self._np
        n = len(votes)
        arr = (_Vote * max(n, 1))()
        keep = []
        for i, v in enumerate(votes):
            if v.get("nil"):
                arr[i].is_nil = 1
                continue
            bufs = [ctypes.create_string_buffer(bytes(v[k]) or b"\0", max(len(v[k]), 1))
                    for k in ("txhash", "addr", "sig")]
            keep.append(bufs)
            arr[i].is_nil = 0
            arr[i].height = v.get("height", 0)
            arr[i].txhash = ctypes.addressof(bufs[0]); arr[i].txhash_len = len(v["txhash"])
            arr[i].ts_sec = v.get("ts_sec", 0); arr[i].ts_nanos = v.get("ts_nanos", 0)
            arr[i].addr = ctypes.addressof(bufs[1]); arr[i].addr_len = len(v["addr"])
            arr[i].sig = ctypes.addressof(bufs[2]); arr[i].sig_len = len(v["sig"])
        status = np.zeros(max(n, 1), np.uint8)
        sums = np.zeros(max(n, 1), np.int64)
        fired = np.zeros(max(n, 1), np.uint8)
        vp = None
        if verdicts is not None:
            vd = np.ascontiguousarray(np.asarray(verdicts, dtype=np.uint8))
            vp = vd.ctypes.data
        import time
        t0 = time.perf_counter()
        lib().orc_flow_add_votes(self._h, ctypes.addressof(arr), n, vp, status.ctypes.data,
                                 sums.ctypes.data, fired.ctypes.data)
        self.last_seconds = time.perf_counter() - t0   # the C loop only (bench cpu_baseline)
        return status[:n], sums[:n], fired[:n]

    def add_batch(self, b, threads: int = 1):
        """orc_flow_add_votes_soa over a txflow_amd.VoteBatch-shaped object (the txv_votes SoA
        layout): Verify on `threads` threads, then the sequential loop.  Returns
        (status, sum_after, fired)."""
        np = self._np
        n = b.n
        soa = _soa(b)
        status = np.zeros(max(n, 1), np.uint8)
        sums = np.zeros(max(n, 1), np.int64)
        fired = np.zeros(max(n, 1), np.uint8)
        lib().orc_flow_add_votes_soa(self._h, ctypes.addressof(soa), threads, status.ctypes.data,
                                     sums.ctypes.data, fired.ctypes.data)
        return status[:n], sums[:n], fired[:n]

    def query(self, txhash: bytes):
        s = ctypes.c_int64(); m = ctypes.c_int32()
        ok = lib().orc_flow_query(self._h, txhash, len(txhash), ctypes.byref(s), ctypes.byref(m))
        return (s.value, bool(m.value)) if ok else None

    def get_votes(self, txhash: bytes):
        """TxVoteSet.GetVotes in validator order: [(validator index, signature bytes)]"""
        np = self._np
        n = lib().orc_flow_get_votes(self._h, txhash, len(txhash), None, None, 0)
        vals = np.zeros(max(n, 1), np.uint32)
        sigs = np.zeros((max(n, 1), 64), np.uint8)
        lib().orc_flow_get_votes(self._h, txhash, len(txhash), vals.ctypes.data, sigs.ctypes.data, n)
        return [(int(vals[j]), sigs[j].tobytes()) for j in range(n)]

    def num_sets(self):
        return lib().orc_flow_num_sets(self._h)

    def num_verifies(self):
        return lib().orc_flow_num_verifies(self._h)


def verify_many(pubs32, val_idx, arena, msg_off, msg_len, sigs64, threads=1):
    """Timed CPU verify (bench cpu_baseline).  Returns (seconds, ok uint8 array)."""
    import numpy as np
    n = len(val_idx)
    out = np.zeros(n, np.uint8)
    arrs = [np.ascontiguousarray(a) for a in (pubs32, val_idx.astype(np.uint32), arena,
                                              msg_off.astype(np.uint32), msg_len.astype(np.uint16), sigs64)]
    t = lib().orc_verify_many(*[a.ctypes.data for a in arrs], n, threads, out.ctypes.data)
    return t, out


def _orc_vote(v, keep):
    """orc_vote from an oracle-style dict (nil, height, txhash, ts_sec, ts_nanos, addr, sig)"""
    ov = _Vote()
    bufs = [ctypes.create_string_buffer(bytes(v.get(k, b"")) or b"\0", max(len(v.get(k, b"")), 1))
            for k in ("txhash", "addr", "sig")]
    keep.append(bufs)
    ov.is_nil = 1 if v.get("nil") else 0
    ov.height = v.get("height", 0)
    ov.txhash = ctypes.addressof(bufs[0]); ov.txhash_len = len(v.get("txhash", b""))
    ov.ts_sec = v.get("ts_sec", 0); ov.ts_nanos = v.get("ts_nanos", 0)
    ov.addr = ctypes.addressof(bufs[1]); ov.addr_len = len(v.get("addr", b""))
    ov.sig = ctypes.addressof(bufs[2]); ov.sig_len = len(v.get("sig", b""))
    return ov


class Pool:
    """Sequential TxVotePool restatement (oracle/pool.c); votes as oracle-style dicts with the
    FULL signature bytes."""

    def __init__(self, size=5000, cache_size=10000, max_txs_bytes=1 << 30, max_msg_bytes=1 << 20, height=0,
                 wal=False):
        self._h = lib().orc_pool_new(size, cache_size, max_txs_bytes, max_msg_bytes, height, int(bool(wal)))

    def __del__(self):
        if getattr(self, "_h", None):
            lib().orc_pool_free(self._h)
            self._h = None

    def check(self, votes):
        import numpy as np
        keep = []
        return np.array([lib().orc_pool_check(self._h, ctypes.byref(_orc_vote(v, keep))) for v in votes], np.uint8)

    def check_batch(self, b, long_sigs=None):
        """orc_pool_check over a VoteBatch-shaped object in arrival order; long_sigs: {index: full
        signature bytes} for votes whose sig_len exceeds 64"""
        import numpy as np
        soa = _soa(b)
        full = off = None
        if long_sigs:
            arena = b"".join(long_sigs[i] for i in sorted(long_sigs))
            full = ctypes.create_string_buffer(arena, max(len(arena), 1))
            offs = np.zeros(max(b.n, 1), np.uint64)
            o = 0
            for i in sorted(long_sigs):
                offs[i] = o
                o += len(long_sigs[i])
            off = offs
        out = np.zeros(max(b.n, 1), np.uint8)
        lib().orc_pool_check_soa(self._h, ctypes.addressof(soa), full, None if off is None else off.ctypes.data,
                                 out.ctypes.data)
        return out[:b.n]

    def check_keys(self, keys, sizes):
        """orc_pool_check over (txVoteKey, Size()) pairs: keys [n, 32] u8, sizes [n] u32"""
        import numpy as np
        keys = np.ascontiguousarray(keys, np.uint8)
        sizes = np.ascontiguousarray(sizes, np.uint32)
        n = len(sizes)
        out = np.zeros(max(n, 1), np.uint8)
        lib().orc_pool_check_keys(self._h, keys.ctypes.data, sizes.ctypes.data, n, out.ctypes.data)
        return out[:n]

    def update(self, height, votes):
        keep = []
        arr = (_Vote * max(len(votes), 1))(*[_orc_vote(v, keep) for v in votes])
        lib().orc_pool_update(self._h, height, ctypes.addressof(arr), len(votes))

    def update_keys(self, height, keys, sizes):
        """orc_pool_update over (txVoteKey, Size()) pairs: keys [n, 32] u8, sizes [n] u32"""
        import numpy as np
        keys = np.ascontiguousarray(keys, np.uint8)
        sizes = np.ascontiguousarray(sizes, np.uint32)
        lib().orc_pool_update_keys(self._h, height, keys.ctypes.data, sizes.ctypes.data, len(sizes))

    def update_batch(self, height, b):
        """orc_pool_update over a VoteBatch-shaped object (signatures of at most 64 bytes)"""
        soa = _soa(b)
        lib().orc_pool_update_soa(self._h, height, ctypes.addressof(soa), None, None)

    def reap(self, max_txs=-1):
        import numpy as np
        n = lib().orc_pool_reap(self._h, max_txs, None, None, 0)
        keys = np.zeros((max(n, 1), 32), np.uint8)
        sizes = np.zeros(max(n, 1), np.uint32)
        lib().orc_pool_reap(self._h, max_txs, keys.ctypes.data, sizes.ctypes.data, n)
        return keys[:n], sizes[:n]

    def cache_keys(self):
        import numpy as np
        n = lib().orc_pool_cache_keys(self._h, None, 0)
        keys = np.zeros((max(n, 1), 32), np.uint8)
        lib().orc_pool_cache_keys(self._h, keys.ctypes.data, n)
        return keys[:n]

    def flush(self):
        lib().orc_pool_flush(self._h)

    def size(self):
        return lib().orc_pool_size(self._h)

    def txs_bytes(self):
        return lib().orc_pool_txs_bytes(self._h)


# ---- TxVoteMessage wire codec (oracle/wire.c; txvotepool/reactor.go:170-190, 273-291) ----
WIRE_OK, WIRE_TOO_LARGE, WIRE_ERR_DECODE, WIRE_NIL = range(4)


class _WireVote(ctypes.Structure):
    _fields_ = [("height", ctypes.c_int64), ("txhash_off", ctypes.c_uint32), ("txhash_len", ctypes.c_uint32),
                ("txkey", ctypes.c_uint8 * 32), ("ts_sec", ctypes.c_int64), ("ts_nanos", ctypes.c_int32),
                ("addr_off", ctypes.c_uint32), ("addr_len", ctypes.c_uint32), ("sig_off", ctypes.c_uint32),
                ("sig_len", ctypes.c_uint32)]


def wire_prefix():
    d, p = ctypes.create_string_buffer(3), ctypes.create_string_buffer(4)
    lib().orc_wire_prefix(d, p)
    return d.raw, p.raw


def wire_encode(height, txhash: bytes, ts_sec, ts_nanos, addr: bytes, sig: bytes, txkey: bytes = bytes(32)):
    """cdc.MarshalBinaryBare(&TxVoteMessage{Tx: vote}); None when amino rejects the timestamp."""
    cap = 64 + len(txhash) + len(addr) + len(sig) + 64
    out = ctypes.create_string_buffer(cap)
    n = lib().orc_wire_encode(height, txhash, len(txhash), txkey, ts_sec, ts_nanos, addr, len(addr), sig, len(sig),
                              out, cap)
    return None if n < 0 else out.raw[:n]


def txvote_bytes(height, txhash: bytes, ts_sec, ts_nanos, addr: bytes, sig: bytes, txkey: bytes = bytes(32)):
    """cdc.MarshalBinaryBare(TxVote) -- a CommitSig's bytes (types/tx_vote.go:154-159)."""
    n = lib().orc_txvote_encode(height, txhash, len(txhash), txkey, ts_sec, ts_nanos, addr, len(addr), sig, len(sig),
                                None)
    if n < 0:
        return None
    out = ctypes.create_string_buffer(max(n, 1))
    lib().orc_txvote_encode(height, txhash, len(txhash), txkey, ts_sec, ts_nanos, addr, len(addr), sig, len(sig), out)
    return out.raw[:n]


def _uvarint(v: int) -> bytes:
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def commit_bytes(txhash: bytes, votes) -> bytes:
    """cdc.MustMarshalBinaryBare(Commit{TxHash, Commits}) (types/vote_set.go:242-287, tx/store.go:92):
    field 1 TxHash (omitted when empty), then field 2 once per CommitSig in the given order, each
    length-prefixed with the accepted TxVote's bytes.  votes: dicts (height, ts_sec, ts_nanos, addr,
    sig, txkey)."""
    out = bytearray()
    if txhash:
        out += b"\x0a" + _uvarint(len(txhash)) + txhash
    for v in votes:
        body = txvote_bytes(v["height"], txhash, v["ts_sec"], v["ts_nanos"], v["addr"], v["sig"], v["txkey"])
        out += b"\x12" + _uvarint(len(body)) + body
    return bytes(out)


def save_tx_bytes(txhash: bytes, txkey: bytes, votes):
    """TxStore.SaveTx's two db.Set calls (tx/store.go:83-107): (calcTxKey = "H:%X", the TxVoteSet's
    bytes -- only its exported TxHash (field 1) and TxKey (field 2) --, calcTxCommitKey = "C:%X",
    the MakeCommit bytes)."""
    hexkey = txhash.hex().upper().encode()
    vs = (b"\x0a" + _uvarint(len(txhash)) + txhash if txhash else b"") + b"\x12\x20" + txkey
    return b"H:" + hexkey, vs, b"C:" + hexkey, commit_bytes(txhash, votes)


def wire_decode(bz: bytes, max_msg_bytes: int = 1 << 20):
    """decodeMsg + the *TxVoteMessage type switch: (status, fields dict or None)."""
    o = _WireVote()
    st = lib().orc_wire_decode(bz, len(bz), max_msg_bytes, ctypes.byref(o))
    if st != WIRE_OK:
        return st, None
    return st, dict(height=o.height, txhash=bz[o.txhash_off:o.txhash_off + o.txhash_len], txkey=bytes(o.txkey),
                    ts_sec=o.ts_sec, ts_nanos=o.ts_nanos, addr=bz[o.addr_off:o.addr_off + o.addr_len],
                    sig=bz[o.sig_off:o.sig_off + o.sig_len], txhash_off=o.txhash_off, addr_off=o.addr_off,
                    sig_off=o.sig_off)


def wire_decode_many(wire, off, length, max_msg_bytes=1 << 20):
    """(seconds, statuses) for the C decoder over n messages on one thread (CPU baseline)"""
    import numpy as np
    n = len(off)
    st = np.zeros(max(n, 1), np.uint8)
    out = (_WireVote * max(n, 1))()
    secs = lib().orc_wire_decode_many(wire.ctypes.data, off.ctypes.data, length.ctypes.data, n, max_msg_bytes,
                                      st.ctypes.data, out)
    return secs, st[:n]

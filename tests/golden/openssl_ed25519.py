"""OpenSSL 3 Ed25519 via ctypes (libcrypto.so.3) — an independent RFC 8032 implementation
used to pin the oracle (canonical signatures from OpenSSL are byte-identical
to Go's ed25519.Sign for the same seed).  Test infrastructure only."""
import ctypes
import ctypes.util

EVP_PKEY_ED25519 = 1087
_c = None


def available():
    try:
        _load()
        return True
    except OSError:
        return False


def _load():
    global _c
    if _c is None:
        name = ctypes.util.find_library("crypto") or "libcrypto.so.3"
        c = ctypes.CDLL(name)
        c.EVP_PKEY_new_raw_private_key.restype = ctypes.c_void_p
        c.EVP_PKEY_new_raw_private_key.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]
        c.EVP_PKEY_new_raw_public_key.restype = ctypes.c_void_p
        c.EVP_PKEY_new_raw_public_key.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]
        c.EVP_PKEY_get_raw_public_key.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_size_t)]
        c.EVP_MD_CTX_new.restype = ctypes.c_void_p
        c.EVP_MD_CTX_free.argtypes = [ctypes.c_void_p]
        c.EVP_PKEY_free.argtypes = [ctypes.c_void_p]
        c.EVP_DigestSignInit.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        c.EVP_DigestSign.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_size_t),
                                     ctypes.c_char_p, ctypes.c_size_t]
        c.EVP_DigestVerifyInit.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        c.EVP_DigestVerify.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t]
        _c = c
    return _c


def pubkey(seed: bytes) -> bytes:
    c = _load()
    k = c.EVP_PKEY_new_raw_private_key(EVP_PKEY_ED25519, None, seed, 32)
    out = ctypes.create_string_buffer(32)
    n = ctypes.c_size_t(32)
    assert c.EVP_PKEY_get_raw_public_key(k, out, ctypes.byref(n)) == 1
    c.EVP_PKEY_free(k)
    return out.raw


def sign(seed: bytes, msg: bytes) -> bytes:
    c = _load()
    k = c.EVP_PKEY_new_raw_private_key(EVP_PKEY_ED25519, None, seed, 32)
    ctx = c.EVP_MD_CTX_new()
    assert c.EVP_DigestSignInit(ctx, None, None, None, k) == 1
    sig = ctypes.create_string_buffer(64)
    n = ctypes.c_size_t(64)
    assert c.EVP_DigestSign(ctx, sig, ctypes.byref(n), msg, len(msg)) == 1
    c.EVP_MD_CTX_free(ctx)
    c.EVP_PKEY_free(k)
    return sig.raw


def verify(pub: bytes, msg: bytes, sig: bytes) -> bool:
    c = _load()
    k = c.EVP_PKEY_new_raw_public_key(EVP_PKEY_ED25519, None, pub, 32)
    if not k:
        return False
    ctx = c.EVP_MD_CTX_new()
    ok = c.EVP_DigestVerifyInit(ctx, None, None, None, k) == 1 and \
        c.EVP_DigestVerify(ctx, sig, len(sig), msg, len(msg)) == 1
    c.EVP_MD_CTX_free(ctx)
    c.EVP_PKEY_free(k)
    return ok

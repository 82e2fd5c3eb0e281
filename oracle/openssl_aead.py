"""CPU baseline for the content-encryption legs (test/measurement infrastructure only: tests/
and bench.py's cpu_baseline legs use it; nothing in kopia_amd/ imports it).

Kopia seals a content with Go's crypto (repo/encryption/aes256_gcm_hmac_sha256_encryptor.go,
chacha20_poly1305_hmac_sha256_encryptor.go): key = HMAC-SHA256(secret, contentID), then
AES-256-GCM or ChaCha20-Poly1305 with a 12-byte nonce and aad = contentID, output
nonce || ciphertext || tag.  Go is not installed here, so the C-speed stand-in is OpenSSL's
EVP AEAD (libcrypto.so.3, which Python's own _hashlib/ssl link) through ctypes, plus the
stdlib's C HMAC.  It reproduces the reference's ciphertext samples byte for byte
(tests/test_aead_oracle.py), so it computes exactly what Kopia computes, at library speed.
ctypes releases the GIL, so threads seal different chunks in parallel.
"""
from __future__ import annotations

import ctypes as C
import hmac
import threading
import time
from hashlib import sha256

_CRYPTO = None
_EVP_CTRL_AEAD_SET_IVLEN = 0x9
_EVP_CTRL_AEAD_GET_TAG = 0x10
_EVP_CTRL_AEAD_SET_TAG = 0x11


def _lib():
    global _CRYPTO
    if _CRYPTO is None:
        L = C.CDLL("libcrypto.so.3")
        L.EVP_CIPHER_CTX_new.restype = C.c_void_p
        L.EVP_CIPHER_CTX_free.argtypes = [C.c_void_p]
        for f in ("EVP_aes_256_gcm", "EVP_chacha20_poly1305"):
            getattr(L, f).restype = C.c_void_p
        L.EVP_EncryptInit_ex.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_char_p, C.c_char_p]
        L.EVP_EncryptUpdate.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_int), C.c_void_p, C.c_int]
        L.EVP_EncryptFinal_ex.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_int)]
        L.EVP_CIPHER_CTX_ctrl.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p]
        _CRYPTO = L
    return _CRYPTO


def available() -> bool:
    try:
        _lib()
        return True
    except OSError:
        return False


AES = "AES256-GCM-HMAC-SHA256"
CHACHA = "CHACHA20-POLY1305-HMAC-SHA256"


class Sealer:
    """One EVP context (one per thread)."""

    def __init__(self, algo: str):
        L = _lib()
        self.L = L
        self.cipher = L.EVP_aes_256_gcm() if algo == AES else L.EVP_chacha20_poly1305()
        self.ctx = L.EVP_CIPHER_CTX_new()

    def __del__(self):
        try:
            self.L.EVP_CIPHER_CTX_free(self.ctx)
        except Exception:
            pass

    def seal_into(self, key: bytes, nonce: bytes, aad: bytes, src_ptr: int, n: int, dst_ptr: int) -> bytes:
        """Encrypt n bytes at src_ptr into dst_ptr; returns the 16-byte tag."""
        L, ctx = self.L, self.ctx
        outl = C.c_int(0)
        ok = L.EVP_EncryptInit_ex(ctx, self.cipher, None, None, None)
        ok &= L.EVP_CIPHER_CTX_ctrl(ctx, _EVP_CTRL_AEAD_SET_IVLEN, 12, None)
        ok &= L.EVP_EncryptInit_ex(ctx, None, None, key, nonce)
        ok &= L.EVP_EncryptUpdate(ctx, None, C.byref(outl), aad, len(aad))
        done = 0
        while done < n:  # EVP takes int lengths
            k = min(n - done, 1 << 30)
            ok &= L.EVP_EncryptUpdate(ctx, dst_ptr + done, C.byref(outl), src_ptr + done, k)
            done += k
        ok &= L.EVP_EncryptFinal_ex(ctx, dst_ptr + n, C.byref(outl))
        tag = C.create_string_buffer(16)
        ok &= L.EVP_CIPHER_CTX_ctrl(ctx, _EVP_CTRL_AEAD_GET_TAG, 16, tag)
        if ok != 1:
            raise RuntimeError("OpenSSL EVP AEAD failed")
        return tag.raw

    def kopia_encrypt(self, secret: bytes, content_id: bytes, nonce: bytes, plaintext: bytes) -> bytes:
        """The reference Encrypt(): nonce || AEAD(HMAC-SHA256(secret, id), nonce, pt, aad = id)."""
        key = hmac.new(secret, content_id, sha256).digest()
        src = C.create_string_buffer(plaintext, len(plaintext))
        dst = C.create_string_buffer(len(plaintext) + 1)
        tag = self.seal_into(key, nonce, content_id, C.addressof(src), len(plaintext), C.addressof(dst))
        return nonce + dst.raw[:len(plaintext)] + tag


def seal_rate(algo: str, secret: bytes, buf, offs, lens, ids, nonces: bytes, nthreads: int) -> dict:
    """Seal chunk i = buf[offs[i]: +lens[i]] (a C-contiguous uint8 numpy array) with content ID
    ids[i] and nonce nonces[12 i: 12 i + 12], every chunk once, over `nthreads` threads
    (chunks dealt round-robin).  Returns wall seconds and plaintext bytes."""
    import numpy as np
    n = len(offs)
    out = np.empty(int(max(lens)) + 16 if n else 16, dtype=np.uint8)
    base = buf.ctypes.data
    keys = [hmac.new(secret, bytes(ids[i]), sha256).digest() for i in range(n)]  # per-content key (HMAC)

    def work(t, outs):
        s = Sealer(algo)
        o = outs[t]
        for i in range(t, n, nthreads):
            s.seal_into(keys[i], nonces[12 * i:12 * i + 12], bytes(ids[i]), base + int(offs[i]), int(lens[i]),
                        o.ctypes.data)

    outs = [np.empty_like(out) for _ in range(nthreads)]
    th = [threading.Thread(target=work, args=(t, outs)) for t in range(nthreads)]
    t0 = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    dt = time.perf_counter() - t0
    return {"seconds": dt, "bytes": int(sum(int(x) for x in lens)), "threads": nthreads}

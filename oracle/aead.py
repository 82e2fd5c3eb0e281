"""ORACLE / TEST INFRASTRUCTURE ONLY -- never imported by the product path.

Restatement of the published algorithms behind Kopia's CHACHA20-POLY1305-HMAC-SHA256
content encryption (repo/encryption/chacha20_poly1305_hmac_sha256_encryptor.go,
aead_helpers.go, encryption.go:82-95), whose arithmetic lives in golang.org/x/crypto
(chacha20poly1305, not vendored here) and the Go standard library (crypto/hkdf,
crypto/hmac, crypto/sha256):
* deriveKey: HKDF-SHA256(masterKey, salt = purpose ("encryption"), info = "", 32 bytes)
  (RFC 5869; Go's hkdf.Key(h, secret, salt, info, n) -- encryption.go:82-95);
* per content: key = HMAC-SHA256(derived, id), id = the content ID the Encryptor is given (the
  content manager passes the last 16 bytes of the content hash,
  repo/content/content_manager_lock_free.go:178-182);
* Seal: output = nonce(12) || ChaCha20-Poly1305(key, nonce, plaintext, aad = iv)
  (RFC 8439 §2.8; aead_helpers.go: random nonce prefix).
Pinned by the RFC 8439 / RFC 5869 example vectors and the reference's own ciphertext samples
(repo/encryption/encryption_test.go:97-127, tests/golden/kopia_encryption_samples.json), which it
re-seals byte for byte (tests/test_aead_oracle.py).
"""
from __future__ import annotations

import hashlib
import hmac
import struct

import numpy as np


def hkdf_sha256(ikm: bytes, salt: bytes, info: bytes, n: int) -> bytes:
    prk = hmac.new(salt, ikm, hashlib.sha256).digest()
    out, t, i = b"", b"", 1
    while len(out) < n:
        t = hmac.new(prk, t + info + bytes([i]), hashlib.sha256).digest()
        out += t
        i += 1
    return out[:n]


def derive_key(master_key: bytes, purpose: bytes = b"encryption", n: int = 32) -> bytes:
    """encryption.go deriveKey (hkdf.Key(sha256.New, masterKey, purpose, "", n))."""
    return hkdf_sha256(master_key, purpose, b"", n)


def _rotl(x, n):
    return ((x << n) | (x >> (32 - n))) & 0xFFFFFFFF


def chacha20_block(key: bytes, counter: int, nonce: bytes) -> bytes:
    """RFC 8439 §2.3."""
    c = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574]
    st = c + list(struct.unpack("<8I", key)) + [counter & 0xFFFFFFFF] + list(struct.unpack("<3I", nonce))
    x = st[:]

    def qr(a, b, cc, d):
        x[a] = (x[a] + x[b]) & 0xFFFFFFFF; x[d] = _rotl(x[d] ^ x[a], 16)
        x[cc] = (x[cc] + x[d]) & 0xFFFFFFFF; x[b] = _rotl(x[b] ^ x[cc], 12)
        x[a] = (x[a] + x[b]) & 0xFFFFFFFF; x[d] = _rotl(x[d] ^ x[a], 8)
        x[cc] = (x[cc] + x[d]) & 0xFFFFFFFF; x[b] = _rotl(x[b] ^ x[cc], 7)

    for _ in range(10):
        qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15)
        qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14)
    return struct.pack("<16I", *[(x[i] + st[i]) & 0xFFFFFFFF for i in range(16)])


def _chacha20_blocks_np(key: bytes, counter: int, nonce: bytes, nblocks: int) -> bytes:
    """The keystream of blocks counter .. counter + nblocks - 1 (RFC 8439 §2.3), every block
    at once as numpy uint32 lanes -- the same rounds as chacha20_block."""
    st = [np.full(nblocks, w, np.uint32) for w in (0x61707865, 0x3320646E, 0x79622D32, 0x6B206574)]
    st += [np.full(nblocks, w, np.uint32) for w in struct.unpack("<8I", key)]
    st += [(np.arange(nblocks, dtype=np.uint64) + counter).astype(np.uint32)]
    st += [np.full(nblocks, w, np.uint32) for w in struct.unpack("<3I", nonce)]
    x = [a.copy() for a in st]

    def rotl(v, n):
        return (v << np.uint32(n)) | (v >> np.uint32(32 - n))

    def qr(a, b, c, d):
        x[a] += x[b]; x[d] = rotl(x[d] ^ x[a], 16)
        x[c] += x[d]; x[b] = rotl(x[b] ^ x[c], 12)
        x[a] += x[b]; x[d] = rotl(x[d] ^ x[a], 8)
        x[c] += x[d]; x[b] = rotl(x[b] ^ x[c], 7)

    for _ in range(10):
        qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15)
        qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14)
    out = np.stack([x[i] + st[i] for i in range(16)], axis=1).astype("<u4")
    return out.tobytes()


def chacha20_xor(key: bytes, counter: int, nonce: bytes, data: bytes) -> bytes:
    """RFC 8439 §2.4 (numpy XOR of the keystream)."""
    n = len(data)
    ks = _chacha20_blocks_np(key, counter, nonce, (n + 63) // 64)
    return (np.frombuffer(data, np.uint8) ^ np.frombuffer(ks[:n], np.uint8)).tobytes()


def poly1305(key: bytes, msg: bytes) -> bytes:
    """RFC 8439 §2.5."""
    r = int.from_bytes(key[:16], "little") & 0x0FFFFFFC0FFFFFFC0FFFFFFC0FFFFFFF
    s = int.from_bytes(key[16:], "little")
    p = (1 << 130) - 5
    acc = 0
    for i in range(0, len(msg), 16):
        blk = msg[i:i + 16]
        acc = (acc + int.from_bytes(blk + b"\x01", "little")) * r % p
    return ((acc + s) & ((1 << 128) - 1)).to_bytes(16, "little")


def _pad16(b: bytes) -> bytes:
    return b"" if len(b) % 16 == 0 else bytes(16 - len(b) % 16)


def chacha20poly1305_seal(key: bytes, nonce: bytes, plaintext: bytes, aad: bytes) -> bytes:
    """RFC 8439 §2.8: ciphertext || tag."""
    otk = chacha20_block(key, 0, nonce)[:32]
    ct = chacha20_xor(key, 1, nonce, plaintext)
    mac = aad + _pad16(aad) + ct + _pad16(ct) + struct.pack("<QQ", len(aad), len(ct))
    return ct + poly1305(otk, mac)


def kopia_encrypt(derived: bytes, content_id: bytes, nonce: bytes, plaintext: bytes) -> bytes:
    """chacha20poly1305hmacSha256Encryptor.Encrypt with a given nonce (the reference draws it
    from crypto/rand): nonce || Seal(key = HMAC-SHA256(derived, content_id), aad = content_id).
    The content manager passes the last 16 bytes of the content hash as content_id."""
    key = hmac.new(derived, content_id, hashlib.sha256).digest()
    return nonce + chacha20poly1305_seal(key, nonce, plaintext, content_id)


def kopia_decrypt(derived: bytes, content_id: bytes, sealed: bytes) -> bytes | None:
    """Decrypt (aeadOpenPrefixedWithNonce): None when authentication fails."""
    if len(sealed) < 28:
        return None
    key = hmac.new(derived, content_id, hashlib.sha256).digest()
    nonce, body = sealed[:12], sealed[12:]
    otk = chacha20_block(key, 0, nonce)[:32]
    ct, tag = body[:-16], body[-16:]
    mac = content_id + _pad16(content_id) + ct + _pad16(ct) + struct.pack("<QQ", len(content_id), len(ct))
    if not hmac.compare_digest(poly1305(otk, mac), tag):
        return None
    return chacha20_xor(key, 1, nonce, ct)

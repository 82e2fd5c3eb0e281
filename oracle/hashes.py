"""TEST INFRASTRUCTURE ONLY (imported by tests/, __graft_entry__.smoke() and bench.py's checks):
Kopia's content hash functions, HashFunc(nil, data) for every registered name
(repo/hashing/hashing.go:55-103, blake_hashes.go:8-13, blake3_hashes.go:10-27, sha_hashes.go:9-15).

- BLAKE2b/2s: Python's hashlib (RFC 7693), keyed with the secret, digest truncated.
- HMAC-SHA224/256, HMAC-SHA3-224/256: Python's hmac over hashlib (RFC 2104; FIPS 180-4 / 202).
- BLAKE3-256(-128): oracle/blake3_oracle.c (restated from the BLAKE3 spec; zeebo/blake3 is not
  vendored), keyed with the secret's first 32 bytes, or with
  DeriveKey("kopia blake3 derived key v1", secret) for a shorter secret (blake3_hashes.go:12-19).
All pinned by published vectors (tests/golden/blake2_kat.json, hash_kat_more.json).
"""
from __future__ import annotations

import ctypes as C
import hashlib
import hmac

# name -> (family, digest parameter, bytes kept)
KOPIA = {
    "BLAKE2B-256": ("blake2b", 32, 32),
    "BLAKE2B-256-128": ("blake2b", 32, 16),
    "BLAKE2S-128": ("blake2s", 16, 16),
    "BLAKE2S-256": ("blake2s", 32, 32),
    "BLAKE3-256": ("blake3", 32, 32),
    "BLAKE3-256-128": ("blake3", 32, 16),
    "HMAC-SHA224": ("sha224", 0, 28),
    "HMAC-SHA256": ("sha256", 0, 32),
    "HMAC-SHA256-128": ("sha256", 0, 16),
    "HMAC-SHA3-224": ("sha3_224", 0, 28),
    "HMAC-SHA3-256": ("sha3_256", 0, 32),
}
BLAKE3_KDF_CONTEXT = "kopia blake3 derived key v1"  # blake3_hashes.go:15


def _lib():
    from oracle import coracle
    L = coracle.lib()
    L.orc_blake3.restype = None
    L.orc_blake3.argtypes = [C.c_char_p, C.c_char_p, C.c_int64, C.c_char_p]
    L.orc_blake3_derive_key.restype = None
    L.orc_blake3_derive_key.argtypes = [C.c_char_p, C.c_char_p, C.c_int64, C.c_char_p]
    return L


def blake3(data: bytes, key: bytes | None = None) -> bytes:
    out = C.create_string_buffer(32)
    _lib().orc_blake3(key, data, len(data), out)
    return out.raw


def blake3_derive_key(context: str, material: bytes) -> bytes:
    out = C.create_string_buffer(32)
    _lib().orc_blake3_derive_key(context.encode(), material, len(material), out)
    return out.raw


def blake3_key(secret: bytes) -> bytes:
    """newBlake3(key) (blake3_hashes.go:10-22): stretch a short secret, else its first 32 bytes."""
    return blake3_derive_key(BLAKE3_KDF_CONTEXT, secret) if len(secret) < 32 else secret[:32]


def kopia_hash(name: str, key: bytes, data: bytes) -> bytes:
    fam, nn, keep = KOPIA[name]
    if fam == "blake2b":
        return hashlib.blake2b(data, key=key, digest_size=nn).digest()[:keep]
    if fam == "blake2s":
        return hashlib.blake2s(data, key=key, digest_size=nn).digest()[:keep]
    if fam == "blake3":
        return blake3(data, blake3_key(key))[:keep]
    return hmac.new(key, data, getattr(hashlib, fam)).digest()[:keep]

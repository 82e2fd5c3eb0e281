"""ORACLE / TEST INFRASTRUCTURE ONLY -- never imported by the product path.

Restatement of the published algorithms behind Kopia's default content encryption,
AES256-GCM-HMAC-SHA256 (repo/encryption/aes256_gcm_hmac_sha256_encryptor.go:24-47 aeadForContent,
:49-65 Encrypt/Decrypt, aead_helpers.go:12-75 nonce prefix), whose arithmetic is Go's crypto/aes and
crypto/cipher NewGCM (standard library, absent here):
* per content: key = HMAC-SHA256(derived, content ID) (32 bytes -> AES-256),
* Seal: nonce(12) || AES-256-GCM(key, nonce, plaintext, aad = content ID) (NIST SP 800-38D,
  96-bit IV: J0 = nonce || 0^31 || 1, CTR from inc32(J0), tag = GHASH ^ E(J0), 16 bytes).
The S-box is derived (FIPS-197 §5.1.1: inverse in GF(2^8), then the affine map) rather than typed in.
Pinned by the FIPS-197 Appendix C.3 AES-256 vector, the SP 800-38D / McGrew-Viega GCM test cases
13-16 (AES-256; tests/golden/aesgcm_kat.json) and the reference's own AES256-GCM-HMAC-SHA256
ciphertext samples (encryption_test.go:97-127), which it opens and re-seals byte for byte.
The keystream is vectorised over blocks with numpy; GHASH uses 4-bit tables over Python ints."""
from __future__ import annotations

import hashlib
import hmac
import struct

import numpy as np


def _xt(a: int) -> int:
    return ((a << 1) ^ 0x11B) & 0xFF if a & 0x80 else a << 1


def _gmul8(a: int, b: int) -> int:
    r = 0
    while b:
        if b & 1:
            r ^= a
        a, b = _xt(a), b >> 1
    return r


def _make_sbox() -> list[int]:
    s = []
    for x in range(256):
        inv = 0
        if x:
            inv = next(y for y in range(1, 256) if _gmul8(x, y) == 1)
        b, out = inv, 0x63
        for k in range(5):  # b ^ rotl(b,1) ^ rotl(b,2) ^ rotl(b,3) ^ rotl(b,4) ^ 0x63
            out ^= ((b << k) | (b >> (8 - k))) & 0xFF
        s.append(out)
    return s


SBOX = _make_sbox()
_SB = np.array(SBOX, dtype=np.uint8)
_M2 = np.array([_xt(x) for x in range(256)], dtype=np.uint8)


def expand_key(key: bytes) -> list[bytes]:
    """FIPS-197 §5.2 for a 32-byte key: 15 round keys of 16 bytes."""
    assert len(key) == 32
    w = [list(key[4 * i:4 * i + 4]) for i in range(8)]
    rcon = 1
    for i in range(8, 60):
        t = list(w[i - 1])
        if i % 8 == 0:
            t = [SBOX[b] for b in t[1:] + t[:1]]
            t[0] ^= rcon
            rcon = _xt(rcon)
        elif i % 8 == 4:
            t = [SBOX[b] for b in t]
        w.append([a ^ b for a, b in zip(w[i - 8], t)])
    return [bytes(sum(w[4 * r:4 * r + 4], [])) for r in range(15)]


def aes_encrypt_blocks(round_keys: list[bytes], blocks: np.ndarray) -> np.ndarray:
    """FIPS-197 §5.1 Cipher on an (N, 16) uint8 array (state column-major: byte 4c + r)."""
    s = blocks.astype(np.uint8) ^ np.frombuffer(round_keys[0], np.uint8)
    shift = np.array([(4 * ((i // 4 + i % 4) % 4) + i % 4) for i in range(16)])  # ShiftRows source
    for rnd in range(1, 15):
        s = _SB[s][:, shift]
        if rnd != 14:
            c = s.reshape(-1, 4, 4)
            a0, a1, a2, a3 = c[:, :, 0], c[:, :, 1], c[:, :, 2], c[:, :, 3]
            t = a0 ^ a1 ^ a2 ^ a3
            c = np.stack([a0 ^ t ^ _M2[a0 ^ a1], a1 ^ t ^ _M2[a1 ^ a2], a2 ^ t ^ _M2[a2 ^ a3],
                          a3 ^ t ^ _M2[a3 ^ a0]], axis=2)
            s = c.reshape(-1, 16)
        s = s ^ np.frombuffer(round_keys[rnd], np.uint8)
    return s


def aes256_encrypt_block(key: bytes, block: bytes) -> bytes:
    return aes_encrypt_blocks(expand_key(key), np.frombuffer(block, np.uint8).reshape(1, 16)).tobytes()


# ---------------------------------------------------------------- GHASH (SP 800-38D §6.3)
_R = 0xE1 << 120


def gf_mul(x: int, y: int) -> int:
    """X * Y in GCM's field, blocks as big-endian 128-bit ints (bit 127 = coefficient of x^0)."""
    z, v = 0, y
    for i in range(127, -1, -1):
        if (x >> i) & 1:
            z ^= v
        v = (v >> 1) ^ _R if v & 1 else v >> 1
    return z


def _ghash_tables(h: int) -> list[list[int]]:
    """t[k][n] = (n at nibble k) * H, so X * H = XOR_k t[k][nibble_k(X)]."""
    p = [0] * 128  # p[i] = H * x^i
    v = h
    for i in range(128):
        p[i] = v
        v = (v >> 1) ^ _R if v & 1 else v >> 1
    tabs = []
    for k in range(32):
        row = []
        for n in range(16):
            acc = 0
            for t in range(4):
                if (n >> t) & 1:
                    acc ^= p[127 - 4 * k - t]
            row.append(acc)
        tabs.append(row)
    return tabs


def ghash(h: int, data: bytes) -> int:
    """GHASH_H over data already padded to 16-byte blocks."""
    tabs = _ghash_tables(h)
    x = 0
    for i in range(0, len(data), 16):
        y = x ^ int.from_bytes(data[i:i + 16], "big")
        z = 0
        for k in range(32):
            z ^= tabs[k][(y >> (4 * k)) & 15]
        x = z
    return x


def ghash_c(h: int, data: bytes) -> int:
    """The same GHASH through oracle/gcm_oracle.c (liboracle.so), for large test chunks."""
    import ctypes as C
    from . import coracle
    out = C.create_string_buffer(16)
    coracle.lib().oracle_ghash(h.to_bytes(16, "big"), data, C.c_uint64(len(data) // 16), out)
    return int.from_bytes(out.raw, "big")


def _ghash(h: int, data: bytes) -> int:
    return ghash_c(h, data) if len(data) > (64 << 10) else ghash(h, data)


def _pad16(b: bytes) -> bytes:
    return b"" if len(b) % 16 == 0 else bytes(16 - len(b) % 16)


def _ctr(rk: list[bytes], nonce: bytes, first: int, nblocks: int) -> bytes:
    ctr = (np.arange(nblocks, dtype=np.uint64) + first).astype(np.uint32).astype(">u4")
    blocks = np.zeros((nblocks, 16), np.uint8)
    blocks[:, :12] = np.frombuffer(nonce, np.uint8)
    blocks[:, 12:] = ctr.view(np.uint8).reshape(nblocks, 4)
    return aes_encrypt_blocks(rk, blocks).tobytes()


def gcm_seal(key: bytes, nonce: bytes, plaintext: bytes, aad: bytes) -> bytes:
    """AES-256-GCM with a 96-bit nonce: ciphertext || tag (SP 800-38D §7.1)."""
    assert len(nonce) == 12
    rk = expand_key(key)
    h = int.from_bytes(aes_encrypt_blocks(rk, np.zeros((1, 16), np.uint8)).tobytes(), "big")
    n = len(plaintext)
    ks = _ctr(rk, nonce, 2, (n + 15) // 16) if n else b""
    ct = (np.frombuffer(plaintext, np.uint8) ^ np.frombuffer(ks[:n], np.uint8)).tobytes()
    s = _ghash(h, aad + _pad16(aad) + ct + _pad16(ct) + struct.pack(">QQ", 8 * len(aad), 8 * n))
    ej0 = int.from_bytes(_ctr(rk, nonce, 1, 1), "big")
    return ct + (s ^ ej0).to_bytes(16, "big")


def gcm_open(key: bytes, nonce: bytes, sealed: bytes, aad: bytes) -> bytes | None:
    if len(sealed) < 16:
        return None
    ct, tag = sealed[:-16], sealed[-16:]
    rk = expand_key(key)
    h = int.from_bytes(aes_encrypt_blocks(rk, np.zeros((1, 16), np.uint8)).tobytes(), "big")
    s = _ghash(h, aad + _pad16(aad) + ct + _pad16(ct) + struct.pack(">QQ", 8 * len(aad), 8 * len(ct)))
    ej0 = int.from_bytes(_ctr(rk, nonce, 1, 1), "big")
    if not hmac.compare_digest((s ^ ej0).to_bytes(16, "big"), tag):
        return None
    n = len(ct)
    ks = _ctr(rk, nonce, 2, (n + 15) // 16) if n else b""
    return (np.frombuffer(ct, np.uint8) ^ np.frombuffer(ks[:n], np.uint8)).tobytes()


def kopia_encrypt(derived: bytes, content_id: bytes, nonce: bytes, plaintext: bytes) -> bytes:
    """aes256GCMHmacSha256.Encrypt with a given nonce (the reference draws it from crypto/rand)."""
    key = hmac.new(derived, content_id, hashlib.sha256).digest()
    return nonce + gcm_seal(key, nonce, plaintext, content_id)


def kopia_decrypt(derived: bytes, content_id: bytes, sealed: bytes) -> bytes | None:
    """aes256GCMHmacSha256.Decrypt: None when the input is short or authentication fails."""
    if len(sealed) < 28:
        return None
    key = hmac.new(derived, content_id, hashlib.sha256).digest()
    return gcm_open(key, sealed[:12], sealed[12:], content_id)

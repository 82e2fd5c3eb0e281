"""The AES256-GCM-HMAC-SHA256 oracle (oracle/aesgcm.py) pinned by the published FIPS-197 and GCM
vectors (tests/golden/aesgcm_kat.json) and by the reference's own ciphertext samples
(repo/encryption/encryption_test.go:97-127, tests/golden/kopia_encryption_samples.json).  CPU only."""
import os
import random

import pytest

from conftest import golden
from oracle import aead, aesgcm

V = golden("aesgcm_kat.json")
ALG = "AES256-GCM-HMAC-SHA256"


def test_sbox_is_fips197():
    s = aesgcm.SBOX
    assert (s[0x00], s[0x01], s[0x53], s[0xFF]) == (0x63, 0x7C, 0xED, 0x16)
    assert sorted(s) == list(range(256))


def test_aes256_block():
    v = V["aes256"]
    got = aesgcm.aes256_encrypt_block(bytes.fromhex(v["key"]), bytes.fromhex(v["plaintext"]))
    assert got.hex() == v["ciphertext"]


@pytest.mark.parametrize("case", V["gcm"], ids=lambda c: str(c["case"]))
def test_gcm_vectors(case):
    key, iv = bytes.fromhex(case["key"]), bytes.fromhex(case["iv"])
    pt, aad = bytes.fromhex(case["plaintext"]), bytes.fromhex(case["aad"])
    out = aesgcm.gcm_seal(key, iv, pt, aad)
    assert out[:-16].hex() == case["ciphertext"]
    assert out[-16:].hex() == case["tag"]
    assert aesgcm.gcm_open(key, iv, out, aad) == pt
    bad = bytearray(out)
    bad[-1] ^= 1
    assert aesgcm.gcm_open(key, iv, bytes(bad), aad) is None


def test_reference_ciphertext_samples():
    """Each AES256-GCM-HMAC-SHA256 sample opens to its payload with the HKDF-derived secret, and
    sealing the payload with the sample's nonce reproduces it byte for byte."""
    for c in golden("kopia_encryption_samples.json")["cases"]:
        secret = aead.derive_key(c["master_key"].encode())
        cid, payload = c["content_id"].encode(), c["payload"].encode()
        sample = bytes.fromhex(c["samples"][ALG])
        assert aesgcm.kopia_decrypt(secret, cid, sample) == payload
        assert aesgcm.kopia_encrypt(secret, cid, sample[:12], payload) == sample
        assert aesgcm.kopia_decrypt(secret, cid + b"x", sample) is None
        assert aesgcm.kopia_decrypt(secret, cid, sample[:27]) is None


def test_c_ghash_matches_python():
    rng = random.Random(5)
    for nblk in (0, 1, 2, 17, 300):
        h = rng.getrandbits(128)
        data = os.urandom(16 * nblk)
        assert aesgcm.ghash_c(h, data) == aesgcm.ghash(h, data)


def test_gf_mul_matches_tables():
    rng = random.Random(9)
    for _ in range(20):
        x, h = rng.getrandbits(128), rng.getrandbits(128)
        assert aesgcm.ghash(h, x.to_bytes(16, "big")) == aesgcm.gf_mul(x, h)

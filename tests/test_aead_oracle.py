"""The encryption oracle (oracle/aead.py) pinned by the published RFC 8439 and RFC 5869
example vectors (tests/golden/aead_kat.json).  CPU only."""
import numpy as np
import pytest

from conftest import golden
from oracle import aead

V = golden("aead_kat.json")


def test_chacha20_block():
    v = V["chacha20_block"]
    got = aead.chacha20_block(bytes.fromhex(v["key"]), v["counter"], bytes.fromhex(v["nonce"]))
    assert got.hex() == v["out"]


def test_chacha20_encrypt():
    v = V["chacha20_encrypt"]
    got = aead.chacha20_xor(bytes.fromhex(v["key"]), v["counter"], bytes.fromhex(v["nonce"]), v["plaintext"].encode())
    assert got.hex() == v["ciphertext"]


def test_poly1305():
    v = V["poly1305"]
    assert aead.poly1305(bytes.fromhex(v["key"]), v["msg"].encode()).hex() == v["tag"]


def test_aead_seal():
    v = V["aead"]
    out = aead.chacha20poly1305_seal(bytes.fromhex(v["key"]), bytes.fromhex(v["nonce"]), v["plaintext"].encode(),
                                     bytes.fromhex(v["aad"]))
    assert out[-16:].hex() == v["tag"]
    assert out[:16].hex() == v["ciphertext_prefix"]


def test_hkdf():
    v = V["hkdf"]
    got = aead.hkdf_sha256(bytes.fromhex(v["ikm"]), bytes.fromhex(v["salt"]), bytes.fromhex(v["info"]), v["L"])
    assert got.hex() == v["okm"]


def test_vectorized_keystream_matches_blocks():
    key, nonce = bytes(range(32)), bytes(range(12))
    ks = aead._chacha20_blocks_np(key, 7, nonce, 5)
    assert ks == b"".join(aead.chacha20_block(key, 7 + j, nonce) for j in range(5))


def test_host_mirror_and_registry():
    """kopia_amd.encryption's host-side key derivation equals the oracle's HKDF, and the
    library's registry and overhead match chacha20_poly1305_hmac_sha256_encryptor.go:16,67."""
    from kopia_amd import encryption as ke
    m = bytes(range(32))
    assert ke.derive_key(m) == aead.derive_key(m)
    assert ke.SupportedAlgorithms() == ["AES256-GCM-HMAC-SHA256", "CHACHA20-POLY1305-HMAC-SHA256"]
    assert ke.overhead("CHACHA20-POLY1305-HMAC-SHA256") == 28
    assert ke.overhead("AES256-GCM-HMAC-SHA256") == 28  # aes256GCMHmacSha256Overhead
    offs, total = ke.sealed_layout([0, 1, 5, 100])
    assert offs.tolist() == [0, 28, 60, 96] and total == 224


def test_reference_ciphertext_samples():
    """The reference's TestCiphertextSamples (encryption_test.go:97-127): the oracle opens every
    CHACHA20-POLY1305-HMAC-SHA256 sample to its payload and, given the sample's nonce, re-seals
    the payload to exactly the sample's bytes."""
    for c in golden("kopia_encryption_samples.json")["cases"]:
        secret = aead.derive_key(c["master_key"].encode())
        cid, payload = c["content_id"].encode(), c["payload"].encode()
        sample = bytes.fromhex(c["samples"]["CHACHA20-POLY1305-HMAC-SHA256"])
        assert aead.kopia_decrypt(secret, cid, sample) == payload
        assert aead.kopia_encrypt(secret, cid, sample[:12], payload) == sample
        bad = bytearray(sample)
        bad[15] ^= 1
        assert aead.kopia_decrypt(secret, cid, bytes(bad)) is None


def test_openssl_cpu_baseline_reproduces_reference_samples():
    """bench.py's CPU baseline for the encryption legs (OpenSSL EVP through ctypes, the C-speed
    stand-in for Go's crypto) seals the reference's TestCiphertextSamples payloads
    (encryption_test.go:97-127) to exactly the samples' bytes, for both encryptors, and agrees with
    the oracles on a 1 MiB chunk."""
    from oracle import aesgcm, openssl_aead as osl
    if not osl.available():
        pytest.skip("libcrypto.so.3 not loadable")
    for c in golden("kopia_encryption_samples.json")["cases"]:
        secret = aead.derive_key(c["master_key"].encode())
        cid, payload = c["content_id"].encode(), c["payload"].encode()
        for algo in (osl.AES, osl.CHACHA):
            sample = bytes.fromhex(c["samples"][algo])
            assert osl.Sealer(algo).kopia_encrypt(secret, cid, sample[:12], payload) == sample
    rng = np.random.default_rng(9)
    pt = rng.integers(0, 256, 1 << 20, dtype=np.uint8).tobytes()
    secret, cid, nonce = bytes(range(32)), bytes(range(16)), bytes(range(12))
    assert osl.Sealer(osl.CHACHA).kopia_encrypt(secret, cid, nonce, pt) == aead.kopia_encrypt(secret, cid, nonce, pt)
    assert osl.Sealer(osl.AES).kopia_encrypt(secret, cid, nonce, pt[:4096]) == \
        aesgcm.kopia_encrypt(secret, cid, nonce, pt[:4096])

"""The encryption oracle (oracle/aead.py) pinned by the published RFC 8439 and RFC 5869
example vectors (tests/golden/aead_kat.json).  CPU only."""
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

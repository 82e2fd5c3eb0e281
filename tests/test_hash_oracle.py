"""The content-hash oracle (Python's hashlib BLAKE2, RFC 7693) pinned by published
known-answer vectors (tests/golden/blake2_kat.json), and Kopia's keyed-hash contract as the
GPU path must reproduce it: blake2b.New256(secret) / blake2s.New128|256(secret), output
truncated (repo/hashing/blake_hashes.go:8-13, hashing.go:78-101).  CPU only."""
import hashlib

import pytest

from conftest import golden

KOPIA = {  # name -> (hashlib constructor, digest_size parameter, bytes kept)
    "BLAKE2B-256-128": (hashlib.blake2b, 32, 16),
    "BLAKE2B-256": (hashlib.blake2b, 32, 32),
    "BLAKE2S-128": (hashlib.blake2s, 16, 16),
    "BLAKE2S-256": (hashlib.blake2s, 32, 32),
}


def kopia_hash(name: str, key: bytes, data: bytes) -> bytes:
    """ORACLE (test infrastructure): HashFunc(nil, data) of repo/hashing for `name`."""
    fn, nn, keep = KOPIA[name]
    return fn(data, key=key, digest_size=nn).digest()[:keep]


@pytest.mark.parametrize("v", golden("blake2_kat.json")["vectors"], ids=lambda v: v["algo"] + "-" + v["hash"][:8])
def test_hashlib_matches_published_vectors(v):
    fn = {"blake2b": hashlib.blake2b, "blake2s": hashlib.blake2s}[v["algo"]]
    got = fn(bytes.fromhex(v["msg_hex"]), key=bytes.fromhex(v["key_hex"]), digest_size=v["digest_size"]).hexdigest()
    assert got == v["hash"]


def test_registered_names_match_the_library():
    from kopia_amd import hashing
    assert hashing.SupportedAlgorithms() == list(KOPIA)
    assert [hashing.hash_size(n) for n in KOPIA] == [k for _, _, k in KOPIA.values()]
    assert hashing.DefaultAlgorithm == "BLAKE2B-256-128"


def test_truncation_is_of_the_256_bit_digest():
    """BLAKE2B-256-128 is the first 16 bytes of the 32-byte digest, not a 16-byte digest
    (the digest length is a BLAKE2 parameter: the two differ)."""
    key, data = b"k" * 32, b"the quick brown fox"
    assert kopia_hash("BLAKE2B-256-128", key, data) == kopia_hash("BLAKE2B-256", key, data)[:16]
    assert kopia_hash("BLAKE2B-256-128", key, data) != hashlib.blake2b(data, key=key, digest_size=16).digest()

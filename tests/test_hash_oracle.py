"""The content-hash oracles (oracle/hashes.py: hashlib BLAKE2 and HMAC-SHA2/SHA3, the C BLAKE3
restatement) pinned by published known-answer vectors (tests/golden/blake2_kat.json,
hash_kat_more.json), and Kopia's keyed-hash contract as the GPU path must reproduce it:
blake2b.New256(secret) / blake2s.New128|256(secret), hmac.New(sha*, secret), blake3.NewKeyed
(derived key for short secrets), output truncated (repo/hashing/*.go).  CPU only."""
import hashlib
import hmac

import pytest

from conftest import golden
from oracle.hashes import KOPIA, blake3, blake3_derive_key, blake3_key, kopia_hash  # noqa: F401


@pytest.mark.parametrize("v", golden("blake2_kat.json")["vectors"], ids=lambda v: v["algo"] + "-" + v["hash"][:8])
def test_hashlib_matches_published_vectors(v):
    fn = {"blake2b": hashlib.blake2b, "blake2s": hashlib.blake2s}[v["algo"]]
    got = fn(bytes.fromhex(v["msg_hex"]), key=bytes.fromhex(v["key_hex"]), digest_size=v["digest_size"]).hexdigest()
    assert got == v["hash"]


def test_registered_names_match_the_library():
    """Every name hashing.go registers, in SupportedAlgorithms()' order (sort.Strings)."""
    from kopia_amd import hashing
    assert list(KOPIA) == sorted(KOPIA)
    assert hashing.SupportedAlgorithms() == list(KOPIA)
    assert [hashing.hash_size(n) for n in KOPIA] == [k for _, _, k in KOPIA.values()]
    assert hashing.DefaultAlgorithm == "BLAKE2B-256-128"


KAT = golden("hash_kat_more.json")


@pytest.mark.parametrize("v", KAT["blake3"], ids=lambda v: str(v["len"]))
def test_blake3_oracle_matches_published_vectors(v):
    data = bytes(i % 251 for i in range(v["len"]))
    assert blake3(data).hex() == v["hash"]
    if "keyed_hash" in v:
        assert blake3(data, b"whats the Elvish word for friend").hex() == v["keyed_hash"]
    if "derive_key" in v:
        assert blake3_derive_key("BLAKE3 2019-12-27 16:29:52 test vectors context", data).hex() == v["derive_key"]


def test_blake3_oracle_abc_and_long_inputs():
    assert blake3(b"abc").hex() == KAT["blake3_abc"]
    # the streaming oracle's stack merges agree with a direct left-complete tree over many chunks
    # (lengths straddling chunk and power-of-two boundaries): determinism + distinctness here,
    # equality with the GPU's level-by-level tree in tests/test_gpu_hash.py
    outs = {n: blake3(bytes(i % 251 for i in range(n))) for n in (1023, 1024, 1025, 2047, 2048, 2049, 8191, 8193)}
    assert len(set(outs.values())) == len(outs)


@pytest.mark.parametrize("v", KAT["hmac"], ids=lambda v: v["algo"])
def test_hmac_oracle_matches_rfc4231(v):
    got = hmac.new(v["key"].encode(), v["data"].encode(), getattr(hashlib, v["algo"])).hexdigest()
    assert got == v["mac"]


def test_kopia_key_rules():
    """blake3_hashes.go:12-19: a secret under 32 bytes is stretched with DeriveKey, a longer
    one is cut to 32 bytes; HMAC names truncate the MAC (sha_hashes.go:10-14)."""
    assert blake3_key(b"k" * 40) == b"k" * 32
    assert blake3_key(b"short") == blake3_derive_key("kopia blake3 derived key v1", b"short")
    d = b"the quick brown fox"
    assert kopia_hash("BLAKE3-256-128", b"s" * 32, d) == blake3(d, b"s" * 32)[:16]
    assert kopia_hash("HMAC-SHA256-128", b"k", d) == hmac.new(b"k", d, hashlib.sha256).digest()[:16]
    assert len(kopia_hash("HMAC-SHA3-224", b"k", d)) == 28


def test_truncation_is_of_the_256_bit_digest():
    """BLAKE2B-256-128 is the first 16 bytes of the 32-byte digest, not a 16-byte digest
    (the digest length is a BLAKE2 parameter: the two differ)."""
    key, data = b"k" * 32, b"the quick brown fox"
    assert kopia_hash("BLAKE2B-256-128", key, data) == kopia_hash("BLAKE2B-256", key, data)[:16]
    assert kopia_hash("BLAKE2B-256-128", key, data) != hashlib.blake2b(data, key=key, digest_size=16).digest()


def _b3_py(data: bytes, key: bytes) -> bytes:
    """A second, recursive BLAKE3 keyed hash in plain Python (small inputs): cross-checks the C
    oracle's streaming construction, including final blocks shorter than 64 bytes."""
    M32 = 0xFFFFFFFF
    IV = [0x6A09E667, 0xBB67AE85, 0x3C6EF372, 0xA54FF53A, 0x510E527F, 0x9B05688C, 0x1F83D9AB, 0x5BE0CD19]
    P = [2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8]
    rot = lambda x, n: ((x >> n) | (x << (32 - n))) & M32

    def g(v, a, b, c, d, x, y):
        v[a] = (v[a] + v[b] + x) & M32; v[d] = rot(v[d] ^ v[a], 16)
        v[c] = (v[c] + v[d]) & M32; v[b] = rot(v[b] ^ v[c], 12)
        v[a] = (v[a] + v[b] + y) & M32; v[d] = rot(v[d] ^ v[a], 8)
        v[c] = (v[c] + v[d]) & M32; v[b] = rot(v[b] ^ v[c], 7)

    def comp(cv, block, t, blen, fl):
        m = [int.from_bytes(block[4 * i:4 * i + 4].ljust(4, b"\0"), "little") for i in range(16)]
        v = cv[:] + IV[:4] + [t & M32, t >> 32, blen, fl]
        for _ in range(7):
            for a, b, c, d, i in ((0, 4, 8, 12, 0), (1, 5, 9, 13, 2), (2, 6, 10, 14, 4), (3, 7, 11, 15, 6),
                                  (0, 5, 10, 15, 8), (1, 6, 11, 12, 10), (2, 7, 8, 13, 12), (3, 4, 9, 14, 14)):
                g(v, a, b, c, d, m[i], m[i + 1])
            m = [m[P[i]] for i in range(16)]
        return [v[i] ^ v[i + 8] for i in range(8)]

    k = [int.from_bytes(key[4 * i:4 * i + 4], "little") for i in range(8)]

    def node(lo, n, root):
        nch = max(1, -(-n // 1024))
        if nch == 1:
            cv, blocks = k[:], [data[lo + i:lo + min(i + 64, n)] for i in range(0, max(n, 1), 64)]
            for j, blk in enumerate(blocks):
                fl = 16 | (1 if j == 0 else 0) | ((2 | (8 if root else 0)) if j == len(blocks) - 1 else 0)
                cv = comp(cv, blk.ljust(64, b"\0"), lo // 1024, len(blk), fl)
            return cv
        left = 1
        while 2 * left < nch:
            left *= 2
        lcv, rcv = node(lo, 1024 * left, False), node(lo + 1024 * left, n - 1024 * left, False)
        blk = b"".join(x.to_bytes(4, "little") for x in lcv + rcv)
        return comp(k, blk, 0, 64, 16 | 4 | (8 if root else 0))

    return b"".join(x.to_bytes(4, "little") for x in node(0, len(data), True))


@pytest.mark.parametrize("n", [0, 1, 63, 64, 65, 119, 1023, 1024, 1025, 2049, 3072, 5000])
def test_blake3_oracle_matches_python_restatement(n):
    data = bytes((7 * i + 3) % 256 for i in range(n))
    key = bytes(range(100, 132))
    assert blake3(data, key) == _b3_py(data, key)

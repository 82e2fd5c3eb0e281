"""ORACLE / TEST INFRASTRUCTURE ONLY — never imported by the product path.

Restatement of the two rolling hashes the reference splitters call, from the
third-party module ``github.com/chmduquesne/rollinghash v4.0.0+incompatible``
(``/root/reference/go.mod:13``, ``go.sum:60-61``; the module is not vendored and
not present in this container).  Call sites that pin the behaviour:

* buzhash32: ``repo/splitter/splitter_buzhash32.go:4,10,21-22,35,47,51,81-82``
  (``buzhash32.New()``, ``Write(64 zero bytes)``, ``Roll``, ``Sum32``, ``Reset``)
* rabinkarp64: ``repo/splitter/splitter_rabinkarp64.go:4,10,21-22,35,47,51,78-79``

Published algorithm restated:

* buzhash32 byte table = 256 *distinct* ``uint32(r.Int63())`` draws from
  ``rand.NewSource(1)``; window 64 bytes; ``Roll``:
  ``sum = rotl32(sum,1) ^ rotl32(T[leave], 64 % 32) ^ T[enter]``.
* rabinkarp64 polynomial = first irreducible ``f`` (Ben-Or test) from 8-byte
  little-endian reads of ``rand.New(rand.NewSource(1))`` with
  ``f &= 2^54-1; f |= 2^53 | 1``.  Tables: ``out[b] = b * x^(8*63) mod P``,
  ``mod[b] = (b * x^53 mod P) | (b << 53)``; ``Roll``:
  ``v ^= out[leave]; i = v >> 45; v = (v << 8 | enter) ^ mod[i]``.
"""
from __future__ import annotations

import hashlib
from functools import lru_cache

import numpy as np

from .gorand import GoRandSource

WINDOW = 64  # splitterSlidingWindowSize, repo/splitter/splitter.go:9


# ----------------------------------------------------------------------------- buzhash32
@lru_cache(maxsize=1)
def buzhash_table() -> np.ndarray:
    """rollinghash/buzhash32 GenerateHashes(1): 256 distinct uint32(Int63())."""
    r = GoRandSource(1)
    used = set()
    out = np.zeros(256, dtype=np.uint32)
    for i in range(256):
        x = r.int63() & 0xFFFFFFFF
        while x in used:
            x = r.int63() & 0xFFFFFFFF
        used.add(x)
        out[i] = x
    return out


def buzhash_table_sha256() -> str:
    return hashlib.sha256(buzhash_table().astype("<u4").tobytes()).hexdigest()


def rotl32(x: int, k: int) -> int:
    k &= 31
    return ((x << k) | (x >> (32 - k))) & 0xFFFFFFFF if k else x


class Buzhash32:
    """Window-of-64 rolling buzhash, state = circular window + sum (module semantics)."""

    def __init__(self):
        self.T = [int(v) for v in buzhash_table()]
        self.reset()

    def reset(self):
        # New() + Write(make([]byte, 64)): window of zeros, sum of 64 zero bytes.
        self.window = bytearray(WINDOW)
        self.oldest = 0
        s = 0
        for i in range(WINDOW):
            s ^= rotl32(self.T[0], WINDOW - 1 - i)
        self.sum = s  # == 0: every rotation of T[0] appears twice

    def roll(self, c: int):
        leave = self.window[self.oldest]
        self.window[self.oldest] = c
        self.oldest = (self.oldest + 1) % WINDOW
        self.sum = rotl32(self.sum, 1) ^ rotl32(self.T[leave], WINDOW % 32) ^ self.T[c]

    def sum32(self) -> int:
        return self.sum


# ----------------------------------------------------------------------------- rabinkarp64
def _gf2_deg(x: int) -> int:
    return x.bit_length() - 1


def _gf2_mod(x: int, m: int) -> int:
    dm = _gf2_deg(m)
    while x and _gf2_deg(x) >= dm:
        x ^= m << (_gf2_deg(x) - dm)
    return x


def _gf2_mulmod(a: int, b: int, m: int) -> int:
    r = 0
    while b:
        if b & 1:
            r ^= a
        b >>= 1
        a <<= 1
    return _gf2_mod(r, m)


def _gf2_gcd(a: int, b: int) -> int:
    while b:
        a, b = b, _gf2_mod(a, b)
    return a


def _irreducible(f: int) -> bool:
    """Ben-Or: gcd(f, x^(2^i) - x mod f) == 1 for i = 1..deg/2."""
    d = _gf2_deg(f)
    xp = 2  # x
    for _ in range(1, d // 2 + 1):
        xp = _gf2_mulmod(xp, xp, f)  # x^(2^i)
        if _gf2_gcd(f, xp ^ 2) != 1:
            return False
    return True


@lru_cache(maxsize=1)
def rabin_polynomial() -> tuple[int, int]:
    """rabinkarp64 RandomPolynomial(1) -> (polynomial, tries)."""
    r = GoRandSource(1)
    for tries in range(1, 1_000_001):
        f = int.from_bytes(r.read(8), "little")
        f &= (1 << 54) - 1
        f |= (1 << 53) | 1
        if _irreducible(f):
            return f, tries
    raise RuntimeError("no irreducible polynomial found")


@lru_cache(maxsize=1)
def rabin_tables() -> tuple[np.ndarray, np.ndarray]:
    P, _ = rabin_polynomial()
    k = _gf2_deg(P)
    xw = _gf2_mod(1 << (8 * (WINDOW - 1)), P)  # x^504 mod P
    out = np.array([_gf2_mulmod(b, xw, P) for b in range(256)], dtype=np.uint64)
    mod = np.array([(_gf2_mod(b << k, P)) | (b << k) for b in range(256)], dtype=np.uint64)
    return out, mod


class RabinKarp64:
    def __init__(self):
        self.P, _ = rabin_polynomial()
        self.shift = _gf2_deg(self.P) - 8
        out, mod = rabin_tables()
        self.out = [int(v) for v in out]
        self.mod = [int(v) for v in mod]
        self.reset()

    def reset(self):
        self.window = bytearray(WINDOW)
        self.oldest = 0
        self.value = 0  # Write(64 zeros): 0 * x^k mod P

    def roll(self, c: int):
        leave = self.window[self.oldest]
        self.window[self.oldest] = c
        self.oldest = (self.oldest + 1) % WINDOW
        v = self.value ^ self.out[leave]
        idx = (v >> self.shift) & 0xFF
        v = ((v << 8) | c) & 0xFFFFFFFFFFFFFFFF
        self.value = v ^ self.mod[idx]

    def sum64(self) -> int:
        return self.value


def rabin_direct(window: bytes) -> int:
    """h = (sum_k b[p-k] x^(8k)) mod P for a 64-byte window (independent check)."""
    P, _ = rabin_polynomial()
    acc = 0
    for b in window:
        acc = (acc << 8) | b
    return _gf2_mod(acc, P)

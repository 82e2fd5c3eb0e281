"""ORACLE / TEST INFRASTRUCTURE ONLY — never imported by the product path.

Restatement of Go's ``math/rand`` (v1) additive lagged-Fibonacci source, which
the reference depends on twice:

* ``repo/splitter/splitter_test.go:13-18`` seeds ``rand.NewSource(5)`` and
  ``Read``s 5,000,000 bytes of KAT input; ``cli/command_benchmark_splitters.go:67-76``
  does the same with seed 42 for ``kopia benchmark splitter``.
* the third-party module ``github.com/chmduquesne/rollinghash v4.0.0+incompatible``
  (``go.mod:13``; absent from /root/reference) derives its buzhash32 byte table and
  its Rabin-Karp polynomial from ``rand.NewSource(1)``.

Go itself is not installed here, so ``rngCooked`` (607 constants of Go's
``math/rand/rng.go``) is regenerated arithmetically, exactly as Go's own
``gen_cooked.go`` defines it: seed a vector with ``srand(1)`` (shifts 20/10, no
cooked XOR) and run 7.8e12 ``vrand`` steps.  Instead of stepping 7.8e12 times we
jump ahead with polynomial arithmetic modulo the recurrence's characteristic
polynomial z^607 - z^334 - 1 over Z/2^64.

Pinned by: SURVEY.md App. A.1 check values (rngCooked[0..2], [606], SHA-256 of
the table; the well-known seed-1 Int63 outputs; SHA-256 of NewSource(5).Read(5e6)
and NewSource(42).Read(1 MiB)) — see tests/test_oracle_gorand.py.
"""
from __future__ import annotations

import hashlib
import os
from functools import lru_cache

import numpy as np

RNG_LEN = 607
RNG_TAP = 273
INT32MAX = (1 << 31) - 1
MASK64 = (1 << 64) - 1
MASK63 = (1 << 63) - 1
N_COOKED_STEPS = 7_800_000_000_000  # gen_cooked.go: 7.8e12 calls to vrand

_CACHE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build", "rngcooked.npy")


def seedrand(x: int) -> int:
    """Go math/rand rng.go seedrand: x*48271 mod (2^31-1) via Schrage."""
    hi, lo = divmod(x, 44488)
    x = 48271 * lo - 3399 * hi
    if x < 0:
        x += INT32MAX
    return x


def _seed_vector(seed: int, shifts: tuple[int, int], cooked) -> np.ndarray:
    """rng.go Seed / gen_cooked.go srand: fill the 607-word vector."""
    seed %= INT32MAX
    if seed < 0:
        seed += INT32MAX
    if seed == 0:
        seed = 89482311
    x = seed
    vec = np.zeros(RNG_LEN, dtype=np.uint64)
    for i in range(-20, RNG_LEN):
        x = seedrand(x)
        if i >= 0:
            u = (x << shifts[0]) & MASK64
            x = seedrand(x)
            u ^= (x << shifts[1]) & MASK64
            x = seedrand(x)
            u ^= x
            if cooked is not None:
                u ^= int(cooked[i])
            vec[i] = u
    return vec


def _polymulmod(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """(a*b) mod (z^607 - z^334 - 1) with uint64 wrap-around coefficients."""
    n = RNG_LEN
    res = np.zeros(2 * n - 1, dtype=np.uint64)
    for j in np.nonzero(a)[0]:
        res[j:j + n] += a[j] * b
    return _reduce(res)


def _reduce(res: np.ndarray) -> np.ndarray:
    n = RNG_LEN
    top = len(res) - 1
    # z^i = z^(i-607) + z^(i-273); process 273-wide blocks from the top so that
    # the targets of a block always lie strictly below the block.
    while top >= n:
        lo = max(n, top - RNG_TAP + 1)
        blk = res[lo:top + 1].copy()
        res[lo:top + 1] = 0
        res[lo - n:top + 1 - n] += blk
        res[lo - RNG_TAP:top + 1 - RNG_TAP] += blk
        top = lo - 1
    return res[:n].copy()


def _z_pow_mod(e: int) -> np.ndarray:
    result = np.zeros(RNG_LEN, dtype=np.uint64)
    result[0] = 1
    base = np.zeros(RNG_LEN, dtype=np.uint64)
    base[1] = 1
    while e:
        if e & 1:
            result = _polymulmod(result, base)
        e >>= 1
        if e:
            base = _polymulmod(base, base)
    return result


def _compute_rng_cooked() -> np.ndarray:
    """gen_cooked.go: srand(1) then 7.8e12 vrand() steps; returns rngVec (as uint64)."""
    v0 = _seed_vector(1, (20, 10), None)
    # Sequence view (see DESIGN.md / oracle notes): step n>=1 writes
    # y_n = y_{n-607} + y_{n-273} to position (334-n) mod 607, with virtual
    # initial values y_n = v0[(334-n) mod 607] for n in [-606, 0].
    # Index shift u_k = y_{k-606}: u_k = u_{k-607} + u_{k-273}, z^607 = z^334 + 1.
    u0 = np.array([v0[(940 - k) % RNG_LEN] for k in range(RNG_LEN)], dtype=np.uint64)
    N = N_COOKED_STEPS
    r = _z_pow_mod(N)  # u_N = sum_j r_j u_j  ->  y_{N-606}
    out = np.zeros(RNG_LEN, dtype=np.uint64)
    with np.errstate(over="ignore"):
        for k in range(RNG_LEN):  # y_{N-606+k} = u_{N+k}
            n = N - 606 + k
            out[(334 - n) % RNG_LEN] = np.sum(r * u0, dtype=np.uint64)
            # multiply r by z
            c = r[-1]
            r = np.concatenate(([np.uint64(0)], r[:-1]))
            r[0] += c
            r[334] += c
    return out


@lru_cache(maxsize=1)
def rng_cooked() -> np.ndarray:
    """The 607 uint64 words of Go's rngCooked (two's-complement of the int64 values)."""
    if os.path.exists(_CACHE):
        v = np.load(_CACHE, allow_pickle=False)
        if v.shape == (RNG_LEN,) and v.dtype == np.uint64:
            return v
    v = _compute_rng_cooked()
    try:
        os.makedirs(os.path.dirname(_CACHE), exist_ok=True)
        np.save(_CACHE, v, allow_pickle=False)
    except OSError:
        pass
    return v


def rng_cooked_sha256() -> str:
    return hashlib.sha256(rng_cooked().astype("<u8").tobytes()).hexdigest()


class GoRandSource:
    """rng.go rngSource + rand.go Rand.Read state (readVal/readPos).

    Scalar Python, for small draws (tables, a few thousand values).  Bulk byte
    streams use ``read_bytes`` below (numpy, block-vectorised) or the C oracle.
    """

    def __init__(self, seed: int):
        self.vec = _seed_vector(seed, (40, 20), rng_cooked()).astype(object)
        self.vec = [int(x) for x in self.vec]
        self.tap = 0
        self.feed = RNG_LEN - RNG_TAP
        self.read_val = 0
        self.read_pos = 0

    def uint64(self) -> int:
        self.tap -= 1
        if self.tap < 0:
            self.tap += RNG_LEN
        self.feed -= 1
        if self.feed < 0:
            self.feed += RNG_LEN
        x = (self.vec[self.feed] + self.vec[self.tap]) & MASK64
        self.vec[self.feed] = x
        return x

    def int63(self) -> int:
        return self.uint64() & MASK63

    def read(self, n: int) -> bytes:
        """rand.go read(): 7 bytes per Int63, state carried across calls."""
        out = bytearray(n)
        pos, val = self.read_pos, self.read_val
        for i in range(n):
            if pos == 0:
                val = self.int63()
                pos = 7
            out[i] = val & 0xFF
            val >>= 8
            pos -= 1
        self.read_pos, self.read_val = pos, val
        return bytes(out)


def uint64_stream(seed: int, count: int) -> np.ndarray:
    """First ``count`` Uint64() outputs of NewSource(seed), numpy-vectorised.

    Step n writes y_n = y_{n-607} + y_{n-273}; 273 consecutive outputs only depend
    on values at least 273 steps older, so blocks of 273 are computed at once.
    """
    v0 = _seed_vector(seed, (40, 20), rng_cooked())
    y = np.zeros(RNG_LEN + count, dtype=np.uint64)
    # y index shift: ys[k] = y_{k-606}; initial y_n = v0[(334-n) mod 607]
    for k in range(RNG_LEN):
        y[k] = v0[(334 - (k - 606)) % RNG_LEN]
    with np.errstate(over="ignore"):
        k = RNG_LEN
        end = RNG_LEN + count
        while k < end:
            e = min(k + RNG_TAP, end)
            y[k:e] = y[k - RNG_LEN:e - RNG_LEN] + y[k - RNG_TAP:e - RNG_TAP]
            k = e
    return y[RNG_LEN:]


def read_bytes(seed: int, n: int) -> bytes:
    """rand.New(rand.NewSource(seed)).Read(make([]byte, n)) on a fresh Rand."""
    nvals = (n + 6) // 7
    v = uint64_stream(seed, nvals) & np.uint64(MASK63)
    b = v.astype("<u8").view(np.uint8).reshape(nvals, 8)[:, :7].reshape(-1)
    return b[:n].tobytes()

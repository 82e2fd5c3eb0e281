"""ORACLE / TEST INFRASTRUCTURE ONLY — ctypes wrapper of oracle/cdc_oracle.c.

Importable only from tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  Loads oracle/_build/liboracle.so (built by ``make -C oracle``).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from functools import lru_cache

import numpy as np

from . import gorand, rollinghash
from .splitter_ref import REGISTRY

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle.so")
KIND = {"fixed": 0, "buzhash": 1, "rabinkarp": 2}
MODES = {"getSplitPoints": 0, "getSplitPointsByteByByte": 1, "getSplitPointsRandomSlices": 2}

_i64p = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")
_u64p = np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS")
_u32p = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


@lru_cache(maxsize=1)
def lib() -> C.CDLL:
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(os.path.join(HERE, "cdc_oracle.c")):
        build()
    L = C.CDLL(LIB)
    L.orc_set_tables.argtypes = [_u32p, _u64p, _u64p, C.c_int]
    L.orc_new.restype = C.c_void_p
    L.orc_new.argtypes = [C.c_int, C.c_int64]
    L.orc_free.argtypes = [C.c_void_p]
    L.orc_reset.argtypes = [C.c_void_p]
    L.orc_next.restype = C.c_int64
    L.orc_next.argtypes = [C.c_void_p, C.c_char_p, C.c_int64]
    L.orc_max_segment.restype = C.c_int64
    L.orc_max_segment.argtypes = [C.c_void_p]
    L.orc_feed.restype = C.c_int64
    L.orc_feed.argtypes = [C.c_void_p, C.c_char_p, C.c_int64, C.c_int, C.c_uint64, _i64p, C.c_int64]
    L.orc_split_stream.restype = C.c_int64
    L.orc_split_stream.argtypes = [C.c_int, C.c_int64, C.c_void_p, C.c_int64, _i64p, C.c_int64]
    L.orc_gorand_read.argtypes = [C.c_int64, _u64p, C.c_void_p, C.c_int64]
    L.orc_gen_stream.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_void_p, C.c_int64]
    L.orc_split_batch.argtypes = [C.c_int, C.c_int64, C.POINTER(C.c_void_p), _i64p, C.c_int64,
                                  _i64p, _i64p, _i64p, _i64p, C.c_int]
    L.orc_split_prng_streams.argtypes = [C.c_int, C.c_int64, C.c_uint64, _u64p, C.c_int64, C.c_int64,
                                         _i64p, _i64p, _i64p, _i64p, C.c_int]
    L.orc_rolled_bytes.restype = C.c_int64
    L.orc_rolled_bytes.argtypes = [C.c_int64, _i64p, C.c_int64]
    out, mod = rollinghash.rabin_tables()
    P, _ = rollinghash.rabin_polynomial()
    L.orc_set_tables(np.ascontiguousarray(rollinghash.buzhash_table()), np.ascontiguousarray(out),
                     np.ascontiguousarray(mod), P.bit_length() - 1 - 8)
    return L


def params(name: str) -> tuple[int, int]:
    kind, size = REGISTRY[name]
    return KIND[kind], size


def min_size(name: str) -> int:
    kind, size = REGISTRY[name]
    return size if kind == "fixed" else size // 2


def cut_capacity(name: str, n: int) -> int:
    """Upper bound on chunks of an n-byte stream: every chunk but the last is >= min."""
    return n // max(min_size(name), 1) + 1


class OracleSplitter:
    """Streaming handle over the C restatement (NextSplitPoint semantics)."""

    def __init__(self, name: str):
        k, size = params(name)
        self._L = lib()
        self._h = self._L.orc_new(k, size)

    def next_split_point(self, b: bytes) -> int:
        return self._L.orc_next(self._h, bytes(b), len(b))

    def max_segment_size(self) -> int:
        return self._L.orc_max_segment(self._h)

    def reset(self):
        self._L.orc_reset(self._h)

    def __del__(self):
        if getattr(self, "_h", None):
            self._L.orc_free(self._h)
            self._h = None


def feed(name: str, data: bytes, mode: str, seed: int = 1) -> np.ndarray:
    """Split points (absolute end offsets) under one of the reference test feeders."""
    kind, size = REGISTRY[name]
    return feed_kind(kind, size, data, mode, seed)


def feed_kind(kind: str, size: int, data: bytes, mode: str, seed: int = 1) -> np.ndarray:
    """As feed() for an unregistered parameterisation (the KAT factories)."""
    k = KIND[kind]
    L = lib()
    h = L.orc_new(k, size)
    try:
        cap = len(data) // max(1, size if kind == "fixed" else size // 2) + 2
        out = np.zeros(cap, dtype=np.int64)
        n = L.orc_feed(h, bytes(data), len(data), MODES[mode], seed, out, cap)
        assert n <= cap
        return out[:n].copy()
    finally:
        L.orc_free(h)


def split_stream(name: str, data) -> np.ndarray:
    """Chunk end offsets of a whole stream, trailing chunk included (last == len)."""
    kind, size = REGISTRY[name]
    return split_stream_kind(kind, size, data)


def split_stream_kind(kind: str, size: int, data) -> np.ndarray:
    """As split_stream() for an unregistered parameterisation (the KAT factories)."""
    k = KIND[kind]
    buf = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    n = buf.size
    cap = n // max(size if kind == "fixed" else size // 2, 1) + 1
    out = np.zeros(max(cap, 1), dtype=np.int64)
    cnt = lib().orc_split_stream(k, size, buf.ctypes.data, n, out, cap)
    assert cnt <= cap
    return out[:cnt].copy()


def split_batch(name: str, streams: list, nthreads: int = 8):
    """Threaded whole-stream split of many host buffers -> list of cut arrays."""
    k, size = params(name)
    arrs = [np.frombuffer(s, dtype=np.uint8) if not isinstance(s, np.ndarray) else s for s in streams]
    lens = np.array([a.size for a in arrs], dtype=np.int64)
    caps = np.array([cut_capacity(name, int(n)) for n in lens], dtype=np.int64)
    base = np.zeros(len(arrs), dtype=np.int64)
    if len(arrs) > 1:
        base[1:] = np.cumsum(caps)[:-1]
    cuts = np.zeros(max(int(caps.sum()), 1), dtype=np.int64)
    counts = np.zeros(len(arrs), dtype=np.int64)
    ptrs = (C.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
    lib().orc_split_batch(k, size, ptrs, lens, len(arrs), cuts, base, caps, counts, nthreads)
    return [cuts[base[i]:base[i] + counts[i]].copy() for i in range(len(arrs))]


def split_prng_streams(name: str, seed: int, sids, stream_len: int, nthreads: int = 8):
    """Generate counter-PRNG streams (same bytes as the GPU generator) and split them."""
    k, size = params(name)
    sids = np.ascontiguousarray(np.asarray(sids, dtype=np.uint64))
    ns = sids.size
    cap = cut_capacity(name, stream_len)
    caps = np.full(ns, cap, dtype=np.int64)
    base = np.arange(ns, dtype=np.int64) * cap
    cuts = np.zeros(max(ns * cap, 1), dtype=np.int64)
    counts = np.zeros(ns, dtype=np.int64)
    lib().orc_split_prng_streams(k, size, seed, sids, ns, stream_len, cuts, base, caps, counts, nthreads)
    return cuts.reshape(ns, cap), counts


def split_prng_stream_blocks(name: str, seed: int, sid: int, stream_len: int, block: int = 256 << 20,
                             gen_threads: int = 8) -> tuple[np.ndarray, float]:
    """One (arbitrarily long) counter-PRNG stream split through the STREAMING oracle
    (NextSplitPoint over successive `block`-byte slices, repo/object/object_writer.go:
    120-136): host memory stays at a few blocks (a 64 GiB stream needs no 64 GiB buffer).
    Blocks are generated ahead on `gen_threads` threads.  Returns (cut end offsets, the
    seconds spent inside NextSplitPoint -- the single-thread split time)."""
    import concurrent.futures as cf
    import time
    k, size = params(name)
    L = lib()
    nxt = L["orc_next"]  # a fresh function object: raw pointer arguments, no bytes copy
    nxt.restype = C.c_int64
    nxt.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
    h = L.orc_new(k, size)
    cuts, split_s = [], 0.0
    try:
        nblk = (stream_len + block - 1) // block
        depth = 2 * gen_threads
        with cf.ThreadPoolExecutor(gen_threads) as ex:
            def gen(j):
                return gen_stream(seed, sid, min(block, stream_len - j * block), offset=j * block)
            futs = {j: ex.submit(gen, j) for j in range(min(depth, nblk))}
            for j in range(nblk):
                buf = futs.pop(j).result()
                if j + depth < nblk:
                    futs[j + depth] = ex.submit(gen, j + depth)
                base, pos, n = j * block, 0, buf.size
                t0 = time.perf_counter()
                while pos < n:
                    r = nxt(h, buf.ctypes.data + pos, n - pos)
                    if r < 0:
                        break
                    pos += r
                    cuts.append(base + pos)
                split_s += time.perf_counter() - t0
    finally:
        L.orc_free(h)
    if not cuts or cuts[-1] < stream_len:
        cuts.append(stream_len)  # the trailing chunk (objectWriter.Result)
    if stream_len == 0:
        cuts = []
    return np.asarray(cuts, dtype=np.int64), split_s


def gen_stream(seed: int, sid: int, n: int, offset: int = 0) -> np.ndarray:
    out = np.empty(n, dtype=np.uint8)
    lib().orc_gen_stream(seed, sid, offset, out.ctypes.data, n)
    return out


def gorand_read(seed: int, n: int) -> np.ndarray:
    out = np.empty(n, dtype=np.uint8)
    lib().orc_gorand_read(seed, np.ascontiguousarray(gorand.rng_cooked()), out.ctypes.data, n)
    return out


def rolled_bytes(name: str, cuts) -> int:
    c = np.ascontiguousarray(np.asarray(cuts, dtype=np.int64))
    return lib().orc_rolled_bytes(min_size(name), c, c.size)

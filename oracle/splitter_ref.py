"""ORACLE / TEST INFRASTRUCTURE ONLY — never imported by the product path.

Pure-Python restatement of Kopia's splitter package for SMALL inputs (the C
oracle ``oracle/cdc_oracle.c`` is the fast twin used at KAT sizes).  Every
method cites the reference line it restates.
"""
from __future__ import annotations

from .rollinghash import WINDOW, Buzhash32, RabinKarp64

KIB = 1 << 10
MIB = 1 << 20

# repo/splitter/splitter.go:50-81 — name -> (kind, size)
_SIZES = {"128K": 128 * KIB, "256K": 256 * KIB, "512K": 512 * KIB, "1M": MIB,
          "2M": 2 * MIB, "4M": 4 * MIB, "8M": 8 * MIB}
REGISTRY: dict[str, tuple[str, int]] = {}
for _k, _v in _SIZES.items():
    REGISTRY[f"FIXED-{_k}"] = ("fixed", _v)
    REGISTRY[f"DYNAMIC-{_k}-BUZHASH"] = ("buzhash", _v)
    REGISTRY[f"DYNAMIC-{_k}-RABINKARP"] = ("rabinkarp", _v)
REGISTRY["FIXED"] = ("fixed", 4 * MIB)          # splitter.go:76
REGISTRY["DYNAMIC"] = ("buzhash", 4 * MIB)      # splitter.go:80
DEFAULT_ALGORITHM = "DYNAMIC-4M-BUZHASH"        # splitter.go:89


def supported_algorithms() -> list[str]:
    return sorted(REGISTRY)  # splitter.go:32-42 (sort.Strings)


class FixedSplitter:
    """repo/splitter/splitter_fixed.go:3-37"""

    def __init__(self, length: int):
        self.chunk_length = length
        self.cur = 0

    def next_split_point(self, b) -> int:  # :15-26
        n = self.chunk_length - self.cur
        if len(b) < n:
            self.cur += len(b)
            return -1
        self.cur = 0
        return n

    def max_segment_size(self) -> int:
        return self.chunk_length

    def reset(self):
        self.cur = 0


class RollingSplitter:
    """repo/splitter/splitter_buzhash32.go:7-86 and splitter_rabinkarp64.go:7-83."""

    def __init__(self, kind: str, avg: int):
        self.kind = kind
        self.rh = Buzhash32() if kind == "buzhash" else RabinKarp64()
        self.mask = avg - 1          # :76 / :74
        self.max_size = 2 * avg
        self.min_size = avg // 2
        self.count = 0

    def _sum(self) -> int:
        return self.rh.sum32() if self.kind == "buzhash" else self.rh.sum64()

    def reset(self):  # :20-24
        self.rh.reset()
        self.count = 0

    def max_segment_size(self) -> int:  # :69-71
        return self.max_size

    def next_split_point(self, b) -> int:  # :26-67
        fast = 0
        left = self.min_size - self.count - 1
        if left > 0:  # :29-40 fast path: roll only the last 64 bytes
            fast = min(left, len(b))
            for i in range(max(fast - WINDOW, 0), fast):
                self.rh.roll(b[i])
            self.count += fast
            b = b[fast:]
        left = self.max_size - self.count
        if left > 0:  # :42-58
            fp = min(left, len(b))
            for i in range(fp):
                self.rh.roll(b[i])
                self.count += 1
                if self._sum() & self.mask == 0:
                    self.count = 0
                    return fast + i + 1
            fast += fp
        if self.count >= self.max_size:  # :60-64
            self.count = 0
            return fast
        return -1


def new_splitter(name: str):
    kind, size = REGISTRY[name]
    return FixedSplitter(size) if kind == "fixed" else RollingSplitter(kind, size)


def split_whole(splitter, data: bytes) -> list[int]:
    """Chunk END offsets for a whole stream, trailing remainder included
    (cli/command_benchmark_splitters.go:88-101 loop shape)."""
    cuts, pos = [], 0
    d = memoryview(data)
    while pos < len(data):
        n = splitter.next_split_point(d[pos:])
        if n < 0:
            cuts.append(len(data))
            break
        pos += n
        cuts.append(pos)
    return cuts


def chunk_rule_cuts(cand, n: int, min_size: int, max_size: int) -> list[int]:
    """SURVEY.md App. A.4 closed form over a candidate predicate cand(p)."""
    cuts, s = [], 0
    while s < n:
        lo, hi = s + min_size - 1, s + max_size - 1
        if lo >= n:
            cuts.append(n)
            break
        p = next((q for q in range(lo, min(hi, n - 1) + 1) if cand(q)), None)
        if p is not None:
            s = p + 1
        elif hi <= n - 1:
            s = hi + 1
        else:
            s = n
        cuts.append(s)
    return cuts

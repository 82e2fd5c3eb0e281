"""``kopia benchmark splitter`` on the GPU (cli/command_benchmark_splitters.go:19-170).

Same flags and defaults (--rand-seed 42, --data-size 32MiB, --block-count 16,
--parallel 1, --print-options), same input (Go ``math/rand`` Read of every block
from one Rand, :66-75), same per-algorithm statistics (count, min, 10th … 90th
percentile, max of the sorted segment lengths, :104-118) and the same two
listings (registry order, then by duration, :120-165).  The blocks are uploaded
once before timing, like the reference generates them before its loop; each
algorithm is one ``kcdc_split_files_device`` call over ``parallel`` copies of the
block list (every goroutine of the reference splits every block, :83-101).

    python -m kopia_amd.benchmark_splitters --data-size 256MiB --block-count 1
"""
from __future__ import annotations

import argparse
import json
import re
import sys
import time

import numpy as np

from . import batch, splitter

_UNITS = {"": 1, "B": 1, "KB": 1 << 10, "KIB": 1 << 10, "MB": 1 << 20, "MIB": 1 << 20, "GB": 1 << 30,
          "GIB": 1 << 30}


def parse_size(s: str) -> int:
    """alecthomas/units Base2Bytes (the --data-size flag type): "32MB" = 32 MiB."""
    m = re.fullmatch(r"\s*(\d+)\s*([A-Za-z]*)\s*", s)
    if not m or m.group(2).upper() not in _UNITS:
        raise ValueError(f"bad size {s!r}")
    return int(m.group(1)) * _UNITS[m.group(2).upper()]


def bytes_string(b: float) -> str:
    """internal/units BytesString: base-10 units, one decimal."""
    for unit, div in (("TB", 1e12), ("GB", 1e9), ("MB", 1e6), ("KB", 1e3)):
        if b >= div:
            return f"{b / div:.1f} {unit}"
    return f"{int(b)} B"


def segment_stats(lengths: np.ndarray) -> dict:
    """:104-118 — sort, then index len*p/100 (integer division)."""
    s = np.sort(np.asarray(lengths, dtype=np.int64))
    n = len(s)
    return {"count": n, "min": int(s[0]), "p10": int(s[n * 10 // 100]), "p25": int(s[n * 25 // 100]),
            "p50": int(s[n * 50 // 100]), "p75": int(s[n * 75 // 100]), "p90": int(s[n * 90 // 100]),
            "max": int(s[-1])}


def lengths_from_cuts(cut_lists) -> np.ndarray:
    """Chunk end offsets per block -> segment lengths, blocks in order (:86-99)."""
    parts = [np.diff(np.concatenate([[0], np.asarray(c, dtype=np.int64)])) for c in cut_lists if len(c)]
    return np.concatenate(parts) if parts else np.zeros(0, dtype=np.int64)


def run(rand_seed: int = 42, data_size: int = 32 << 20, block_count: int = 16, parallel: int = 1,
        names=None, device: int = 0, repeats: int = 1) -> list[dict]:
    import torch
    dev = torch.device("cuda", device)
    host = batch.gorand_read(rand_seed, data_size * block_count)  # one Rand, block after block
    data = torch.from_numpy(host).to(dev)
    base = data.data_ptr()
    ptrs = [base + i * data_size for i in range(block_count)] * parallel
    lens = [data_size] * (block_count * parallel)
    results = []
    for name in names or splitter.SupportedAlgorithms():
        best = None
        for _ in range(max(1, repeats)):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            cuts, counts, cbase, cap = batch.split_files_device(name, ptrs, lens, dev)
            torch.cuda.synchronize(dev)
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        st = segment_stats(lengths_from_cuts(batch.read_files(cuts, counts, cbase, cap)))
        st.update(splitter=name, seconds=best, bytes_per_second=parallel * block_count * data_size / best)
        results.append(st)
    return results


def _line(r: dict) -> str:
    return (f"{r['splitter']:<25} {bytes_string(r['bytes_per_second']):>12}/s count:{r['count']} min:{r['min']} "
            f"10th:{r['p10']} 25th:{r['p25']} 50th:{r['p50']} 75th:{r['p75']} 90th:{r['p90']} max:{r['max']}")


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="Run splitter benchmarks (GPU)")
    ap.add_argument("--rand-seed", type=int, default=42)
    ap.add_argument("--data-size", default="32MB")
    ap.add_argument("--block-count", type=int, default=16)
    ap.add_argument("--print-options", action="store_true")
    ap.add_argument("--parallel", type=int, default=1)
    ap.add_argument("--repeats", type=int, default=3, help="best of N timings per algorithm (reference: 1)")
    ap.add_argument("--json", action="store_true", help="one JSON object per algorithm instead of text")
    a = ap.parse_args(argv)
    size = parse_size(a.data_size)
    print(f"splitting {a.block_count} blocks of {size} each, parallelism {a.parallel}", file=sys.stderr)
    res = run(a.rand_seed, size, a.block_count, a.parallel, repeats=a.repeats)
    if a.json:
        for r in res:
            print(json.dumps(r))
        return 0
    for r in res:
        print(_line(r))
    print("-----------------------------------------------------------------")
    ranked = sorted(res, key=lambda r: r["seconds"])
    for i, r in enumerate(ranked):
        print(f"{i:3}. {_line(r)}")
    if a.print_options:
        best = next((r for r in ranked if not r["splitter"].startswith("FIXED")), None)
        if best:
            print(f"Fastest option for this machine is: --object-splitter={best['splitter']}")
    return 0


if __name__ == "__main__":
    sys.exit(main())

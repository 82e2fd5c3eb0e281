"""Golden statistics of ``kopia benchmark splitter`` (cli/command_benchmark_splitters.go:63-131)
for every registered splitter, computed by the oracle (run from the repo root:
``python tests/golden/make_bench_splitters.py``; about a minute on 8 cores).

Two harness configurations, both with the reference's --rand-seed default 42:
* ``config1``: --data-size 256MiB --block-count 1;
* ``default``: the command's own defaults, --data-size 32MB (= 32 MiB, Base2Bytes)
  --block-count 16 (blocks read one after another from one Rand).
Statistics restate :104-118: sort the segment lengths, count, min, s[n*p/100] for
p = 10, 25, 50, 75, 90, max.  The oracle is pinned by the reference KAT table
(tests/test_oracle.py); the reference itself cannot run here (no Go toolchain)."""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import coracle  # noqa: E402
from oracle.splitter_ref import supported_algorithms  # noqa: E402

CONFIGS = {"config1": (42, 256 << 20, 1), "default": (42, 32 << 20, 16)}


def stats(lengths) -> dict:
    s = np.sort(np.asarray(lengths, dtype=np.int64))
    n = len(s)
    return {"count": n, "min": int(s[0]), "p10": int(s[n * 10 // 100]), "p25": int(s[n * 25 // 100]),
            "p50": int(s[n * 50 // 100]), "p75": int(s[n * 75 // 100]), "p90": int(s[n * 90 // 100]),
            "max": int(s[-1])}


def main():
    out = {}
    for key, (seed, size, count) in CONFIGS.items():
        data = coracle.gorand_read(seed, size * count)
        blocks = [data[i * size:(i + 1) * size] for i in range(count)]
        rows = {}
        for name in supported_algorithms():
            cut_lists = coracle.split_batch(name, blocks, nthreads=8)
            lens = np.concatenate([np.diff(np.concatenate([[0], np.asarray(c, dtype=np.int64)])) for c in cut_lists])
            assert int(lens.sum()) == size * count
            rows[name] = stats(lens)
            print(key, name, rows[name], flush=True)
        out[key] = {"rand_seed": seed, "data_size": size, "block_count": count, "stats": rows}
    json.dump(out, open(os.path.join(HERE, "bench_splitters.json"), "w"), indent=1)


if __name__ == "__main__":
    main()

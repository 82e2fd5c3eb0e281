"""Multi-GPU host logic: one process per GPU, streams sharded with no data-path
collective.  The only collectives are the timing barrier and the
max-over-ranks of elapsed time, over gloo (CPU); no RCCL.

* Static sharding (configs 2 and 4): rank r owns stream ids [r*per, (r+1)*per).
* LPT balancing (config 5, Zipf file sizes): streams sorted by size descending,
  each assigned to the currently least-loaded rank (bytes), ties to the lowest
  rank — deterministic, so every rank computes the same plan independently.
"""
from __future__ import annotations

import heapq
import os

import numpy as np


def env_rank_world() -> tuple[int, int, int]:
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def static_shard(rank: int, world: int, per_rank: int) -> np.ndarray:
    """Stream ids owned by `rank` under weak scaling (per_rank streams each)."""
    return np.arange(rank * per_rank, (rank + 1) * per_rank, dtype=np.uint64)


def lpt_plan(sizes, world: int) -> list[list[int]]:
    """Longest-processing-time-first assignment of stream indices to ranks by bytes."""
    order = sorted(range(len(sizes)), key=lambda i: (-int(sizes[i]), i))
    heap = [(0, r) for r in range(world)]
    plan: list[list[int]] = [[] for _ in range(world)]
    for i in order:
        load, r = heapq.heappop(heap)
        plan[r].append(i)
        heapq.heappush(heap, (load + int(sizes[i]), r))
    return plan


def zipf_sizes(total_bytes: int, seed: int = 0x5A1F, s: float = 1.1, classes: int = 19,
               base: int = 4096) -> np.ndarray:
    """BASELINE.json configs[4] / SURVEY.md §8d: file sizes from a Zipf law over size
    classes base*2^j (j = 0..classes-1, 4 KiB .. 1 GiB), exponent s, fixed seed,
    drawn until the total reaches `total_bytes`."""
    rng = np.random.default_rng(seed)
    w = 1.0 / np.arange(1, classes + 1) ** s
    w /= w.sum()
    out = []
    acc = 0
    while acc < total_bytes:
        j = int(rng.choice(classes, p=w))
        sz = base << j
        out.append(sz)
        acc += sz
    return np.array(out, dtype=np.int64)


def max_over_ranks(value: float, device=None) -> float:
    """All-reduce MAX of a scalar (the bench's elapsed time) over the CPU (gloo) process
    group; identity when not distributed.  `device` is unused (kept for callers)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())

"""N>1 host path on CPU: world_size-2 gloo ranks shard streams with no data-path
collective, each splits its shard (the C oracle stands in for the device here),
and the union of the shards' cut lists equals a single-process run; timing
aggregation is max-over-ranks."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from kopia_amd import dist as kd

SEED = 0x6B6F706961


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, per, L, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import coracle
    ids = kd.static_shard(rank, world, per)
    cuts, counts = coracle.split_prng_streams("DYNAMIC-128K-BUZHASH", SEED, ids, L, nthreads=1)
    elapsed = kd.max_over_ranks(float(rank + 1))
    out[rank] = {"ids": ids.tolist(), "cuts": [cuts[i, :counts[i]].tolist() for i in range(len(ids))],
                 "elapsed": elapsed}
    dist.barrier()
    dist.destroy_process_group()


def test_static_sharding_gloo_world2():
    world, per, L = 2, 6, 1 << 20
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_worker, args=(world, _free_port(), per, L, out), nprocs=world, join=True,
                       start_method="spawn")
    ids = sorted(i for r in range(world) for i in out[r]["ids"])
    assert ids == list(range(world * per))  # disjoint and complete
    assert all(out[r]["elapsed"] == float(world) for r in range(world))  # max over ranks
    from oracle import coracle
    cuts, counts = coracle.split_prng_streams("DYNAMIC-128K-BUZHASH", SEED, np.arange(world * per), L)
    for r in range(world):
        for k, sid in enumerate(out[r]["ids"]):
            assert out[r]["cuts"][k] == cuts[sid, :counts[sid]].tolist()


def test_lpt_plan_balanced_and_deterministic():
    sizes = kd.zipf_sizes(64 << 30)
    assert sizes.min() >= 4096 and sizes.max() <= (1 << 30)
    for world in (1, 2, 4, 8):
        plan = kd.lpt_plan(sizes, world)
        assert sorted(i for p in plan for i in p) == list(range(len(sizes)))
        loads = [int(sizes[p].sum()) if p else 0 for p in plan]
        # LPT bound: max load <= OPT + largest item <= avg + largest
        assert max(loads) <= sum(loads) / world + sizes.max()
        assert plan == kd.lpt_plan(sizes, world)


def test_max_over_ranks_single_process():
    assert kd.max_over_ranks(3.5) == 3.5


def test_library_lpt_assign_matches_lpt_plan():
    """The library's kcdc_lpt_assign (the device-set host path, kcdc_split_batch_host_devices)
    makes the same assignment as kd.lpt_plan (bench.py's rank plan)."""
    from kopia_amd import batch
    rng = np.random.default_rng(8)
    for world in (1, 2, 3, 8):
        sizes = kd.zipf_sizes(64 << 30, seed=world)
        sizes[::7] = sizes[1]  # ties
        plan = kd.lpt_plan(sizes, world)
        got = batch.lpt_assign(sizes, world)
        want = np.zeros(len(sizes), np.uint32)
        for r, idx in enumerate(plan):
            want[idx] = r
        assert (got == want).all(), world
        sizes2 = rng.integers(0, 1 << 30, 500)
        plan2 = kd.lpt_plan(sizes2, world)
        want2 = np.zeros(500, np.uint32)
        for r, idx in enumerate(plan2):
            want2[idx] = r
        assert (batch.lpt_assign(sizes2, world) == want2).all()

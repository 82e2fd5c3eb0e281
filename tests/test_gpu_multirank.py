"""GPU: the multi-rank path with each rank driving libkcdc on a device.

bench.spawn_ranks starts two rank processes (as `bench.py --gpus 2` does; the reference's
`--parallel` harness is cli/command_benchmark.go:67-82).  Each rank takes the device
LOCAL_RANK % device_count (both share the one GPU of a test box), splits its disjoint static
shard of config-2-shaped streams through the batch kernel, and computes the config-5 LPT plan
independently; results come back over gloo (no RCCL, no data-path collective).  Every stream's
cuts must equal the oracle's, the shards must be disjoint and complete, and every rank must
hold the same LPT plan."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from kopia_amd import dist as kd
from oracle import coracle

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SEED = 0x6B6F706961


@pytest.mark.parametrize("name", ["DYNAMIC-4M-BUZHASH", "DYNAMIC-1M-RABINKARP"])
def test_two_ranks_split_their_shards(tmp_path, name):
    out = tmp_path / "ranks.json"
    world, per, mib = 2, 24, 4
    # a child process (it never touches the GPU) spawns the rank processes
    code = (f"import sys; sys.path.insert(0, {ROOT!r}); import bench; "
            f"bench.spawn_ranks({world}, [{str(out)!r}, '{per}', '{mib}', {name!r}], entry='multirank_check')")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    subprocess.run([sys.executable, "-c", code], check=True, timeout=300, env=env, cwd=ROOT)
    ranks = json.load(open(out))
    assert [r["rank"] for r in ranks] == list(range(world))
    ids = sorted(i for r in ranks for i in r["ids"])
    assert ids == list(range(world * per))  # disjoint and complete
    assert len({r["plan"] for r in ranks}) == 1  # the same LPT plan on every rank
    plan = kd.lpt_plan(kd.zipf_sizes(1 << 36), world)
    assert [r["mine"] for r in ranks] == [len(p) for p in plan]
    cuts, counts = coracle.split_prng_streams(name, SEED, np.arange(world * per), mib << 20, nthreads=8)
    for r in ranks:
        for k, sid in enumerate(r["ids"]):
            assert r["cuts"][k] == cuts[sid, :counts[sid]].tolist(), f"rank {r['rank']} stream {sid}"

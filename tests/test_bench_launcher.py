"""bench.py's own multi-process launcher (`--gpus N` without torchrun): N spawned rank
processes, gloo barrier / max / gather (no RCCL), whole-job aggregation.  CPU only: the
ranks report made-up timings through bench.launcher_selftest."""
import json

import bench


def test_aggregate_weak_scaling():
    per = [{"bytes_per_step": 1 << 30, "elapsed_s": 2.0, "own_s": 1.0},
           {"bytes_per_step": 1 << 30, "elapsed_s": 4.0, "own_s": 2.0}]
    a = bench.aggregate(per, 4)
    assert a["value"] == 2.0  # 8 GiB over the slowest rank's 4 s
    assert a["ms_per_step"] == 1000.0
    assert a["per_gpu_gib_s"] == [4.0, 2.0]


def test_spawn_gloo_world2(tmp_path):
    out = tmp_path / "agg.json"
    bench.spawn_ranks(2, [str(out)], entry="launcher_selftest")
    d = json.loads(out.read_text())
    assert d["world"] == 2
    assert d["max"] == 1.0
    # (1 + 2) GiB per step x 2 steps over max elapsed 2 s
    assert d["agg"]["value"] == 3.0
    assert d["agg"]["per_gpu_gib_s"] == [4.0, round(2 * 2 / 1.5, 3)]


def test_parse_config4_shape():
    a = bench.parse(["--config", "4", "--gpus", "8"])
    assert (a.streams, a.stream_mib, a.gpus) == (8192, 8, 8)


def test_host_cpu_info():
    info = bench.host_cpu_info()
    assert info["logical_cores"] >= 1 and 1 <= info["threads_all"] <= info["logical_cores"]

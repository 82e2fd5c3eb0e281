"""`kopia benchmark splitter` harness (kopia_amd/benchmark_splitters.py) and the
library's Go math/rand reader: host-side pieces (no GPU)."""
import hashlib

import numpy as np
import pytest

from conftest import golden
from kopia_amd import batch
from kopia_amd import benchmark_splitters as kb
from oracle import coracle

CHECK = golden("check_values.json")


def test_gorand_read_matches_oracle_and_check_values():
    """kcdc_gorand_read = rand.New(rand.NewSource(seed)).Read (SURVEY App. A digests)."""
    assert hashlib.sha256(batch.gorand_read(42, 1 << 20).tobytes()).hexdigest() == CHECK["seed42_read1MiB_sha256"]
    assert hashlib.sha256(batch.gorand_read(5, 5_000_000).tobytes()).hexdigest() == CHECK["seed5_read5e6_sha256"]
    for seed, n in [(1, 0), (1, 1), (7, 13), (-3, 1000), (0, 777)]:
        assert batch.gorand_read(seed, n).tobytes() == coracle.gorand_read(seed, n).tobytes()


def test_consecutive_blocks_are_one_read():
    """:66-75 reads block after block from ONE Rand (7-byte Int63 remainders carry over)."""
    whole = batch.gorand_read(42, 3 * 1000)
    assert whole.tobytes() == coracle.gorand_read(42, 3000).tobytes()


def test_parse_size_base2():
    assert kb.parse_size("32MB") == 32 << 20  # alecthomas/units Base2Bytes
    assert kb.parse_size("256MiB") == 256 << 20
    assert kb.parse_size("4KB") == 4096
    assert kb.parse_size("100") == 100
    with pytest.raises(ValueError):
        kb.parse_size("12XB")


def test_segment_stats_indexing():
    """:104-118 index the sorted list at len*p/100 with integer division."""
    lens = np.array([9, 1, 8, 2, 7, 3, 6, 4, 5, 10, 11])
    st = kb.segment_stats(lens)
    s = np.sort(lens)
    assert st == {"count": 11, "min": 1, "p10": int(s[1]), "p25": int(s[2]), "p50": int(s[5]), "p75": int(s[8]),
                  "p90": int(s[9]), "max": 11}


def test_lengths_from_cuts_and_golden_consistency():
    g = golden("bench_splitters.json")
    for key, cfg in g.items():
        total = cfg["data_size"] * cfg["block_count"]
        for name, st in cfg["stats"].items():
            assert st["min"] <= st["p10"] <= st["p25"] <= st["p50"] <= st["p75"] <= st["p90"] <= st["max"]
            assert st["count"] * st["min"] <= total <= st["count"] * st["max"], (key, name)
    cuts = [np.array([3, 10]), np.array([]), np.array([5])]
    assert kb.lengths_from_cuts(cuts).tolist() == [3, 7, 5]


def test_golden_config1_small_names_match_oracle():
    """Spot-check the committed fixture against the oracle on one dynamic name."""
    g = golden("bench_splitters.json")["config1"]
    data = coracle.gorand_read(42, g["data_size"])
    for name in ["DYNAMIC-8M-BUZHASH", "FIXED-4M"]:
        cuts = coracle.split_stream(name, data)
        lens = np.diff(np.concatenate([[0], cuts]))
        assert kb.segment_stats(lens) == g["stats"][name]

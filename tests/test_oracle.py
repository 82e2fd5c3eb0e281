"""The oracle is pinned before it is trusted (CPU only).

Pins: the reference's own TestSplitterStability table
(repo/splitter/splitter_test.go:27-52), Go math/rand check values, rollinghash
table check values and the object-writer FIXED pins
(repo/object/object_manager_test.go:216-264).
"""
import hashlib

import numpy as np
import pytest

from conftest import golden
from oracle import coracle, gorand, rollinghash
from oracle import splitter_ref as ref

CHECK = golden("check_values.json")


def test_rng_cooked_regenerated():
    c = gorand.rng_cooked().view(np.int64)
    assert c[:3].tolist() == CHECK["rng_cooked_first3"]
    assert int(c[606]) == CHECK["rng_cooked_606"]
    assert gorand.rng_cooked_sha256() == CHECK["rng_cooked_sha256"]


def test_go_rand_known_outputs():
    r = gorand.GoRandSource(1)
    assert [r.int63() for _ in range(4)] == CHECK["seed1_int63"]
    assert hashlib.sha256(gorand.read_bytes(5, 5_000_000)).hexdigest() == CHECK["seed5_read5e6_sha256"]
    assert hashlib.sha256(gorand.read_bytes(42, 1 << 20)).hexdigest() == CHECK["seed42_read1MiB_sha256"]


def test_c_go_rand_matches_python():
    assert coracle.gorand_read(42, 1 << 20).tobytes() == gorand.read_bytes(42, 1 << 20)
    r = gorand.GoRandSource(5)  # Read state carried across calls (rand.go read)
    a = r.read(3) + r.read(10) + r.read(1000)
    assert a == gorand.read_bytes(5, 1013)


def test_rollinghash_tables():
    T = rollinghash.buzhash_table()
    assert [f"{int(x):08x}" for x in T[:4]] == CHECK["buzhash_first4"]
    assert f"{int(T[255]):08x}" == CHECK["buzhash_255"]
    assert rollinghash.buzhash_table_sha256() == CHECK["buzhash_sha256"]
    assert len(set(T.tolist())) == 256
    P, tries = rollinghash.rabin_polynomial()
    assert hex(P) == CHECK["rabin_pol"] and tries == CHECK["rabin_tries"]
    out, mod = rollinghash.rabin_tables()
    assert hex(int(out[1])) == CHECK["rabin_out1"]
    g = golden("tables.json")
    assert g["buzhash"] == [f"{int(x):08x}" for x in T]
    assert g["rabin_out"] == [f"{int(x):016x}" for x in out]
    assert g["rabin_mod"] == [f"{int(x):016x}" for x in mod]


def test_rolling_hash_equals_window_hash():
    """The identity the GPU design rests on: Roll state == hash of
    the last 64 bytes, zeros before the start; zero window hashes to 0."""
    rng = np.random.default_rng(1)
    data = rng.integers(0, 256, 300, dtype=np.uint8).tobytes()
    bz, rk = rollinghash.Buzhash32(), rollinghash.RabinKarp64()
    T = [int(x) for x in rollinghash.buzhash_table()]
    for p, c in enumerate(data):
        bz.roll(c)
        rk.roll(c)
        win = (bytes(64) + data[:p + 1])[-64:]
        direct = 0
        for k in range(64):
            direct ^= rollinghash.rotl32(T[win[63 - k]], k & 31)
        assert bz.sum32() == direct
        assert rk.sum64() == rollinghash.rabin_direct(win)


KAT = golden("kat_stability.json")["kat"]


def _name(kind, size):
    return (kind, size)


@pytest.mark.parametrize("row", KAT, ids=lambda r: f"{r[0]}-{r[1]}{'-pooled' if r[6] else ''}")
@pytest.mark.parametrize("mode", list(coracle.MODES))
def test_kat_stability_c_oracle(kat_data, row, mode):
    """repo/splitter/splitter_test.go:73-115 against the C restatement, 2 repeats
    through one reset splitter (reset-on-reuse)."""
    kind, size, count, avg, mn, mx, _pooled = row
    L = coracle.lib()
    h = L.orc_new(coracle.KIND[kind], size)
    try:
        for rep in range(2):
            assert L.orc_max_segment(h) == mx
            cap = len(kat_data) // max(1, (size if kind == "fixed" else size // 2)) + 2
            out = np.zeros(cap, dtype=np.int64)
            n = L.orc_feed(h, kat_data, len(kat_data), coracle.MODES[mode], 11 + rep, out, cap)
            lens = np.diff(np.concatenate(([0], out[:n])))
            assert (n, len(kat_data) // n, int(lens.min()), int(lens.max())) == (count, avg, mn, mx)
            L.orc_reset(h)
    finally:
        L.orc_free(h)


@pytest.mark.parametrize("kind,avg", [("buzhash", 32), ("buzhash", 1024), ("rabinkarp", 32), ("rabinkarp", 1024)])
def test_python_restatement_matches_c(kat_data, kind, avg):
    d = kat_data[:60000]
    s = ref.RollingSplitter(kind, avg)
    py = ref.split_whole(s, d)
    L = coracle.lib()
    h = L.orc_new(coracle.KIND[kind], avg)
    out = np.zeros(len(d) // (avg // 2) + 2, dtype=np.int64)
    n = L.orc_feed(h, d, len(d), 0, 0, out, out.size)
    L.orc_free(h)
    c = out[:n].tolist()
    if not c or c[-1] != len(d):
        c.append(len(d))
    assert py == c


@pytest.mark.parametrize("kind,avg", [("buzhash", 32), ("rabinkarp", 64), ("buzhash", 256)])
def test_chunk_rule_closed_form(kat_data, kind, avg):
    """Cuts == closed-form rule over cand(p) = hash(window ending at p) & mask == 0."""
    d = kat_data[:20000]
    h = rollinghash.Buzhash32() if kind == "buzhash" else rollinghash.RabinKarp64()
    cand = []
    for c in d:
        h.roll(c)
        cand.append(((h.sum32() if kind == "buzhash" else h.sum64()) & (avg - 1)) == 0)
    want = ref.chunk_rule_cuts(lambda p: cand[p], len(d), avg // 2, 2 * avg)
    assert ref.split_whole(ref.RollingSplitter(kind, avg), d) == want


def test_fixed_object_writer_pins():
    data = np.tile(np.arange(1, 12, dtype=np.uint8), 128 << 10)
    for name, want in CHECK["fixed_object_lengths"].items():
        cuts = coracle.split_stream(name, data)
        assert np.diff(np.concatenate(([0], cuts))).tolist() == want


def test_registry_names():
    names = ref.supported_algorithms()
    assert len(names) == 23 and ref.DEFAULT_ALGORITHM == "DYNAMIC-4M-BUZHASH"
    assert names == sorted(names)


def test_golden_cut_lists_regression(kat_data):
    g = golden("cuts_kat_input.json")["cuts"]
    for name, cuts in g.items():
        assert coracle.split_stream(name, kat_data).tolist() == cuts, name


def test_rolled_bytes_formula():
    # one chunk of len e-s: rolled = len - max(min(min-1, len) - 64, 0)
    name = "DYNAMIC-128K-BUZHASH"
    mn = 64 << 10
    assert coracle.rolled_bytes(name, [10]) == 10
    assert coracle.rolled_bytes(name, [mn]) == mn - (mn - 1 - 64)
    assert coracle.rolled_bytes(name, [3 * mn]) == 3 * mn - (mn - 1 - 64)

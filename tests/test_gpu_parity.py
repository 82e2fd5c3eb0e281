"""GPU parity: the HIP kernels behind libkcdc.so vs the oracle, bit-exact.

Mirrors repo/splitter/splitter_test.go (KAT rows, three feeding modes, reuse
through the pool) and adds the batch hot path on BASELINE.json's shapes."""
import ctypes as C

import numpy as np
import pytest

from conftest import golden
from kopia_amd import _lib, batch
from kopia_amd import splitter as ks
from oracle import coracle
from oracle import splitter_ref as ref

pytestmark = pytest.mark.gpu
SEED = 0x6B6F706961
KAT = golden("kat_stability.json")["kat"]


def kat_name(kind, size):
    return ks.custom_algorithm(kind, size)


def oracle_cuts(kind, size, data):
    L = coracle.lib()
    cap = len(data) // max(1, (size if kind == "fixed" else size // 2)) + 2
    out = np.zeros(cap, dtype=np.int64)
    n = L.orc_split_stream(coracle.KIND[kind], size, np.frombuffer(data, np.uint8).ctypes.data, len(data), out, cap)
    return out[:n]


def stats(cuts_abs, n):
    """(count, avg, min, max) as splitter_test.go computes them (split points only)."""
    pts = [c for c in cuts_abs if c <= n]
    lens = np.diff(np.concatenate(([0], pts)))
    return len(pts), n // len(pts), int(lens.min()), int(lens.max())


# ------------------------------------------------------------------ KAT rows
@pytest.mark.parametrize("row", KAT, ids=lambda r: f"{r[0]}-{r[1]}{'-pooled' if r[6] else ''}")
def test_kat_batch(gpu, kat_data, row):
    """TestSplitterStability rows (splitter_test.go:27-52) through the batch hot path."""
    kind, size, count, avg, mn, mx, _ = row
    got = batch.split_batch_host(kat_name(kind, size), [kat_data])[0]
    np.testing.assert_array_equal(got, oracle_cuts(kind, size, kat_data))
    # split points are the cuts NextSplitPoint returns: all but a trailing remainder
    points = coracle.feed_kind(kind, size, kat_data, "getSplitPoints")
    np.testing.assert_array_equal(got[:len(points)], points)
    assert stats(got[:len(points)], len(kat_data)) == (count, avg, mn, mx)


def _feed(s, data, mode, rng):
    cuts, i, n = [], 0, len(data)
    mv = memoryview(data)
    if mode == "getSplitPoints":
        while i < n:
            k = s.NextSplitPoint(mv[i:])
            if k < 0:
                break
            i += k
            cuts.append(i)
    elif mode == "getSplitPointsByteByByte":
        for i in range(n):
            if s.NextSplitPoint(mv[i:i + 1]) != -1:
                cuts.append(i + 1)
    else:
        while i < n:
            num = min(int(rng.integers(1, 1001)), n - i)
            k = s.NextSplitPoint(mv[i:i + num])
            if k == -1:
                i += num
                continue
            i += k
            cuts.append(i)
    return cuts


@pytest.mark.parametrize("row", [r for r in KAT if not r[6] and r[0] != "fixed"],
                         ids=lambda r: f"{r[0]}-{r[1]}")
@pytest.mark.parametrize("mode", ["getSplitPoints", "getSplitPointsRandomSlices", "getSplitPointsByteByByte"])
def test_kat_streaming_handle(gpu, kat_data, row, mode):
    """NextSplitPoint through the C ABI handle under the reference's three feeders,
    2 repeats per factory (splitter_test.go:55-56,67-71,109-110)."""
    kind, size, count, avg, mn, mx, _ = row
    # byte-by-byte costs one GPU call per tested byte: check a prefix against the oracle
    data = kat_data if mode != "getSplitPointsByteByByte" else kat_data[:12000 if size <= 2048 else 200000]
    want = coracle.feed_kind(kind, size, data, "getSplitPoints").tolist()
    rng = np.random.default_rng(size)
    fac = ks.GetFactory(kat_name(kind, size))
    for _ in range(2):
        s = fac()
        assert s.MaxSegmentSize() == mx
        assert _feed(s, data, mode, rng) == want
        s.Close()
    if data is kat_data:
        assert stats(want, len(data)) == (count, avg, mn, mx)


def test_pooled_reuse_is_reset(gpu, kat_data):
    """Close() returns a Reset splitter to the pool (splitter_pool.go:18-22): one
    abandoned mid-chunk must not leak state into the next object."""
    name = "DYNAMIC-128K-BUZHASH"
    s = ks.GetFactory(name)()
    assert s.NextSplitPoint(kat_data[:70000]) == -1 or True  # leaves count/window mid-chunk
    s.Close()
    s2 = ks.GetFactory(name)()
    got = _feed(s2, kat_data, "getSplitPoints", None)
    s2.Close()
    assert got == coracle.feed(name, kat_data, "getSplitPoints").tolist()


# --------------------------------------------------------- registered names
@pytest.mark.parametrize("name", ref.supported_algorithms())
def test_all_names_on_kat_input(gpu, kat_data, name):
    got = batch.split_batch_host(name, [kat_data])[0]
    assert got.tolist() == golden("cuts_kat_input.json")["cuts"][name]


def _materialize(kind, n):
    if kind == "prng":
        return coracle.gen_stream(SEED, 7, n)
    if kind == "zeros":
        return np.zeros(n, dtype=np.uint8)
    return np.tile(np.arange(1, 12, dtype=np.uint8), n // 11 + 1)[:n]


def test_edge_inputs(gpu):
    g = golden("cuts_edge.json")["cases"]
    for key, case in g.items():
        d = _materialize(case["kind"], case["len"])
        for name, want in case["cuts"].items():
            got = batch.split_batch_host(name, [d])[0]
            assert got.tolist() == want, (key, name)


def test_edge_inputs_streaming(gpu):
    g = golden("cuts_edge.json")["cases"]
    for key, case in g.items():
        d = _materialize(case["kind"], case["len"]).tobytes()
        for name, want in case["cuts"].items():
            s = ks.GetFactory(name)()
            got = _feed(s, d, "getSplitPointsRandomSlices", np.random.default_rng(3))
            s.Close()
            assert got == coracle.feed(name, d, "getSplitPoints").tolist(), (key, name)
            assert want[:len(got)] == got


@pytest.mark.parametrize("name", [n for n in ref.supported_algorithms()])
def test_random_batch_parity(gpu, name):
    """Many streams of ragged lengths (0 .. 3*max) in one launch, every name."""
    import torch
    rng = np.random.default_rng(abs(hash(name)) % (1 << 32))
    info = ks.lookup(name)
    mx = info.max_size
    lens = [0, 1, 63, 64, int(info.min_size) - 1, int(info.min_size), int(mx), int(mx) + 1]
    lens += [int(x) for x in rng.integers(0, 3 * mx, 24)]
    streams = [coracle.gen_stream(SEED, 100 + i, L) for i, L in enumerate(lens)]
    # device layout with deliberately misaligned starts
    offs, pos = [], 0
    for i, L in enumerate(lens):
        pos += (i * 7) % 16
        offs.append(pos)
        pos += L + 64
    buf = np.zeros(pos + 64, dtype=np.uint8)
    for o, s in zip(offs, streams):
        buf[o:o + s.size] = s
    dbuf = torch.from_numpy(buf).to(gpu)
    b = batch.make_device_batch(name, [dbuf.data_ptr() + o for o in offs], lens, gpu)
    batch.split_batch_device(name, b)
    torch.cuda.synchronize()
    got = batch.read_cuts(b)
    want = coracle.split_batch(name, streams)
    for i in range(len(lens)):
        np.testing.assert_array_equal(got[i], want[i], err_msg=f"{name} stream {i} len {lens[i]}")


def test_zero_runs_and_dense_candidates(gpu):
    """All-zero windows hash to 0 for both hashes: every position is a candidate."""
    for name in ["DYNAMIC-128K-BUZHASH", "DYNAMIC-128K-RABINKARP", "DYNAMIC-4M-BUZHASH"]:
        d = np.zeros(20 << 20, dtype=np.uint8)
        d[5 << 20:(5 << 20) + 1000] = 7  # a non-zero island
        got = batch.split_batch_host(name, [d])[0]
        np.testing.assert_array_equal(got, coracle.split_stream(name, d))


# ------------------------------------------------ config 2 (bench workload)
@pytest.mark.parametrize("name", ["DYNAMIC-4M-BUZHASH", "DYNAMIC-4M-RABINKARP", "DYNAMIC-128K-RABINKARP"])
def test_config2_full_parity(gpu, name):
    """BASELINE configs[1]: 4096 x 4 MiB counter-PRNG streams (the default splitter, and the
    Rabin-Karp kernel at two averages), every stream's cut list bit-exact vs the oracle
    (threaded C restatement)."""
    import torch
    ns, L = 4096, 4 << 20
    data = torch.empty(ns * L, dtype=torch.uint8, device=gpu)
    batch.fill_prng(data, L, ns, L, SEED, 0)
    b = batch.make_device_batch(name, [data.data_ptr() + i * L for i in range(ns)], [L] * ns, gpu)
    batch.split_batch_device(name, b)
    torch.cuda.synchronize()
    got = batch.read_cuts(b)
    # spot-check the device generator against the oracle's generator
    for sid in (0, 1234, 4095):
        assert data[sid * L:sid * L + 4096].cpu().numpy().tobytes() == coracle.gen_stream(SEED, sid, 4096).tobytes()
    cuts, counts = coracle.split_prng_streams(name, SEED, np.arange(ns), L, nthreads=16)
    for i in range(ns):
        assert got[i].tolist() == cuts[i, :counts[i]].tolist(), f"stream {i}"

"""GPU: the mixed-size entry point (kcdc_split_files_device, config 5 shapes) and the
`kopia benchmark splitter` harness against the golden statistics, bit-exact."""
import numpy as np
import pytest
import torch

from conftest import golden
from kopia_amd import batch
from kopia_amd import benchmark_splitters as kb
from kopia_amd import dist as kd
from kopia_amd import splitter as ks
from oracle import coracle

pytestmark = pytest.mark.gpu
SEED = 0x6B6F706961


def _arena(sizes, sid0=0):
    """Streams laid out back to back at 1-byte-misaligned offsets, counter-PRNG bytes."""
    offs, o = [], 3
    for L in sizes:
        offs.append(o)
        o += int(L) + 5
    host = np.zeros(o, dtype=np.uint8)
    for i, (L, off) in enumerate(zip(sizes, offs)):
        host[off:off + L] = coracle.gen_stream(SEED, sid0 + i, int(L))
    return host, offs


@pytest.mark.parametrize("name", ["DYNAMIC-4M-BUZHASH", "DYNAMIC-1M-RABINKARP", "DYNAMIC-128K-BUZHASH",
                                  "FIXED-1M"])
def test_files_mixed_sizes_match_oracle(name):
    """Zipf-like mix: tiny files, a batch of mid-size ones and a few large ones that
    route to the long path; every stream's cuts equal the oracle's."""
    rng = np.random.default_rng(11)
    sizes = [0, 1, 63, 64, 4096, 65537] + list(rng.integers(1, 3 << 20, 40)) + [40 << 20, 96 << 20 | 7]
    host, offs = _arena(sizes)
    dev = torch.device("cuda", 0)
    d = torch.from_numpy(host).to(dev)
    ptrs = [d.data_ptr() + o for o in offs]
    cuts, counts, base, cap = batch.split_files_device(name, ptrs, sizes, dev)
    got = batch.read_files(cuts, counts, base, cap)
    want = coracle.split_batch(name, [host[o:o + L] for o, L in zip(offs, sizes)], nthreads=8)
    for i, (g, w) in enumerate(zip(got, want)):
        assert np.array_equal(g, np.asarray(w, dtype=np.int64)), (name, i, sizes[i])


def test_files_zipf_every_name():
    """Config 5 in miniature: Zipf sizes over the 19 classes (capped at 64 MiB here), every
    registered name, one rank of an LPT plan over 8; full parity."""
    sizes = kd.zipf_sizes(256 << 20, classes=15)
    plan = kd.lpt_plan(sizes, 8)
    mine = [int(sizes[i]) for i in plan[0]]
    host, offs = _arena(mine, sid0=100)
    dev = torch.device("cuda", 0)
    d = torch.from_numpy(host).to(dev)
    ptrs = [d.data_ptr() + o for o in offs]
    streams = [host[o:o + L] for o, L in zip(offs, mine)]
    for name in ks.SupportedAlgorithms():
        cuts, counts, base, cap = batch.split_files_device(name, ptrs, mine, dev)
        got = batch.read_files(cuts, counts, base, cap)
        want = coracle.split_batch(name, streams, nthreads=8)
        for i, (g, w) in enumerate(zip(got, want)):
            assert np.array_equal(g, np.asarray(w, dtype=np.int64)), (name, i, mine[i])


@pytest.mark.parametrize("key", ["config1", "default"])
def test_benchmark_splitter_stats_match_golden(key):
    """`kopia benchmark splitter` statistics for all 23 names (golden: oracle, seed 42)."""
    g = golden("bench_splitters.json")[key]
    res = kb.run(g["rand_seed"], g["data_size"], g["block_count"])
    assert [r["splitter"] for r in res] == ks.SupportedAlgorithms()
    for r in res:
        want = g["stats"][r["splitter"]]
        got = {k: r[k] for k in want}
        assert got == want, r["splitter"]
        assert r["bytes_per_second"] > 0


def test_host_batch_routes_large_streams():
    """kcdc_split_batch_host goes through the same router: a 100 MiB stream next to small ones
    (the long path) and a batch of mid-size ones, all equal to the oracle."""
    name = "DYNAMIC-1M-BUZHASH"
    sizes = [100 << 20, 1024, 3 << 20, 0, 5 << 20 | 3]
    streams = [coracle.gen_stream(SEED, 700 + i, L) for i, L in enumerate(sizes)]
    got = batch.split_batch_host(name, streams)
    want = coracle.split_batch(name, streams, nthreads=8)
    for i, (g, w) in enumerate(zip(got, want)):
        assert np.array_equal(g, np.asarray(w, dtype=np.int64)), (i, sizes[i])


def test_host_batch_adjacent_runs():
    """kcdc_split_batch_host copies streams that are adjacent in host memory as one run (the
    device keeps their relative layout, so odd offsets inside a run): views of one buffer
    with and without gaps, empty views among them, groups larger than one 256 MiB arena."""
    name = "DYNAMIC-1M-BUZHASH"
    rng = np.random.default_rng(5)
    buf = coracle.gen_stream(SEED, 4242, 600 << 20)
    views, pos = [], 0
    while pos < buf.size - (8 << 20):
        n = int(rng.integers(0, 6 << 20))
        views.append(buf[pos:pos + n])
        pos += n + (int(rng.integers(1, 4096)) if rng.random() < 0.3 else 0)  # sometimes a gap
    got = batch.split_batch_host(name, views)
    want = coracle.split_batch(name, views, nthreads=8)
    for i, (g, w) in enumerate(zip(got, want)):
        assert np.array_equal(g, np.asarray(w, dtype=np.int64)), (i, views[i].size)


def test_files_overflowing_batch_stream_stays_in_its_range():
    """A batch stream whose caller-sized cut range is too small (1 slot for many chunks) sits
    between two long-path streams: its overflow is reported (count > its capacity) and never
    lands in the long streams' ranges (their cuts stay exact; a sentinel after them too)."""
    import ctypes as C
    from kopia_amd import _lib
    name = "DYNAMIC-128K-BUZHASH"
    sizes = [96 << 20, 3 << 20, 96 << 20]  # long, batch (about 20 chunks), long
    host, offs = _arena(sizes, sid0=900)
    dev = torch.device("cuda", 0)
    d = torch.from_numpy(host).to(dev)
    caps = [ks.cut_capacity(name, sizes[0]), 1, ks.cut_capacity(name, sizes[2])]
    base = np.array([0, caps[0], caps[0] + 1], dtype=np.uint64)
    cap = int(sum(caps))
    cuts = torch.full((cap + 8,), -7, dtype=torch.int64, device=dev)
    counts = torch.zeros(3, dtype=torch.int64, device=dev)
    ptrs = np.array([d.data_ptr() + o for o in offs], dtype=np.uint64)
    lens = np.array(sizes, dtype=np.uint64)
    _lib.check(_lib.lib().kcdc_split_files_device(name.encode(), ptrs.ctypes.data, lens.ctypes.data, 3,
                                                  cuts.data_ptr(), cap, base.ctypes.data, counts.data_ptr(),
                                                  C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)))
    torch.cuda.synchronize()
    c, k = cuts.cpu().numpy(), counts.cpu().numpy()
    want = coracle.split_batch(name, [host[o:o + L] for o, L in zip(offs, sizes)], nthreads=8)
    assert k[1] == len(want[1]) > 1  # the true count: larger than its 1-slot range
    assert c[base[1]] == want[1][0]
    for i in (0, 2):
        assert k[i] == len(want[i])
        assert np.array_equal(c[int(base[i]):int(base[i]) + k[i]], want[i]), i
    assert (c[cap:] == -7).all()


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0], []])
def test_host_batch_device_set(devices):
    """kcdc_split_batch_host_devices: host files spread over a device set by bytes (LPT), each
    device splitting its share from its own thread; every file's cuts equal the oracle's."""
    rng = np.random.default_rng(31)
    sizes = [int(x) for x in rng.integers(0, 9 << 20, 40)] + [70 << 20, 0, 1, 63]
    streams = [coracle.gen_stream(0x6B6F706961, 500 + i, n) for i, n in enumerate(sizes)]
    for name in ("DYNAMIC-4M-BUZHASH", "DYNAMIC-512K-RABINKARP", "FIXED-1M"):
        got = batch.split_batch_host_devices(name, streams, devices)
        for i, d in enumerate(streams):
            assert got[i].tolist() == coracle.split_stream(name, d).tolist(), (name, i, sizes[i])

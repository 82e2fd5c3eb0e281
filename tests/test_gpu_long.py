"""Config 3 path: one long stream split by the tiled candidate-scan + device
resolver (kcdc_split_long_device) must give the sequential cut set exactly."""
import numpy as np
import pytest

from kopia_amd import batch
from kopia_amd import splitter as ks
from oracle import coracle

pytestmark = pytest.mark.gpu
SEED = 0x6B6F706961


def _long(gpu, name, host: np.ndarray, misalign: int = 0):
    import torch
    buf = torch.zeros(host.size + 64, dtype=torch.uint8, device=gpu)
    buf[misalign:misalign + host.size] = torch.from_numpy(host).to(gpu)
    cuts, count, _ws = batch.split_long_device(name, buf.data_ptr() + misalign, host.size, gpu)
    torch.cuda.synchronize()
    return batch.read_long(cuts, count)


@pytest.mark.parametrize("name", ["DYNAMIC-4M-BUZHASH", "DYNAMIC-128K-BUZHASH", "DYNAMIC-128K-RABINKARP",
                                  "DYNAMIC-1M-RABINKARP", "DYNAMIC-8M-BUZHASH"])
@pytest.mark.parametrize("misalign", [0, 5])
def test_long_random(gpu, name, misalign):
    host = coracle.gen_stream(SEED, 99, (256 << 20) + 12345)
    np.testing.assert_array_equal(_long(gpu, name, host, misalign), coracle.split_stream(name, host))


@pytest.mark.parametrize("name", ["DYNAMIC-128K-BUZHASH", "DYNAMIC-128K-RABINKARP", "DYNAMIC-2M-BUZHASH"])
def test_long_dense_candidates(gpu, name):
    """Zero runs make every position a candidate (truncated segments -> rescans)."""
    host = coracle.gen_stream(SEED, 5, 40 << 20)
    host[3 << 20:20 << 20] = 0
    host[30 << 20:30 << 20 + 777] = 0
    np.testing.assert_array_equal(_long(gpu, name, host), coracle.split_stream(name, host))


def test_long_small_and_edge_lengths(gpu):
    name = "DYNAMIC-128K-BUZHASH"
    info = ks.lookup(name)
    for L in [1, 63, 64, 65, int(info.min_size) - 1, int(info.min_size), int(info.max_size) + 1, (1 << 20) + 3]:
        host = coracle.gen_stream(SEED, L, L)
        np.testing.assert_array_equal(_long(gpu, name, host, L % 16), coracle.split_stream(name, host), str(L))


def test_long_kat_custom(gpu, kat_data):
    """Small-average KAT parameterisations: many candidates per segment."""
    host = np.frombuffer(kat_data, dtype=np.uint8).copy()
    for kind, avg in [("buzhash", 32), ("rabinkarp", 1024), ("buzhash", 65536)]:
        got = _long(gpu, ks.custom_algorithm(kind, avg), host)
        L = coracle.lib()
        cap = host.size // (avg // 2) + 2
        out = np.zeros(cap, dtype=np.int64)
        n = L.orc_split_stream(coracle.KIND[kind], avg, host.ctypes.data, host.size, out, cap)
        np.testing.assert_array_equal(got, out[:n], f"{kind}-{avg}")


def test_long_matches_batch_path_4gib(gpu):
    """Two independent GPU paths (per-wave sequential vs tiled + resolve) on a 4 GiB
    stream, and the oracle on the same bytes."""
    import torch
    name, L = "DYNAMIC-4M-BUZHASH", 4 << 30
    data = torch.empty(L, dtype=torch.uint8, device=gpu)
    batch.fill_prng(data, L, 1, L, SEED, 0)
    cuts, count, _ws = batch.split_long_device(name, data.data_ptr(), L, gpu)
    b = batch.make_device_batch(name, [data.data_ptr()], [L], gpu)
    batch.split_batch_device(name, b)
    torch.cuda.synchronize()
    got_long = batch.read_long(cuts, count)
    got_seq = batch.read_cuts(b)[0]
    np.testing.assert_array_equal(got_long, got_seq)
    want, cnt = coracle.split_prng_streams(name, SEED, [0], L, nthreads=1)
    np.testing.assert_array_equal(got_long, want[0, :cnt[0]])

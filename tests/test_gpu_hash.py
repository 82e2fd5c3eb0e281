"""GPU: content hashes of many chunks (kcdc_hash_chunks_device) bit-exact against the oracle
(oracle/hashes.py, pinned by tests/test_hash_oracle.py): keyed BLAKE2, HMAC-SHA2/SHA3, keyed BLAKE3: random chunk lengths and
misaligned offsets, every registered name and key length class, the chunks the splitter
cuts on config-2 streams, and the error contract -- through both kernels (one lane per chunk,
and a quad of lanes per chunk)."""
import concurrent.futures as cf

import numpy as np
import pytest

from kopia_amd import _lib, batch
from kopia_amd import hashing as kh
from oracle import coracle
from test_hash_oracle import kopia_hash

pytestmark = pytest.mark.gpu
SEED = 0x6B6F706961


def _hash_all(name, key, host, offs, lens):
    import torch
    dev = torch.device("cuda", 0)
    d = torch.from_numpy(host).to(dev)
    out = kh.hash_chunks_device(name, d.data_ptr(), offs, lens, key, dev)
    torch.cuda.synchronize()
    return out.cpu().numpy()


@pytest.fixture(params=[1, 4], ids=["lane", "quad"])
def lanes(request):
    """Both kernels: one lane per chunk, and a quad of lanes per chunk (KCDC_TEST_HASH_LANES)."""
    L = _lib.lib()
    L.kcdc_test_set(_lib.TEST_HASH_LANES, request.param)
    yield request.param
    L.kcdc_test_set(_lib.TEST_HASH_LANES, 0)


@pytest.mark.parametrize("name", ["BLAKE2B-256-128", "BLAKE2B-256", "BLAKE2S-128", "BLAKE2S-256"])
def test_random_chunks(gpu, name, lanes):
    rng = np.random.default_rng(len(name))
    host = coracle.gen_stream(SEED, 31, 4 << 20)
    n = 700
    lens = rng.integers(0, 20000, n)
    lens[:16] = [0, 1, 3, 4, 15, 16, 17, 31, 32, 33, 63, 64, 65, 127, 128, 129]
    lens[16:20] = [255, 256, 96, 97]
    offs = np.array([int(rng.integers(0, host.size - int(L))) for L in lens], dtype=np.int64)
    maxk = 64 if name.startswith("BLAKE2B") else 32
    for klen in sorted({0, 1, 17, 32, maxk}):
        if name == "BLAKE2S-128" and klen == 0:
            continue
        key = bytes(rng.integers(0, 256, klen, dtype=np.uint8))
        got = _hash_all(name, key, host, offs, lens)
        for i in range(n):
            want = kopia_hash(name, key, host[offs[i]:offs[i] + lens[i]].tobytes())
            assert got[i].tobytes() == want, (name, klen, i, int(lens[i]), int(offs[i]))


def test_config2_chunks(gpu, lanes):
    """The chunks the batch splitter cuts from 256 x 4 MiB counter-PRNG streams, hashed with
    the default algorithm and a 32-byte secret, equal the oracle's digests."""
    import torch
    name, ns, L = "DYNAMIC-4M-BUZHASH", 256, 4 << 20
    dev = torch.device("cuda", 0)
    data = torch.empty(ns * L, dtype=torch.uint8, device=dev)
    batch.fill_prng(data, L, ns, L, SEED, 0)
    b = batch.make_device_batch(name, [data.data_ptr() + i * L for i in range(ns)], [L] * ns, dev)
    batch.split_batch_device(name, b)
    cuts = batch.read_cuts(b)
    offs, lens = kh.chunk_table([i * L for i in range(ns)], cuts)
    key = bytes(range(32))
    out = kh.hash_chunks_device(kh.DefaultAlgorithm, data.data_ptr(), offs, lens, key, dev)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    host = data.cpu().numpy()
    with cf.ThreadPoolExecutor(16) as ex:
        want = list(ex.map(lambda i: kopia_hash(kh.DefaultAlgorithm, key, host[offs[i]:offs[i] + lens[i]].tobytes()),
                           range(len(offs))))
    bad = [i for i in range(len(offs)) if got[i].tobytes() != want[i]]
    assert not bad, f"{len(bad)} of {len(offs)} chunks differ"


def test_errors(gpu):
    import torch
    dev = torch.device("cuda", 0)
    d = torch.zeros(64, dtype=torch.uint8, device=dev)
    with pytest.raises(_lib.KcdcError):
        kh.hash_chunks_device("BLAKE2B-256", d.data_ptr(), [0], [10], b"x" * 65, dev)
    with pytest.raises(_lib.KcdcError):
        kh.hash_chunks_device("BLAKE2S-256", d.data_ptr(), [0], [10], b"x" * 33, dev)
    with pytest.raises(_lib.KcdcError):
        kh.hash_chunks_device("BLAKE2S-128", d.data_ptr(), [0], [10], b"", dev)
    with pytest.raises(_lib.KcdcError):
        kh.hash_chunks_device("SHA256", d.data_ptr(), [0], [10], b"k", dev)


@pytest.mark.parametrize("name", ["BLAKE2B-256-128", "BLAKE2S-256"])
def test_large_chunks(gpu, name, lanes):
    """Chunks of 64 MiB to 256 MiB + 5 at odd offsets (block counters past 2^21 blocks,
    unaligned tails) through both kernels, against hashlib."""
    import torch
    sizes = [64 << 20, (128 << 20) + 1, (256 << 20) + 5]
    offs = np.array([3, 3 + sizes[0] + 7, 3 + sizes[0] + 7 + sizes[1] + 1], dtype=np.int64)
    total = int(offs[-1] + sizes[-1] + 16)
    host = coracle.gen_stream(SEED, 41, total)
    key = bytes(range(7, 39))
    got = _hash_all(name, key, host, offs, np.array(sizes, np.int64))
    for i, L in enumerate(sizes):
        assert got[i].tobytes() == kopia_hash(name, key, host[offs[i]:offs[i] + L].tobytes()), (name, L)
    del torch


NEW = ["BLAKE3-256", "BLAKE3-256-128", "HMAC-SHA224", "HMAC-SHA256", "HMAC-SHA256-128", "HMAC-SHA3-224",
       "HMAC-SHA3-256"]


@pytest.mark.parametrize("name", NEW)
def test_hmac_and_blake3_random_chunks(gpu, name):
    """HMAC-SHA2/SHA3 (one lane per chunk) and keyed BLAKE3 (one wave per chunk, tree of 1 KiB
    chunk CVs) against the oracle: lengths at every block / rate / chunk / round boundary, keys
    shorter and longer than the HMAC block (hashed first) and than BLAKE3's 32 bytes (derived)."""
    rng = np.random.default_rng(len(name) * 7)
    host = coracle.gen_stream(SEED, 33, 8 << 20)
    edge = [0, 1, 3, 55, 56, 63, 64, 65, 119, 120, 135, 136, 137, 143, 144, 145, 271, 272, 273, 1023, 1024, 1025,
            2047, 2048, 2049, 3072, 3073, 65535, 65536, 65537, 262143, 262144, 262145, 524288, 786432 + 5]
    lens = np.array(edge + [int(x) for x in rng.integers(0, 300000, 300)], dtype=np.int64)
    offs = np.array([int(rng.integers(0, host.size - int(L))) for L in lens], dtype=np.int64)
    for klen in (0, 1, 31, 32, 33, 64, 65, 137, 145, 200):
        key = bytes(rng.integers(0, 256, klen, dtype=np.uint8))
        got = _hash_all(name, key, host, offs, lens)
        with cf.ThreadPoolExecutor(16) as ex:
            want = list(ex.map(lambda i: kopia_hash(name, key, host[offs[i]:offs[i] + lens[i]].tobytes()),
                               range(len(lens))))
        bad = [(i, int(lens[i])) for i in range(len(lens)) if got[i].tobytes() != want[i]]
        assert not bad, (name, klen, bad[:5])


@pytest.mark.parametrize("name", ["BLAKE3-256", "HMAC-SHA256", "HMAC-SHA3-256"])
def test_hmac_and_blake3_large_chunks(gpu, name):
    """Multi-round BLAKE3 trees (stack merges over 256-chunk rounds, a ragged last round) and
    long HMAC chains: 4 MiB, 16 MiB + 3 and 64 MiB + 1025 at odd offsets."""
    sizes = [4 << 20, (16 << 20) + 3, (64 << 20) + 1025]
    offs = np.array([5, 5 + sizes[0] + 1, 5 + sizes[0] + 1 + sizes[1] + 9], dtype=np.int64)
    host = coracle.gen_stream(SEED, 43, int(offs[-1] + sizes[-1] + 16))
    key = bytes(range(32))
    got = _hash_all(name, key, host, offs, np.array(sizes, np.int64))
    for i, L in enumerate(sizes):
        assert got[i].tobytes() == kopia_hash(name, key, host[offs[i]:offs[i] + L].tobytes()), (name, L)

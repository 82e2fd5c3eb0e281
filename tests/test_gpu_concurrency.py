"""GPU: many batch launches in flight at once on different HIP streams (more than the 64
per-device queue workspaces), every result bit-exact against the oracle."""
import numpy as np
import pytest
import torch

from kopia_amd import batch
from oracle import coracle

pytestmark = pytest.mark.gpu
SEED = 0x6B6F706961


def test_more_launches_than_queue_slots_across_streams():
    name, ns, L, nl = "DYNAMIC-128K-BUZHASH", 6, 3 << 20, 96
    dev = torch.device("cuda", 0)
    data = torch.empty(ns * L, dtype=torch.uint8, device=dev)
    batch.fill_prng(data, L, ns, L, SEED, first_sid=300)
    streams = [torch.cuda.Stream(dev) for _ in range(8)]
    batches = []
    torch.cuda.synchronize(dev)
    for k in range(nl):  # rotate the stream ids per launch so every launch has different inputs
        order = [(i + k) % ns for i in range(ns)]
        b = batch.make_device_batch(name, [data.data_ptr() + i * L for i in order], [L] * ns, dev)
        batches.append((order, b))
    torch.cuda.synchronize(dev)
    for k, (order, b) in enumerate(batches):
        batch.split_batch_device(name, b, streams[k % len(streams)])
    torch.cuda.synchronize(dev)
    host = data.cpu().numpy()
    want = coracle.split_batch(name, [host[i * L:(i + 1) * L] for i in range(ns)], nthreads=8)
    for k, (order, b) in enumerate(batches):
        got = batch.read_cuts(b)
        for j, i in enumerate(order):
            assert np.array_equal(got[j], np.asarray(want[i], dtype=np.int64)), (k, j)


def test_many_tiny_streams_one_launch():
    """200,000 streams of 0..4096 bytes in one batch launch (n >> waves: every ticket, ring
    entry and tombstone path of the queue at scale); all below min size, so each stream is
    one chunk ending at its length (empty streams: none)."""
    name, n = "DYNAMIC-128K-BUZHASH", 200_000
    rng = np.random.default_rng(5)
    lens = rng.integers(0, 4097, n)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]])
    dev = torch.device("cuda", 0)
    data = torch.zeros(int(lens.sum()) + 64, dtype=torch.uint8, device=dev)
    b = batch.make_device_batch(name, [data.data_ptr() + int(o) for o in offs], lens.tolist(), dev)
    batch.split_batch_device(name, b)
    torch.cuda.synchronize(dev)
    got = batch.read_cuts(b)
    for i in range(n):
        want = [int(lens[i])] if lens[i] else []
        assert got[i].tolist() == want, (i, int(lens[i]))

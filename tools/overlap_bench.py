"""Config-2 batches back to back: one stream vs consecutive launches alternating over S streams
(each stream its own cut buffers), wall time per batch; every launch's cuts equal the first's."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kopia_amd import batch  # noqa: E402

name, ns, L = "DYNAMIC-4M-BUZHASH", 4096, 4 << 20
dev = torch.device("cuda:0")
data = torch.empty(ns * L, dtype=torch.uint8, device=dev)
batch.fill_prng(data, L, ns, L, 0x6B6F706961, 0)
ptrs = [data.data_ptr() + i * L for i in range(ns)]
bs = [batch.make_device_batch(name, ptrs, [L] * ns, dev) for _ in range(4)]
sts = [torch.cuda.Stream(dev) for _ in range(4)]
batch.split_batch_device(name, bs[0])
torch.cuda.synchronize()
ref = batch.read_cuts(bs[0])
K = int(sys.argv[1]) if len(sys.argv) > 1 else 40
for rnd in range(3):
    for S in (1, 2, 3):
        for i in range(8):  # warm
            batch.split_batch_device(name, bs[i % S], sts[i % S])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(K):
            batch.split_batch_device(name, bs[i % S], sts[i % S])
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / K
        bad = sum(0 if all(np.array_equal(a, b) for a, b in zip(batch.read_cuts(bs[s]), ref)) else 1 for s in range(S))
        print(f"round {rnd} streams {S}: {dt * 1e3:.4f} ms/batch = {ns * L / dt / 2**30:.0f} GiB/s  parity_bad={bad}", flush=True)

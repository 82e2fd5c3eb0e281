"""Per-launch durations of consecutive config-2 launches (HIP events around each), from a cold
start and after idle / memory-traffic preambles: does the kernel's duration ramp over the first
launches, and what makes it settle?  Prints one line per scenario."""
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
b = batch.make_device_batch(name, [data.data_ptr() + i * L for i in range(ns)], [L] * ns, dev)
st = torch.cuda.current_stream(dev)
scratch = torch.empty(4 << 30, dtype=torch.uint8, device=dev)


def launches(k):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(k)]
    for e0, e1 in ev:
        e0.record(st)
        batch.split_batch_device(name, b, st)
        e1.record(st)
    torch.cuda.synchronize()
    return [e0.elapsed_time(e1) for e0, e1 in ev]


def show(tag, t):
    t = np.array(t)
    print(f"{tag:28s} first10 {' '.join(f'{x:.3f}' for x in t[:10])} | 10-29 {t[10:30].mean():.4f} "
          f"| 30-59 {t[30:60].mean():.4f} | 5-24 {t[5:25].mean():.4f}", flush=True)


show("cold (after fill)", launches(60))
time.sleep(2.0)
show("after 2 s idle", launches(60))
time.sleep(2.0)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.3:
    scratch.add_(1)
show("after 300 ms of add_ traffic", launches(60))
time.sleep(2.0)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.3:
    batch.split_batch_device(name, b, st)
    torch.cuda.synchronize()
show("after 300 ms of splits", launches(60))

"""FETCH_SIZE calibration: kernels with a known number of HBM bytes read.
(1) torch sum over a 4 GiB uint8 buffer (coalesced 16 B/lane streaming read);
(2) the long-path candidate scan (kcdc cand_scan_kernel) over a 4 GiB stream,
    which reads every byte once (+64 B warm-up per 1 KiB lane range)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kopia_amd import batch  # noqa: E402

L = 4 << 30
dev = torch.device("cuda:0")
x = torch.empty(L, dtype=torch.uint8, device=dev)
batch.fill_prng(x, L, 1, L, 1, 0)
for _ in range(3):
    x.view(torch.int64).sum()
for _ in range(3):
    batch.split_long_device("DYNAMIC-4M-BUZHASH", x.data_ptr(), L, dev)
torch.cuda.synchronize()
print("calib bytes", L)

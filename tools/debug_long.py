"""Dump the long-path workspace phases and compare with oracle candidates."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kopia_amd import batch  # noqa: E402
from oracle import coracle, rollinghash  # noqa: E402

name = "DYNAMIC-4M-BUZHASH"
n = (256 << 20) + 12345
host = coracle.gen_stream(0x6B6F706961, 99, n)
dev = torch.device("cuda:0")
buf = torch.from_numpy(host).to(dev)
cuts, count, ws = batch.split_long_device(name, buf.data_ptr(), n, dev)
torch.cuda.synchronize()
S, K = 64 << 10, 4
nseg = (n + 15 + S - 1) // S
al = lambda x: (x + 255) & ~255
w = ws.cpu().numpy()
o = 0
seg_cnt = w[o:o + nseg * 4].view(np.uint32); o += al(nseg * 4)
seg_cand = w[o:o + nseg * K * 8].view(np.uint64).reshape(nseg, K); o += al(nseg * K * 8)
seg_off = w[o:o + nseg * 8].view(np.uint64); o += al(nseg * 8)
lst = w[o:o + nseg * K * 8].view(np.uint64); o += al(nseg * K * 8)
total = w[o:o + 8].view(np.uint64)[0]
print("count", int(count.item()), "total", total, "nonzero segs", int((seg_cnt & 0x7fffffff).sum()))
# oracle candidates: positions p with hash & mask == 0 (C oracle via tiny avg? use python on first 4 MiB)
T = [int(x) for x in rollinghash.buzhash_table()]
mask = (4 << 20) - 1
h = 0
win = [0] * 64
cands = []
m = 16 << 20
for p in range(m):
    c = int(host[p])
    out = win[p & 63]
    win[p & 63] = c
    h = (((h << 1) | (h >> 31)) & 0xFFFFFFFF) ^ T[out] ^ T[c]
    if h & mask == 0:
        cands.append(p)
print("oracle cands in first 16 MiB:", cands)
g = [(i, int(seg_cnt[i]), seg_cand[i].tolist()) for i in range(min(nseg, 256)) if seg_cnt[i]]
print("gpu segs with cands in first 16MiB:", g)
print("list head", lst[:min(int(total), 10)].tolist())
print("cuts", cuts[:int(count.item())].cpu().numpy()[:10].tolist())

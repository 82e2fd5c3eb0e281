import os, sys, time
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kopia_amd import batch
from oracle import coracle
name, L = "DYNAMIC-4M-BUZHASH", int(sys.argv[1]) << 20
dev = torch.device("cuda:0")
t = time.time()
def log(*a):
    print(f"[{time.time()-t:7.2f}s]", *a, flush=True)
data = torch.empty(L, dtype=torch.uint8, device=dev)
batch.fill_prng(data, L, 1, L, 0x6B6F706961, 0); torch.cuda.synchronize(); log("filled")
cuts, count, ws = batch.split_long_device(name, data.data_ptr(), L, dev); torch.cuda.synchronize(); log("long done", int(count.item()))
b = batch.make_device_batch(name, [data.data_ptr()], [L], dev)
batch.split_batch_device(name, b); torch.cuda.synchronize(); log("batch done")
gl = batch.read_long(cuts, count); gs = batch.read_cuts(b)[0]
log("equal", np.array_equal(gl, gs), len(gl), len(gs))
want, cnt = coracle.split_prng_streams(name, 0x6B6F706961, [0], L, nthreads=1); log("oracle done")
log("oracle equal", np.array_equal(gl, want[0, :cnt[0]]))

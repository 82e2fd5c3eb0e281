"""Tiny single-process check of one library (path) on a few streams vs the oracle."""
import ctypes as C, os, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kopia_amd import _lib, batch
from oracle import coracle
path, ns, mib = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
f = C.CDLL(path).kcdc_split_batch_device
f.restype = C.c_int; f.argtypes = _lib._SIGS["kcdc_split_batch_device"][1]
name, L = "DYNAMIC-4M-BUZHASH", mib << 20
dev = torch.device("cuda:0")
data = torch.empty(ns * L, dtype=torch.uint8, device=dev)
batch.fill_prng(data, L, ns, L, 0x6B6F706961, 0)
b = batch.make_device_batch(name, [data.data_ptr() + i * L for i in range(ns)], [L] * ns, dev)
st = torch.cuda.current_stream(dev)
assert f(name.encode(), b.ptrs.data_ptr(), b.lens.data_ptr(), b.n, b.cuts.data_ptr(), b.cap, b.cut_base.data_ptr(), b.counts.data_ptr(), C.c_void_p(st.cuda_stream)) == 0
torch.cuda.synchronize()
got = batch.read_cuts(b)
want, cnt = coracle.split_prng_streams(name, 0x6B6F706961, np.arange(ns), L, nthreads=8)
bad = sum(1 for i in range(ns) if got[i].tolist() != want[i, :cnt[i]].tolist())
print(os.path.basename(path), ns, mib, "mismatches", bad, flush=True)
sys.exit(1 if bad else 0)

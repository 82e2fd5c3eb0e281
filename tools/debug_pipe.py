"""Debug run of a library build with -DKCDC_DEBUG_CHECKS=1 on the config-2 workload:
prints the queue header (head/tail/done/err and the first recorded check failure) and
the streams whose cut lists differ from the oracle."""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from kopia_amd import _lib, batch  # noqa: E402
from oracle import coracle  # noqa: E402

lib_path = sys.argv[1]
ns = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
mib = int(sys.argv[3]) if len(sys.argv) > 3 else 4
name, L, SEED = "DYNAMIC-4M-BUZHASH", mib << 20, 0x6B6F706961
dev = torch.device("cuda:0")
data = torch.empty(ns * L, dtype=torch.uint8, device=dev)
batch.fill_prng(data, L, ns, L, SEED, 0)
b = batch.make_device_batch(name, [data.data_ptr() + i * L for i in range(ns)], [L] * ns, dev)
lib = C.CDLL(lib_path)
f = lib.kcdc_split_batch_device
f.restype = C.c_int
f.argtypes = _lib._SIGS["kcdc_split_batch_device"][1]
st = torch.cuda.current_stream(dev)
rc = f(name.encode(), b.ptrs.data_ptr(), b.lens.data_ptr(), ns, b.cuts.data_ptr(), b.cap, b.cut_base.data_ptr(),
       b.counts.data_ptr(), C.c_void_p(st.cuda_stream))
torch.cuda.synchronize()
hdr = np.zeros(2048, dtype=np.uint32)
print("rc", rc, "copy", lib.kcdc_debug_queue_copy(hdr.ctypes.data_as(C.c_void_p)))
S = 1792
print({"head": int(hdr[0]), "done": int(hdr[512]), "tail": int(hdr[1024]), "err": int(hdr[1536]),
       "first_fail": [int(x) for x in hdr[S + 16:S + 24]]}, flush=True)
got = batch.read_cuts(b)
cuts, counts = coracle.split_prng_streams(name, SEED, np.arange(ns), L, nthreads=16)
bad = [i for i in range(ns) if got[i].tolist() != cuts[i, :counts[i]].tolist()]
print("mismatched streams", len(bad), bad[:10])
for i in bad[:3]:
    print(i, "got", got[i].tolist()[:6], "want", cuts[i, :counts[i]].tolist()[:6])

"""Per-wave start/end trace of the pipelined batch kernel (library built with
-DKCDC_TRACE=1): how much of the kernel's span the waves are alive, and
the spread of their end times (the scheduling tail).  usage: trace_pipe.py LIB [ns mib]"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from kopia_amd import _lib, batch  # noqa: E402

lib_path = sys.argv[1]
ns = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
mib = int(sys.argv[3]) if len(sys.argv) > 3 else 4
name, L = "DYNAMIC-4M-BUZHASH", mib << 20
dev = torch.device("cuda:0")
data = torch.empty(ns * L, dtype=torch.uint8, device=dev)
batch.fill_prng(data, L, ns, L, 0x6B6F706961, 0)
b = batch.make_device_batch(name, [data.data_ptr() + i * L for i in range(ns)], [L] * ns, dev)
lib = C.CDLL(lib_path)
f = lib.kcdc_split_batch_device
f.restype = C.c_int
f.argtypes = _lib._SIGS["kcdc_split_batch_device"][1]
st = torch.cuda.current_stream(dev)
for _ in range(4):
    assert f(name.encode(), b.ptrs.data_ptr(), b.lens.data_ptr(), ns, b.cuts.data_ptr(), b.cap,
             b.cut_base.data_ptr(), b.counts.data_ptr(), C.c_void_p(st.cuda_stream)) == 0
    torch.cuda.synchronize()
tr = np.zeros(3 * ns, dtype=np.uint64)
assert lib.kcdc_debug_trace_copy(tr.ctypes.data_as(C.c_void_p), C.c_uint64(ns)) == 0
waves = int(torch.cuda.get_device_properties(0).multi_processor_count) * 8
t = tr[:4 * waves].reshape(waves, 4).astype(np.float64)
t = t[(t[:, 0] > 0) & (t[:, 1] > 0)]
t0 = t[:, 0].min()
st_us, en_us = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0  # 100 MHz
blk_us = t[:, 2] / 100.0
span = en_us.max()
print(json.dumps({"waves": int(t.shape[0]), "span_us": round(span, 1),
                  "busy_frac": round(float((en_us - st_us).mean() / span), 4),
                  "blocking_take_us_per_wave": round(float(blk_us.mean()), 1),
                  "final_idle_us_pct": {p: round(float(np.percentile(en_us - (t[:, 3] - t0) / 100.0, p)), 1)
                                        for p in (10, 50, 90, 99)},
                  "blocking_take_us_pct": {p: round(float(np.percentile(blk_us, p)), 1) for p in (10, 50, 90, 99)},
                  "start_us_max": round(float(st_us.max()), 1),
                  "end_us_pct": {p: round(float(np.percentile(en_us, p)), 1) for p in (1, 10, 25, 50, 75, 90, 99, 100)}}))

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
knob = [int(x) for x in os.environ.get("KCDC_TRACE_KNOB", "").split("=")] if os.environ.get("KCDC_TRACE_KNOB") else None
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
if knob:
    lib.kcdc_test_set(knob[0], knob[1])
for _ in range(4):
    assert f(name.encode(), b.ptrs.data_ptr(), b.lens.data_ptr(), ns, b.cuts.data_ptr(), b.cap,
             b.cut_base.data_ptr(), b.counts.data_ptr(), C.c_void_p(st.cuda_stream)) == 0
    torch.cuda.synchronize()
waves = int(torch.cuda.get_device_properties(0).multi_processor_count) * 8
nrec = max(ns, 3 * waves)  # the library reserves 3 words per max(streams, 3 x waves)
tr = np.zeros(3 * nrec, dtype=np.uint64)
assert lib.kcdc_debug_trace_copy(tr.ctypes.data_as(C.c_void_p), C.c_uint64(nrec)) == 0
t = tr[:8 * waves].reshape(waves, 8).astype(np.float64)
t = t[(t[:, 0] > 0) & (t[:, 1] > 0)]
t0 = t[:, 0].min()
st_us, en_us = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0  # 100 MHz
blk_us = t[:, 2] / 100.0
own_end = np.where(t[:, 6] > 0, (t[:, 6] - t0) / 100.0, 0.0)
span = en_us.max()
# waves still scanning a stream of their own at time x (the tail's shape)
grid = np.linspace(0, span, 41)
owners = [int((own_end >= x).sum()) for x in grid]
print(json.dumps({"waves": int(t.shape[0]), "span_us": round(span, 1),
                  "busy_frac": round(float((en_us - st_us).mean() / span), 4),
                  "blocking_take_us_per_wave": round(float(blk_us.mean()), 1),
                  "final_idle_us_pct": {p: round(float(np.percentile(en_us - (t[:, 3] - t0) / 100.0, p)), 1)
                                        for p in (10, 50, 90, 99)},
                  "blocking_take_us_pct": {p: round(float(np.percentile(blk_us, p)), 1) for p in (10, 50, 90, 99)},
                  "start_us_max": round(float(st_us.max()), 1),
                  "end_us_pct": {p: round(float(np.percentile(en_us, p)), 1) for p in (1, 10, 25, 50, 75, 90, 99, 100)},
                  "help_tiles": int(t[:, 4].sum()), "own_tiles": int(t[:, 7].sum()),
                  "help_tile_us_mean": round(float(t[:, 5].sum() / max(t[:, 4].sum(), 1) / 100.0), 2),
                  "last_own_tile_end_us_pct": {p: round(float(np.percentile(own_end, p)), 1)
                                               for p in (10, 50, 90, 99, 100)},
                  "owners_vs_time": {f"{x:.0f}": o for x, o in zip(grid, owners)}}))

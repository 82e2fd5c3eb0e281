"""Per-stream timing trace of the persistent batch kernel (build/variants/libkcdc_trace.so,
built with -DKCDC_TRACE=1): start/end s_memrealtime (100 MHz) and the workgroup/wave
that ran each stream.  Reports how the waves' busy time is distributed over the
kernel's span (the scheduling tail) and writes the raw trace to gpurun_out/."""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from kopia_amd import _lib, batch  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "DYNAMIC-4M-BUZHASH"
ns = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
mib = int(sys.argv[3]) if len(sys.argv) > 3 else 4
L = mib << 20
dev = torch.device("cuda:0")
data = torch.empty(ns * L, dtype=torch.uint8, device=dev)
batch.fill_prng(data, L, ns, L, 0x6B6F706961, 0)
b = batch.make_device_batch(name, [data.data_ptr() + i * L for i in range(ns)], [L] * ns, dev)
lib = C.CDLL(os.path.join(ROOT, os.environ.get("TRACE_LIB", "build/variants/libkcdc_trace.so")))
f = lib.kcdc_split_batch_device
f.restype = C.c_int
f.argtypes = _lib._SIGS["kcdc_split_batch_device"][1]
stream = torch.cuda.current_stream(dev)
out = {}
for rep in range(4):
    rc = f(name.encode(), b.ptrs.data_ptr(), b.lens.data_ptr(), ns, b.cuts.data_ptr(), b.cap,
           b.cut_base.data_ptr(), b.counts.data_ptr(), C.c_void_p(stream.cuda_stream))
    assert rc == 0, rc
    torch.cuda.synchronize()
tr = np.zeros(3 * ns, dtype=np.uint64)
assert lib.kcdc_debug_trace_copy(tr.ctypes.data_as(C.c_void_p), C.c_uint64(ns)) == 0
tr = tr.reshape(ns, 3)
t0 = tr[:, 0].min()
st = (tr[:, 0] - t0).astype(np.float64) * 10e-3  # us
en = (tr[:, 1] - t0).astype(np.float64) * 10e-3
span = en.max()
wg = (tr[:, 2] & 0xFFFF).astype(int)
wv = (tr[:, 2] >> 16).astype(int)
dur = en - st
# active streams over time
grid = np.linspace(0, span, 41)
active = [int(((st <= t) & (en > t)).sum()) for t in grid]
per_wave_end = {}
for i in range(ns):
    k = (wg[i], wv[i])
    per_wave_end[k] = max(per_wave_end.get(k, 0), en[i])
ends = np.array(sorted(per_wave_end.values()))
out = {"streams": ns, "span_us": span, "dur_us": {"mean": dur.mean(), "min": dur.min(), "max": dur.max()},
       "busy_frac": float(dur.sum() / (len(per_wave_end) * span)), "waves": len(per_wave_end),
       "wave_end_us_pct": {p: float(np.percentile(ends, p)) for p in (1, 10, 25, 50, 75, 90, 99)},
       "active_streams_over_time": active, "second_stream_starts": int((st > 1.0).sum())}
print(json.dumps(out, indent=1))
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.save(os.path.join(ROOT, "gpurun_out", "trace_sched.npy"), tr)
hdr = np.zeros(2048, dtype=np.uint32)  # kQHeaderBytes / 4
if lib.kcdc_debug_queue_copy(hdr.ctypes.data_as(C.c_void_p)) == 0:
    S = 1792  # kQStat
    c64 = lambda w: int(hdr[w]) | (int(hdr[w + 1]) << 32)
    q = {"head": int(hdr[0]), "done": int(hdr[512]), "tail": int(hdr[1024]), "err": int(hdr[1536]),
         "yields": int(hdr[S]), "entry_wait_spins": int(hdr[S + 2]), "slot_wait_spins": int(hdr[S + 3]),
         "take_ms_wave_sum": c64(S + 4) / 100e3, "yield_ms_wave_sum": c64(S + 6) / 100e3,
         "run_ms_wave_sum": c64(S + 8) / 100e3}
    print(json.dumps({"queue": q}))

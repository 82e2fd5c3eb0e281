"""Per-wave time breakdown of the Rabin-Karp batch kernel (library built with -DKCDC_TRACE=1,
`make instrumented`): the span each wave is alive, its blocking takes, and -- in shader cycles --
its line-fill DMA waits, walks and warm fills, against the rest (queue, help, tile bookkeeping).
usage: trace_rk.py LIB [name] [streams] [mib]"""
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
name = sys.argv[2] if len(sys.argv) > 2 else "DYNAMIC-4M-RABINKARP"
ns = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
L = (int(sys.argv[4]) if len(sys.argv) > 4 else 4) << 20
dev = torch.device("cuda:0")
data = torch.empty(ns * L, dtype=torch.uint8, device=dev)
batch.fill_prng(data, L, ns, L, 0x6B6F706961, 0)
b = batch.make_device_batch(name, [data.data_ptr() + i * L for i in range(ns)], [L] * ns, dev)
lib = C.CDLL(lib_path)
f = lib.kcdc_split_batch_device
f.restype = C.c_int
f.argtypes = _lib._SIGS["kcdc_split_batch_device"][1]
st = torch.cuda.current_stream(dev)
ms = []
for _ in range(6):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    assert f(name.encode(), b.ptrs.data_ptr(), b.lens.data_ptr(), ns, b.cuts.data_ptr(), b.cap,
             b.cut_base.data_ptr(), b.counts.data_ptr(), C.c_void_p(st.cuda_stream)) == 0
    e1.record(st)
    torch.cuda.synchronize()
    ms.append(e0.elapsed_time(e1))
waves = int(torch.cuda.get_device_properties(0).multi_processor_count) * 8
nrec = max(ns, 3 * waves)
tr = np.zeros(3 * nrec, dtype=np.uint64)
assert lib.kcdc_debug_trace_copy(tr.ctypes.data_as(C.c_void_p), C.c_uint64(nrec)) == 0
t = tr[:8 * waves].reshape(waves, 8).astype(np.float64)
mt = tr[8 * waves:9 * waves].astype(np.float64)
ok = (t[:, 0] > 0) & (t[:, 1] > 0)
t, mt = t[ok], mt[ok]
t0 = t[:, 0].min()
st_us, en_us = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0  # s_memrealtime: 100 MHz
life_us = en_us - st_us
clk = mt / (life_us * 1e3)  # shader GHz per wave
cyc_us = lambda c: c / (clk * 1e3)  # noqa: E731
block_us = t[:, 2] / 100.0
dma_us, walk_us, warm_us = cyc_us(t[:, 5]), cyc_us(t[:, 6]), cyc_us(t[:, 7])
own = (t[:, 4].astype(np.uint64) >> np.uint64(32)).astype(np.float64)
helpt = (t[:, 4].astype(np.uint64) & np.uint64(0xFFFFFFFF)).astype(np.float64)
m = lambda x: round(float(np.mean(x)), 1)  # noqa: E731
print(json.dumps({"name": name, "streams": ns, "launch_ms": [round(x, 3) for x in ms], "waves": int(t.shape[0]),
                  "span_us": round(float(en_us.max()), 1), "clock_ghz": round(float(np.median(clk)), 3),
                  "per_wave_us": {"alive": m(life_us), "blocking_takes": m(block_us), "walk": m(walk_us),
                                  "of_which_dma_wait": m(dma_us), "warm_fill": m(warm_us),
                                  "other": m(life_us - block_us - walk_us - warm_us)},
                  "final_idle_us_pct": {p: round(float(np.percentile(en_us - (t[:, 3] - t0) / 100.0, p)), 1)
                                        for p in (10, 50, 90)},
                  "own_tiles": int(own.sum()), "help_tiles": int(helpt.sum())}))

"""A/B microbench of library variants (build/variants/libkcdc_*.so) on the config-2
workload, interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24).
Every variant's cut lists must equal the production library's."""
import argparse
import ctypes as C
import glob
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from kopia_amd import _lib, batch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--name", default="DYNAMIC-4M-BUZHASH")
ap.add_argument("--streams", type=int, default=4096)
ap.add_argument("--mib", type=int, default=4)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--glob", default="build/variants/libkcdc_*.so")
ap.add_argument("--knob", action="append", default=[],
                help="KEY=VALUE: also time the production library with kcdc_test_set(KEY, VALUE) "
                     "(e.g. 6=1: no intra-region help)")
args = ap.parse_args()

dev = torch.device("cuda:0")
name, ns, L = args.name, args.streams, args.mib << 20
data = torch.empty(ns * L, dtype=torch.uint8, device=dev)
batch.fill_prng(data, L, ns, L, 0x6B6F706961, 0)
b = batch.make_device_batch(name, [data.data_ptr() + i * L for i in range(ns)], [L] * ns, dev)
stream = torch.cuda.current_stream(dev)
batch.split_batch_device(name, b, stream)
torch.cuda.synchronize()
ref = [c.copy() for c in batch.read_cuts(b)]

libs = {}
for p in sorted(glob.glob(os.path.join(ROOT, args.glob))):
    Lb = C.CDLL(p)
    f = Lb.kcdc_split_batch_device
    f.restype = C.c_int
    f.argtypes = _lib._SIGS["kcdc_split_batch_device"][1]
    libs[os.path.basename(p)[8:-3]] = f
libs["prod"] = _lib.lib().kcdc_split_batch_device
knobs = {}
for kv in args.knob:
    k, v = (int(x) for x in kv.split("="))
    libs[f"prod_knob{k}={v}"] = _lib.lib().kcdc_split_batch_device
    knobs[f"prod_knob{k}={v}"] = (k, v)


def run(f, key=None):
    kv = knobs.get(key)
    if kv:
        _lib.lib().kcdc_test_set(kv[0], kv[1])
    rc = f(name.encode(), b.ptrs.data_ptr(), b.lens.data_ptr(), b.n, b.cuts.data_ptr(), b.cap,
           b.cut_base.data_ptr(), b.counts.data_ptr(), C.c_void_p(stream.cuda_stream))
    if kv:
        _lib.lib().kcdc_test_set(kv[0], 0)
    assert rc == 0, rc


times = {k: [] for k in libs}
for k, f in libs.items():  # warm + parity
    b.cuts.zero_()
    run(f, k)
    torch.cuda.synchronize()
    got = batch.read_cuts(b)
    bad = sum(1 for i in range(ns) if not np.array_equal(got[i], ref[i]))
    print(f"{k}: parity mismatches {bad}", flush=True)
for r in range(args.rounds):
    for k, f in libs.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.reps):
            run(f, k)
        e1.record(stream)
        torch.cuda.synchronize()
        times[k].append(e0.elapsed_time(e1) / args.reps)
res = {k: {"median_ms": float(np.median(v)), "min_ms": float(np.min(v)),
           "GiBps": ns * L / (1 << 30) / (np.median(v) * 1e-3)} for k, v in times.items()}
print(json.dumps(res, indent=1))

# reference: coalesced streaming read of the same 16 GiB with torch (sum of int64)
x = data.view(torch.int64)
x.sum()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(stream)
for _ in range(3):
    x.sum()
e1.record(stream)
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 3
print(f"torch.sum over {ns * L / 2**30:.0f} GiB: {ms:.3f} ms = {ns * L / ms / 1e6:.0f} GB/s")

"""Probe one batch launch with a bounded wait (test knob KCDC_TEST_SPIN_CAP: waves give up after
that many polls with no stream finishing, so a lost stream ends the launch with an error instead of
spinning), then print the launch's queue statistics and the streams whose cuts differ from the
oracle.  usage: batch_probe.py NAME STREAMS MIB [SPIN_CAP] [NO_HELP]"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from kopia_amd import _lib, batch  # noqa: E402
from oracle import coracle  # noqa: E402

name, ns, mib = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
cap = int(sys.argv[4]) if len(sys.argv) > 4 else 1 << 22
no_help = int(sys.argv[5]) if len(sys.argv) > 5 else 0
SEED, L = 0x6B6F706961, mib << 20
dev = torch.device("cuda:0")
data = torch.empty(ns * L, dtype=torch.uint8, device=dev)
batch.fill_prng(data, L, ns, L, SEED, 0)
b = batch.make_device_batch(name, [data.data_ptr() + i * L for i in range(ns)], [L] * ns, dev)
lib = _lib.lib()
lib.kcdc_test_set(_lib.TEST_SPIN_CAP, cap)
lib.kcdc_test_set(_lib.TEST_NO_HELP, no_help)
reps = int(os.environ.get("PROBE_REPS", "1"))
for rep in range(reps):  # until a launch loses a stream (a race shows in some launches only)
    t = time.time()
    rc = None
    try:
        batch.split_batch_device(name, b)
        torch.cuda.synchronize()
        rc = 0
    except Exception as e:  # noqa: BLE001
        rc = repr(e)
    # held-ticket audit and (KCDC_HELP_DIAG builds) lane-divergence record, header words kQDiag..
    diag = [int(lib.kcdc_test_queue_stat(k)) for k in range(5, 10)]
    print("launch", rep, rc, "%.3f s" % (time.time() - t), "helps", int(lib.kcdc_test_queue_stat(_lib.STAT_HELPS)),
          "ticket audit [mismatches, reg, mem]", diag[:3], "divergent [bits, count]", [hex(diag[3]), diag[4]], flush=True)
    if int(lib.kcdc_test_queue_stat(_lib.STAT_DONE)) < ns:
        break
st = {k: int(lib.kcdc_test_queue_stat(v)) for k, v in (("giveups", _lib.STAT_GIVEUPS), ("done", _lib.STAT_DONE),
                                                        ("steals", _lib.STAT_STEALS), ("helps", _lib.STAT_HELPS))}
print(st, flush=True)
import ctypes as C  # noqa: E402
_h = np.zeros(2048, np.uint32)
assert lib.kcdc_test_ws_copy(_h.ctypes.data_as(C.c_void_p), 0, 8192) == 0
# debug builds (KCDC_DEBUG_CHECKS): entries reserved / entries written (every reservation is written once)
print("head", int(_h[0]), "tail", int(_h[1]), "reserved (debug)", int(_h[1792 + 32]), "written (debug)", int(_h[1792 + 33]),
      "first check failure", _h[1792 + 16:1792 + 24].tolist(), flush=True)
counts = b.counts.cpu().numpy()[:ns].astype(np.int64)
print("failed counts", int((counts == -1).sum()), "max count", int(counts.max()), flush=True)
cuts, cnt = coracle.split_prng_streams(name, SEED, np.arange(ns), L, nthreads=16)
bad = []
allc = b.cuts.cpu().numpy()
base = b.cut_base.cpu().numpy()
for i in range(ns):
    c = int(counts[i])
    capi = (base[i + 1] if i + 1 < ns else b.cap) - base[i]
    if c < 0 or c > capi:
        bad.append(i)
        continue
    if allc[base[i]:base[i] + c].tolist() != cuts[i, :cnt[i]].tolist():
        bad.append(i)
print("mismatched streams", len(bad), bad[:10], flush=True)
for i in bad[:3]:
    c = int(counts[i])
    print(i, "count", c, "got", allc[base[i]:base[i] + min(max(c, 0), 6)].tolist(), "want", cuts[i, :cnt[i]].tolist()[:6])

# Post-mortem of the queue: header {head, tail}, then every ring entry up to the tail (7 tagged
# 16-byte granules each: cnt|sid, s, ct, ptr, n, cb, cap) -- where the lost streams' states are.
if bad:
    import ctypes as C
    hdr = np.zeros(2048, np.uint32)
    assert lib.kcdc_test_ws_copy(hdr.ctypes.data_as(C.c_void_p), 0, 8192) == 0
    head, tail = int(hdr[0]), int(hdr[1])
    print("head", head, "tail", tail, "done", int(hdr[512]), "first check failure (debug builds)",
          hdr[1792 + 16:1792 + 24].tolist(), flush=True)
    nw = 256 * 8
    live = ns + 8 * nw
    ring = 1
    while ring <= live:
        ring <<= 1
    ent = np.zeros((ring, 32), np.uint32)
    assert lib.kcdc_test_ws_copy(ent.ctypes.data_as(C.c_void_p), 8192, ring * 128) == 0
    lost = set(bad)
    unw = [e for e in range(ns, tail) if int(ent[e % ring][0]) != e + 1]
    print("reserved entries below the tail never written:", len(unw), unw[:10], flush=True)
    for e in range(max(tail, head) + 4):
        g = ent[e % ring]
        tags = g[0:28:4]
        sid = int(g[3])
        if sid in lost or e >= ns:
            s_ = int(g[4 + 1]) | (int(g[4 + 2]) << 32)
            ct = int(g[8 + 1]) | (int(g[8 + 2]) << 32)
            if sid in lost:
                print("entry", e, "tags", tags.tolist(), "sid", sid if sid != 0xFFFFFFFF else "tomb", "s", s_, "ct", ct)
    # tickets the waves gave up on (post-mortem words of their help slots' claim lines)
    hw = np.zeros(nw * 16, np.uint64)
    assert lib.kcdc_test_ws_copy(hw.ctypes.data_as(C.c_void_p), 8192 + ring * 128, nw * 128) == 0
    held = sorted(int(x) & 0xFFFFFFFF for x in hw.reshape(nw, 16)[:, 1] if int(x) >> 32 == 1)
    print("waves with a recorded ticket", len(held), "below tail", sum(1 for t in held if t < tail),
          "in [tail, head)", sum(1 for t in held if tail <= t < head), flush=True)
    hs = set(held)
    print("tickets in [tail, head) nobody holds:", [t for t in range(tail, head) if t not in hs][:40], flush=True)
    print("tickets below tail held:", [t for t in held if t < tail][:40], flush=True)

"""Tile-geometry sweep of the buzhash batch kernel (KCDC_TEST_LANE_CAP): for each name and lane
cap, a few launches of the config-2 workload, each checked bit-exact against the C oracle and
for the ring invariant (tickets - entries in {waves - 1, waves}: every reserved entry written,
DESIGN.md §2.1c), under a small spin cap so a lost stream ends the launch in ~1 s.  Prints one
JSON line per (name, cap).

  python tools/geometry_sweep.py [--names DYNAMIC-128K-BUZHASH,...] [--caps 256,512,...]
                                 [--streams 4096] [--mib 4] [--launches 3] [--help-mode 0]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from kopia_amd import _lib, batch  # noqa: E402
from oracle import coracle  # noqa: E402  (checker only)

ap = argparse.ArgumentParser()
ap.add_argument("--names", default="DYNAMIC-128K-BUZHASH,DYNAMIC-512K-BUZHASH,DYNAMIC-2M-BUZHASH,DYNAMIC-8M-BUZHASH")
ap.add_argument("--caps", default="256,512,1024,2048,4096")
ap.add_argument("--streams", type=int, default=4096)
ap.add_argument("--mib", type=int, default=4)
ap.add_argument("--launches", type=int, default=3)
ap.add_argument("--help-mode", type=int, default=0, help="KCDC_TEST_NO_HELP value: 0 policy, 1 off, 2 on")
args = ap.parse_args()

SEED, L, ns = 0x6B6F706961, args.mib << 20, args.streams
dev = torch.device("cuda:0")
lib = _lib.lib()
data = torch.empty(ns * L, dtype=torch.uint8, device=dev)
batch.fill_prng(data, L, ns, L, SEED, 0)
assert lib.kcdc_test_set(_lib.TEST_SPIN_CAP, 200000) == 0
assert lib.kcdc_test_set(_lib.TEST_NO_HELP, args.help_mode) == 0
bad_total = 0
try:
    for name in args.names.split(","):
        cuts, counts = coracle.split_prng_streams(name, SEED, np.arange(ns), L, nthreads=16)
        want = [cuts[i, :counts[i]].tolist() for i in range(ns)]
        b = batch.make_device_batch(name, [data.data_ptr() + i * L for i in range(ns)], [L] * ns, dev)
        for cap in (int(c) for c in args.caps.split(",")):
            assert lib.kcdc_test_set(_lib.TEST_LANE_CAP, cap) == 0
            rec = {"name": name, "lane_cap": cap, "launches": []}
            for _ in range(args.launches):
                t = time.time()
                batch.split_batch_device(name, b)
                torch.cuda.synchronize()
                dt = time.time() - t
                st = {k: int(lib.kcdc_test_queue_stat(v)) for k, v in (
                    ("tickets", _lib.STAT_TICKETS), ("entries", _lib.STAT_ENTRIES), ("waves", _lib.STAT_WAVES),
                    ("giveups", _lib.STAT_GIVEUPS), ("helps", _lib.STAT_HELPS))}
                cnt = b.counts.cpu().numpy()[:ns].astype(np.int64)
                got_all, base = b.cuts.cpu().numpy(), b.cut_base.cpu().numpy()
                bad = [i for i in range(ns) if cnt[i] < 0 or got_all[base[i]:base[i] + cnt[i]].tolist() != want[i]]
                gap = st["tickets"] - st["entries"]
                ok = not bad and st["giveups"] == 0 and st["waves"] - 1 <= gap <= st["waves"]
                bad_total += 0 if ok else 1
                rec["launches"].append({"s": round(dt, 4), "ok": ok, "bad_streams": len(bad), "ticket_gap": gap, **st})
            print(json.dumps(rec), flush=True)
finally:
    lib.kcdc_test_set(_lib.TEST_LANE_CAP, 0)
    lib.kcdc_test_set(_lib.TEST_SPIN_CAP, 0)
    lib.kcdc_test_set(_lib.TEST_NO_HELP, 0)
print(json.dumps({"failed_launches": bad_total}), flush=True)
sys.exit(1 if bad_total else 0)

"""Per-name table of the config-2-shaped batch (4096 x 4 MiB PRNG streams) from tools/kbench.py
logs with knob 6 (help: policy / 1 off / 2 on): kernel time, rolled bytes R (the reference
loop's reads, SURVEY.md §8d, from the C oracle's cut lists of the same streams) and R / t against
the 8 TB/s HBM peak.  Measurement infrastructure: runs on the CPU over logs the GPU wrote.
  python tools/name_sweep_table.py LOGDIR [--streams 4096] [--mib 4]"""
import argparse
import glob
import json
import os
import re
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import coracle  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("logdir")
ap.add_argument("--streams", type=int, default=4096)
ap.add_argument("--mib", type=int, default=4)
args = ap.parse_args()
SEED = 0x6B6F706961
rows = []
for p in sorted(glob.glob(os.path.join(args.logdir, "kbench___name_DYNAMIC_*_knob_6_1___knob_6_2___rounds_5_.log"))):
    name = re.search(r"name_(DYNAMIC_[0-9A-Z]+_[A-Z]+)", p).group(1).replace("_", "-")
    txt = open(p).read()
    res = json.loads(txt[txt.index("{"):txt.rindex("}") + 1])
    n = args.mib << 20
    cuts, counts = coracle.split_prng_streams(name, SEED, np.arange(args.streams), n, nthreads=8)
    R = sum(coracle.rolled_bytes(name, cuts[i, :counts[i]]) for i in range(args.streams))
    t = {k: v["median_ms"] for k, v in res.items()}
    rows.append((name, R, t["prod"], t["prod_knob6=1"], t["prod_knob6=2"]))
print("| name | R (GB) | policy (ms) | help off | help on | R / t (TB/s) | R frac of 8 TB/s |")
print("|---|---|---|---|---|---|---|")
for name, R, tp, toff, ton in rows:
    print(f"| {name} | {R / 1e9:.2f} | {tp:.3f} | {toff:.3f} | {ton:.3f} | {R / tp / 1e9:.2f} | {R / tp / 1e9 / 8:.3f} |")

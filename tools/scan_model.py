"""Byte accounting of the buzhash batch kernel's tile walk (split_batch_pipe_kernel), from cut
lists alone: what each chunk's region costs in DMA'd bytes against R, the rolled bytes the
reference loop reads.  Splits the kernel's traffic above R into
  - warm-up: the 64 bytes every lane segment of every tile reads before its segment,
  - alignment: the region's first tile starts at (s + min - 1) rounded down to 128,
  - overshoot: the rest of the region's last tile past the cut (a tile is scanned whole),
  - rounding: lane segments rounded up to 128 bytes in a region's short last tile.
No GPU: the cuts come from the C oracle on the config-2 PRNG streams (the bench's data).
Help (tiles scanned by waiting waves) is not modelled: helpers scan the same tiles, plus tiles
past the cut that the owner has not closed yet, so the model is a lower bound on traffic.

  python tools/scan_model.py [--name DYNAMIC-4M-BUZHASH] [--streams 512] [--mib 4]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import coracle  # noqa: E402  (test/measurement infrastructure only)

WAVE, SEED = 64, 0x6B6F706961
LANE_MAX = int(os.environ.get("KCDC_LANE_MAX", "2048"))  # kcdc_kernels.hip kLaneMax
TILE_DIV = int(os.environ.get("KCDC_TILE_DIV", "256"))  # kcdc_kernels.hip kTileDiv


def lane_cap(avg):
    cap = LANE_MAX
    while cap > 256 and cap * TILE_DIV > avg:
        cap >>= 1
    return cap


def account(name, cuts, n):
    """Per stream of n bytes with final cuts `cuts`: dict of byte counts."""
    mn = coracle.min_size(name)
    mx = coracle.cut_capacity  # (unused: max from params)
    _, avg = coracle.params(name)
    mxs = 2 * avg
    cap = lane_cap(avg)
    acc = dict(R=0, tiles=0, warm=0, align=0, over=0, rounding=0, chunks=0, tile_count=0)
    s = 0
    for e in cuts:
        e = int(e)
        L = e - s
        acc["R"] += L - max(min(mn - 1, L) - 64, 0)
        acc["chunks"] += 1
        if s + mn - 1 < n:  # a region is scanned
            lo = s + mn - 1
            hi = min(s + mxs - 1, n - 1)
            ct = lo & ~127
            acc["align"] += lo - ct
            f = e - 1  # the cut's position (a candidate, or the forced cut / the end)
            while True:
                rem = hi - ct + 1
                per = -(-rem // WAVE)
                per = (per + 127) & ~127
                Lh = min(per, cap)
                T = WAVE * Lh
                acc["tiles"] += T
                acc["warm"] += WAVE * 64
                acc["tile_count"] += 1
                end = ct + T - 1
                if f <= end or ct + T > hi:
                    if end > hi:
                        acc["rounding"] += end - hi
                    acc["over"] += max(min(end, hi) - f, 0)
                    break
                ct += T
        s = e
    return acc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--name", default="DYNAMIC-4M-BUZHASH")
    ap.add_argument("--streams", type=int, default=512)
    ap.add_argument("--mib", type=int, default=4)
    args = ap.parse_args()
    n = args.mib << 20
    cuts, counts = coracle.split_prng_streams(args.name, SEED, np.arange(args.streams), n, nthreads=8)
    tot = {}
    for i in range(args.streams):
        a = account(args.name, cuts[i, :counts[i]], n)
        for k, v in a.items():
            tot[k] = tot.get(k, 0) + v
    R = tot["R"]
    dma = tot["tiles"] + tot["warm"]
    out = {"name": args.name, "streams": args.streams, "stream_mib": args.mib, "lane_cap": lane_cap(coracle.params(args.name)[1]),
           "chunks": tot["chunks"], "tiles": tot["tile_count"], "R": R, "dma_bytes": dma, "dma_over_R": round(dma / R, 4),
           "warm_frac_of_R": round(tot["warm"] / R, 4), "align_frac_of_R": round(tot["align"] / R, 4),
           "overshoot_frac_of_R": round(tot["over"] / R, 4), "rounding_frac_of_R": round(tot["rounding"] / R, 4),
           "overshoot_bytes_per_chunk": round(tot["over"] / tot["chunks"]), "tiles_per_chunk": round(tot["tile_count"] / tot["chunks"], 2)}
    import json
    print(json.dumps(out))


if __name__ == "__main__":
    main()

"""Turn a rocprofv3 `--pmc FETCH_SIZE` pass into per-launch HBM read bytes.

usage: python tools/pmc_traffic.py <run_counter_collection.csv> <kernel> <config> [out.json]

The entry is keyed "<kernel>|<config>" (e.g. "kcdc::dev::split_batch_pipe_kernel<true>|config2"),
which is what bench.py looks up for that configuration's roofline.

FETCH_SIZE is reported in KiB and derives from TCC_EA0_RDREQ x 64 B; on gfx950 a
wide (16 B/lane) read is tallied at half its bytes (/opt/skills/guides/
MI355X_MICROARCH.md §HBM: "FETCH_SIZE reports exactly 1/2 of the bytes of a wide
coalesced streaming read ... double it").  Both our kernels read 16 B per lane
(buffer_load_dwordx4 / buffer_load_dwordx4 ... lds), so the correction factor 2
is applied.  The raw KiB value is kept next to the corrected bytes.
"""
import csv
import json
import statistics
import sys


def main():
    path, kernel, config = sys.argv[1], sys.argv[2], sys.argv[3]
    out = sys.argv[4] if len(sys.argv) > 4 else "profiles/pmc_traffic.json"
    key = f"{kernel}|{config}"
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE"]
    if not vals:
        sys.exit(f"no FETCH_SIZE rows for kernels matching {kernel!r}")
    kib = statistics.median(vals)
    try:
        d = json.load(open(out))
    except (OSError, ValueError):
        d = {}
    d[key] = {"fetch_size_kib_per_launch": kib, "correction": 2,
              "hbm_bytes_per_launch": int(kib * 1024 * 2), "launches": len(vals), "source": path}
    json.dump(d, open(out, "w"), indent=1)
    print(json.dumps(d[key]))


if __name__ == "__main__":
    main()

"""Median per-launch counter values of one kernel from rocprofv3 --pmc CSV outputs.
usage: python tools/pmc_summary.py KERNEL_SUBSTRING DIR [DIR ...]"""
import collections
import csv
import glob
import sys

sub, dirs = sys.argv[1], sys.argv[2:]
acc = collections.defaultdict(list)
for d in dirs:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if sub in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    v = sorted(v)
    print(f"{k:28s} n={len(v):3d} median={v[len(v) // 2]:.5g}")

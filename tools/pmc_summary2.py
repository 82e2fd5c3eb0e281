"""Per-kernel averages of rocprofv3 --pmc counter CSVs (one or more passes) for kernels
matching a substring: python tools/pmc_summary2.py SUBSTR run_counter_collection.csv..."""
import csv
import sys
from collections import defaultdict

sub = sys.argv[1]
acc = defaultdict(list)
for path in sys.argv[2:]:
    for r in csv.DictReader(open(path)):
        if sub in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(acc):
    v = acc[k]
    print(f"{k:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")

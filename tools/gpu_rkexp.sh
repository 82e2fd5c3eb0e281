#!/bin/bash
# Rabin-Karp experiments: A/B of variants (two-byte hop, 4 waves per workgroup) against the
# production one-byte kernel, then SQ counter passes (LDS latency and issue) on production.
set -u
OUT=gpurun_out/rkexp
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/kbench.py --name DYNAMIC-4M-RABINKARP --rounds 5 --reps 5 > $OUT/kbench_rk4m.log 2>&1 || { tail -30 $OUT/kbench_rk4m.log; exit 1; }
grep -A20 '^{' $OUT/kbench_rk4m.log | head -24
A="--splitter DYNAMIC-4M-RABINKARP --steps 5 --warmup 2 --no-hash --no-encrypt --no-cpu-baseline --no-host-inclusive"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $OUT/sq1 -o run --output-format csv -- python3 bench.py $A > $OUT/sq1.log 2>&1 || { tail -5 $OUT/sq1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $OUT/sq2 -o run --output-format csv -- python3 bench.py $A > $OUT/sq2.log 2>&1 || { tail -5 $OUT/sq2.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
for p in ("sq1", "sq2"):
    agg = collections.defaultdict(float); n = collections.Counter()
    for f in glob.glob(f"gpurun_out/rkexp/{p}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "split_batch_rk_kernel" in r["Kernel_Name"]:
                agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(p, {k: (v / max(n[k], 1)) for k, v in agg.items()})
PY

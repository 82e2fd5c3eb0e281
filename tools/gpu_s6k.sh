#!/bin/bash
# round 6 (late): 4 KiB buzhash lanes when streams < waves -- shapes x names, same-process A/B
set -o pipefail
O=gpurun_out/s6k; mkdir -p $O
for shape in "2048 8" "1024 16" "512 32" "256 64" "64 256"; do
  set -- $shape
  for nm in DYNAMIC-4M-BUZHASH DYNAMIC-1M-BUZHASH DYNAMIC-2M-BUZHASH DYNAMIC-8M-BUZHASH; do
    timeout -k 10 200 python3 -u tools/kbench.py --name $nm --streams $1 --mib $2 --glob 'none' --knob 8=4096 --rounds 5 > $O/kb_${nm}_$1_$2.log 2>> $O/err.log || exit 1
    python3 - $O/kb_${nm}_$1_$2.log $nm $1 $2 <<'PY'
import json,sys
t=open(sys.argv[1]).read(); bad=[l for l in t.splitlines() if 'mismatches' in l and not l.endswith(' 0')]
j=json.loads(t[t.index('{'):t.rindex('}')+1])
print(sys.argv[2], sys.argv[3], sys.argv[4], 'prod %.3f'%j['prod']['median_ms'], 'cap4096 %.3f'%j['prod_knob8=4096']['median_ms'], 'BAD' if bad else 'ok')
PY
  done
done

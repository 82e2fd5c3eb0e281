#!/bin/bash
# round 6 (late): help windows (knob 9 = tiles per published window) vs whole-region publish
set -o pipefail
O=gpurun_out/s6n; mkdir -p $O
for shape in "1024 16" "2048 8" "4096 4" "512 32"; do
  set -- $shape
  for nm in DYNAMIC-4M-BUZHASH DYNAMIC-1M-BUZHASH; do
    timeout -k 10 200 python3 -u tools/kbench.py --name $nm --streams $1 --mib $2 --glob 'none' --knob 9=4 --knob 9=8 --knob 9=16 --knob 9=32 --rounds 5 > $O/kb_${nm}_$1_$2.log 2>> $O/err.log || exit 1
    python3 - $O/kb_${nm}_$1_$2.log $nm $1 $2 <<'PY'
import json,sys
t=open(sys.argv[1]).read(); bad=[l for l in t.splitlines() if 'mismatches' in l and not l.endswith(' 0')]
j=json.loads(t[t.index('{'):t.rindex('}')+1])
print(sys.argv[2], sys.argv[3], sys.argv[4], ' '.join('%s %.3f'%(k.replace('prod_knob9=','w'),v['median_ms']) for k,v in j.items()), 'BAD' if bad else 'ok')
PY
  done
done

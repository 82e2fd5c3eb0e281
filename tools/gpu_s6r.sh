#!/bin/bash
# round 6 (late): writers on the final build (their launches now take the few-streams policies),
# and the buzhash help-window width at 16-32 waves per stream
set -o pipefail
O=gpurun_out/s6r; mkdir -p $O
for h in none BLAKE2B-256-128; do
  timeout -k 10 300 ./build/writer_bench 32 512 64 DYNAMIC-4M-BUZHASH 256 3 $h > $O/writer_32_512_$h.json 2> $O/writer_32_512_$h.err || exit 1
  head -c 400 $O/writer_32_512_$h.json; echo
done
for shape in "128 128" "64 256"; do
  set -- $shape
  nm=DYNAMIC-4M-BUZHASH
  timeout -k 10 200 python3 -u tools/kbench.py --name $nm --streams $1 --mib $2 --glob 'none' --knob 9=6 --knob 9=8 --knob 9=12 --rounds 3 --reps 2 > $O/kb_${nm}_$1_$2.log 2>> $O/err.log || exit 1
  python3 - $O/kb_${nm}_$1_$2.log $nm $1 $2 <<'PY'
import json,sys
t=open(sys.argv[1]).read(); bad=[l for l in t.splitlines() if 'mismatches' in l and not l.endswith(' 0')]
j=json.loads(t[t.index('{'):t.rindex('}')+1])
print(sys.argv[2], sys.argv[3], sys.argv[4], ' '.join('%s %.3f'%(k.replace('prod_knob9=','w'),v['median_ms']) for k,v in j.items()), 'BAD' if bad else 'ok')
PY
done

#!/bin/bash
# round 6 (late): the scaled buzhash window width (policy) vs W = 4, then the help/parity tests
set -o pipefail
O=gpurun_out/s6s; mkdir -p $O
for shape in "128 128" "64 256" "256 64"; do
  set -- $shape
  nm=DYNAMIC-4M-BUZHASH
  timeout -k 10 200 python3 -u tools/kbench.py --name $nm --streams $1 --mib $2 --glob 'none' --knob 9=4 --rounds 3 --reps 2 > $O/kb_${nm}_$1_$2.log 2>> $O/err.log || exit 1
  python3 - $O/kb_${nm}_$1_$2.log $nm $1 $2 <<'PY'
import json,sys
t=open(sys.argv[1]).read(); bad=[l for l in t.splitlines() if 'mismatches' in l and not l.endswith(' 0')]
j=json.loads(t[t.index('{'):t.rindex('}')+1])
print(sys.argv[2], sys.argv[3], sys.argv[4], ' '.join('%s %.3f'%(k.replace('prod_knob9=','w'),v['median_ms']) for k,v in j.items()), 'BAD' if bad else 'ok')
PY
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_help.py tests/test_gpu_writer.py tests/test_gpu_queue.py tests/test_gpu_files.py tests/test_gpu_multirank.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; exit $rc

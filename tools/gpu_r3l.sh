#!/bin/bash
# Round 3 final: full GPU suite + smoke, the driver's default bench line, configs 3/4/5 lines.
set -u
OUT=gpurun_out/r3l
mkdir -p $OUT
export TMPDIR=/tmp
echo "== suite $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/suite.log 2>&1
rc=$?; tail -2 $OUT/suite.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke $(date +%T)"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
for c in default c4 c3 c5; do
  case $c in
    default) A="";;
    c4) A="--config 4 --no-hash --no-encrypt --no-host-inclusive --no-cpu-baseline";;
    c3) A="--config 3 --no-cpu-baseline";;
    c5) A="--config 5 --no-cpu-baseline";;
  esac
  echo "== bench $c $(date +%T)"
  timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 $A > $OUT/bench_$c.json 2> $OUT/bench_$c.err || exit $?
  python -c "import json;d=json.loads(open('$OUT/bench_$c.json').read().strip().splitlines()[-1]);r=d.get('roofline',{});print('$c',d['value'],d['ms_per_step'],r.get('kernel_ms'),r.get('hbm_frac_measured'))"
done

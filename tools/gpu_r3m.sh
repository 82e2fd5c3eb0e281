#!/bin/bash
# Round 3 closing run: full GPU suite + smoke on the final build, the driver's default bench line,
# then the default command under rocprofv3 (kernel trace + stats, FETCH_SIZE pass).
set -u
OUT=gpurun_out/r3m
mkdir -p $OUT
export TMPDIR=/tmp
echo "== suite $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/suite.log 2>&1
rc=$?; tail -2 $OUT/suite.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke $(date +%T)"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
echo "== bench $(date +%T)"
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_default.json 2> $OUT/bench_default.err || exit $?
python -c "import json;d=json.loads(open('$OUT/bench_default.json').read().strip().splitlines()[-1]);r=d['roofline'];print(d['value'],d['ms_per_step'],r['kernel_ms'],r['frac'],r['hbm_frac_measured'])"
bash tools/profile_configs.sh $OUT default "--gpus 1 --steps 20 --warmup 5" || exit 1

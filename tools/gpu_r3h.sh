#!/bin/bash
# Round 3 (re-entry): RK lane-length A/B, the full GPU suite + smoke on the RK_LMUL=2 build,
# the driver's default bench line and the Rabin-Karp config-2 bench line.
set -u
OUT=gpurun_out/r3h
mkdir -p $OUT
export TMPDIR=/tmp
echo "== kbench RK $(date +%T)"
timeout -k 10 150 python -u tools/kbench.py --name DYNAMIC-4M-RABINKARP --rounds 6 --reps 4 > $OUT/k4m.log 2>&1 || exit $?
timeout -k 10 150 python -u tools/kbench.py --name DYNAMIC-128K-RABINKARP --rounds 6 --reps 4 > $OUT/k128k.log 2>&1 || exit $?
grep -E "parity|median" $OUT/k4m.log $OUT/k128k.log
echo "== suite $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/suite.log 2>&1
rc=$?; tail -3 $OUT/suite.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke $(date +%T)"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
echo "== bench $(date +%T)"
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_default.json 2> $OUT/bench_default.err || exit $?
python -c "import json;d=json.load(open('$OUT/bench_default.json'));print(d['value'],d['ms_per_step'],d['warmup_steps_run'],d['roofline']['kernel_ms'],d['roofline']['hbm_frac_measured'])"
echo "== bench RK $(date +%T)"
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --splitter DYNAMIC-4M-RABINKARP --no-hash --no-encrypt --no-host-inclusive > $OUT/bench_rk.json 2> $OUT/bench_rk.err || exit $?
python -c "import json;d=json.load(open('$OUT/bench_rk.json'));r=d['roofline'];print(d['value'],r['kernel_ms'],r['hbm_frac_measured'],r.get('valu_floor_ms'),r.get('valu_busy'))"

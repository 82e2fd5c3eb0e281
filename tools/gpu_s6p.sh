#!/bin/bash
# round 6 (final build): the whole GPU suite + smoke + default bench + kernel stats
set -o pipefail
O=gpurun_out/s6p; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1
rc=$?; tail -3 $O/suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/default_trace -o run --output-format csv -- python3 bench.py > $O/bench_default_prof.json 2> $O/bench_prof.err || exit $?
timeout -k 10 200 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
f=$(find $O/default_trace -name '*kernel_stats.csv' | head -1); cp "$f" $O/default_kernel_stats.csv
head -3 $O/default_kernel_stats.csv | cut -c1-200
python3 -c "
import json; d=json.load(open('$O/bench_default.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['frac'], r['hbm_frac_measured'], r['kernel_ms'])"

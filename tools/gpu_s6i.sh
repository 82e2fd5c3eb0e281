#!/bin/bash
# round 6 (late): the whole GPU suite + smoke + default bench on the HEAD build
set -o pipefail
O=gpurun_out/s6i; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1
rc=$?; tail -3 $O/suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 200 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
cat $O/bench_default.json | head -c 600

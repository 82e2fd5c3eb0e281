#!/bin/bash
# Round 3 (re-entry): full GPU suite + smoke on the rebuilt tree.
set -u
OUT=gpurun_out/r3e
mkdir -p $OUT
export TMPDIR=/tmp
echo "== suite $(date +%T)"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/suite.log 2>&1
rc=$?; tail -5 $OUT/suite.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke $(date +%T)"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -2 $OUT/smoke.log

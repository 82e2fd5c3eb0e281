# round 6: the whole GPU suite + smoke on the HEAD build
set -o pipefail
O=gpurun_out/s6h; mkdir -p $O
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1
rc=$?; tail -3 $O/suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log

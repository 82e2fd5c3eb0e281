#!/bin/bash
# Round 3 (re-entry): the GPU test files after the stream-ordered workspace fix, smoke, then gpu_r3f.sh.
set -u
OUT=gpurun_out/r3g
mkdir -p $OUT
export TMPDIR=/tmp
echo "== tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_queue.py tests/test_gpu_server.py tests/test_gpu_writer.py -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke $(date +%T)"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -2 $OUT/smoke.log
bash tools/gpu_r3f.sh

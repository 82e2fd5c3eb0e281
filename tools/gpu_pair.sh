#!/bin/bash
# Paired buzhash frame: parity on every buzhash path, then an A/B against the previous frame.
set -u
OUT=gpurun_out/pair
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_long.py tests/test_gpu_files.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
tail -2 $OUT/parity.log
timeout -k 10 300 python -u tools/kbench.py --rounds 5 --reps 5 > $OUT/kb4m.log 2>&1 || { tail -20 $OUT/kb4m.log; exit 1; }
grep -A16 '^{' $OUT/kb4m.log
timeout -k 10 300 python -u tools/kbench.py --name DYNAMIC-128K-BUZHASH --rounds 3 --reps 5 > $OUT/kb128k.log 2>&1 || { tail -20 $OUT/kb128k.log; exit 1; }
grep -A16 '^{' $OUT/kb128k.log

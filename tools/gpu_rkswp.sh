#!/bin/bash
set -u
OUT=gpurun_out/rkswp
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "RABINKARP or rabinkarp or kat or KAT" > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
tail -2 $OUT/parity.log
timeout -k 10 300 python -u tools/kbench.py --name DYNAMIC-4M-RABINKARP --rounds 5 --reps 5 > $OUT/kb4m.log 2>&1 || { tail -20 $OUT/kb4m.log; exit 1; }
grep -A16 '^{' $OUT/kb4m.log
timeout -k 10 300 python -u tools/kbench.py --name DYNAMIC-128K-RABINKARP --rounds 3 --reps 5 > $OUT/kb128k.log 2>&1 || { tail -20 $OUT/kb128k.log; exit 1; }
grep -A16 '^{' $OUT/kb128k.log

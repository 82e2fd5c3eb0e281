#!/bin/bash
# 4-chain Rabin-Karp variant: parity vs the production library on config 2 (all 4096 streams,
# 4M and 128K), A/B timing, then the RK parity tests on the variant library.
set -u
OUT=gpurun_out/rk4
mkdir -p $OUT
export TMPDIR=/tmp
echo "== kbench 4M $(date +%T)"
timeout -k 10 240 python -u tools/kbench.py --name DYNAMIC-4M-RABINKARP --rounds 5 --reps 4 > $OUT/kbench_4m.log 2>&1 || exit $?
grep -E "parity|median" $OUT/kbench_4m.log
echo "== kbench 128K $(date +%T)"
timeout -k 10 240 python -u tools/kbench.py --name DYNAMIC-128K-RABINKARP --rounds 5 --reps 4 > $OUT/kbench_128k.log 2>&1 || exit $?
grep -E "parity|median" $OUT/kbench_128k.log
echo "== tests on rk4 $(date +%T)"
KCDC_LIB=$PWD/build/variants/libkcdc_rk4.so KCDC_ALLOW_VARIANT_LIB=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_files.py -x -q -k "RABINKARP or rabin or RK or rk or kat or files" --timeout 200 --timeout-method thread > $OUT/tests_rk4.log 2>&1
rc=$?; tail -3 $OUT/tests_rk4.log; exit $rc

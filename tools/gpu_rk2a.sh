set -u
OUT=gpurun_out/rk2a
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_long.py -x -v --timeout 200 --timeout-method thread > $OUT/parity.log 2>&1 || { tail -40 $OUT/parity.log; exit 1; }
tail -3 $OUT/parity.log
timeout -k 10 300 python -u tools/kbench.py --name DYNAMIC-4M-RABINKARP --rounds 5 --reps 5 > $OUT/kbench_rk4m.log 2>&1 || { tail -30 $OUT/kbench_rk4m.log; exit 1; }
cat $OUT/kbench_rk4m.log
timeout -k 10 300 python -u tools/kbench.py --name DYNAMIC-128K-RABINKARP --rounds 3 --reps 5 > $OUT/kbench_rk128k.log 2>&1 || { tail -30 $OUT/kbench_rk128k.log; exit 1; }
cat $OUT/kbench_rk128k.log

set -o pipefail
O=gpurun_out/r6c; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -2 $O/parity.log
timeout -k 10 300 python -u tools/kbench.py --name DYNAMIC-4M-RABINKARP --rounds 7 > $O/kb_rk4m.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/kbench.py --name DYNAMIC-128K-RABINKARP --rounds 5 > $O/kb_rk128k.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/kbench.py --name DYNAMIC-1M-RABINKARP --rounds 5 > $O/kb_rk1m.log 2>&1 || exit 1
echo ok

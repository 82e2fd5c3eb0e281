# round 6: tail tiles (KCDC_TAIL_SMALL) A/B and the parity/help tests on the new kernels
set -o pipefail
O=gpurun_out/s6f; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_help.py tests/test_gpu_queue.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for nm in DYNAMIC-4M-BUZHASH DYNAMIC-2M-BUZHASH DYNAMIC-1M-BUZHASH DYNAMIC-4M-RABINKARP DYNAMIC-1M-RABINKARP DYNAMIC-128K-RABINKARP; do
  timeout -k 10 300 python -u tools/kbench.py --name $nm --rounds 7 > $O/kb_$nm.log 2>&1 || exit 1
done
echo ok

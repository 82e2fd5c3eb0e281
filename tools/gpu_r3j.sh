#!/bin/bash
# Slot affinity: the queue/concurrency/parity tests, then the default command's kernel trace (gaps).
set -u
OUT=gpurun_out/r3j
mkdir -p $OUT
export TMPDIR=/tmp
echo "== tests $(date +%T)"
timeout -k 10 700 python -u -m pytest tests/test_gpu_queue.py tests/test_gpu_concurrency.py tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_writer.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
echo "== bench $(date +%T)"
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-hash --no-encrypt --no-host-inclusive --no-cpu-baseline > $OUT/bench.json 2>&1 || exit $?
python -c "import json;d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['roofline']['hbm_frac_measured'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-hash --no-encrypt --no-host-inclusive --no-cpu-baseline > $OUT/trace.json 2> $OUT/trace.err || exit $?
echo done

#!/bin/bash
# deflate: the compression tests, the plan trace, the bench
set -o pipefail
mkdir -p gpurun_out/z8
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_compress.py > gpurun_out/z8/t.log 2>&1
rc=$?; tail -2 gpurun_out/z8/t.log; [ $rc -eq 0 ] || exit $rc
KCDC_LIB=build/libkcdc_trace.so KCDC_ALLOW_VARIANT_LIB=1 timeout -k 10 300 python3 -u tools/ztrace.py 64 deflate-default > gpurun_out/z8/deflate.json 2> gpurun_out/z8/err.log
rc=$?; cat gpurun_out/z8/deflate.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/compress_bench.py --gib 4 --name deflate-default --iters 3 > gpurun_out/z8/bench_deflate.log 2>&1
rc=$?; grep -h '"mixed"\|"random"\|"pattern"' gpurun_out/z8/bench_deflate.log | head -3 | cut -c1-160; exit $rc

#!/bin/bash
# zstd with sequence-balanced blocks: the zstd tests, the phase trace, the bench
set -o pipefail
mkdir -p gpurun_out/z12
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_compress.py -k "zstd" > gpurun_out/z12/t.log 2>&1
rc=$?; tail -3 gpurun_out/z12/t.log; [ $rc -eq 0 ] || exit $rc
KCDC_LIB=build/libkcdc_trace.so KCDC_ALLOW_VARIANT_LIB=1 timeout -k 10 300 python3 -u tools/ztrace.py 64 > gpurun_out/z12/zstd.json 2> gpurun_out/z12/err.log
rc=$?; head -c 1500 gpurun_out/z12/zstd.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/compress_bench.py --gib 4 --name zstd --iters 3 > gpurun_out/z12/bench_zstd.log 2>&1
rc=$?; grep -h '"mixed"\|"random"\|"pattern"' gpurun_out/z12/bench_zstd.log | head -3 | cut -c1-200; exit $rc

#!/bin/bash
# zstd: tests, phase trace, bench
set -o pipefail
mkdir -p gpurun_out/z4
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_compress.py -k "zstd or mixed_ratio" > gpurun_out/z4/t.log 2>&1
rc=$?; tail -2 gpurun_out/z4/t.log; [ $rc -eq 0 ] || exit $rc
KCDC_LIB=build/libkcdc_trace.so KCDC_ALLOW_VARIANT_LIB=1 timeout -k 10 300 python3 -u tools/ztrace.py 64 > gpurun_out/z4/trace.json 2> gpurun_out/z4/err.log
rc=$?; python3 -c "import json;d=json.load(open('gpurun_out/z4/trace.json'));print({k:(v['mean'] if isinstance(v,dict) else v) for k,v in d.items()})"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/compress_bench.py --gib 4 --name zstd --iters 3 > gpurun_out/z4/bench_zstd.log 2>&1
rc=$?; grep -h '"mixed"\|"random"\|"pattern"' gpurun_out/z4/bench_zstd.log | head -3 | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/compress_bench.py --gib 4 --name zstd-better-compression --only mixed --iters 3 > gpurun_out/z4/bench_zbetter.log 2>&1
rc=$?; grep -h '"mixed"' gpurun_out/z4/bench_zbetter.log | head -1 | cut -c1-200; exit $rc

#!/bin/bash
# compression tests, deflate + zstd traces, both benches
set -o pipefail
mkdir -p gpurun_out/z10
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_compress.py > gpurun_out/z10/t.log 2>&1
rc=$?; tail -2 gpurun_out/z10/t.log; [ $rc -eq 0 ] || exit $rc
KCDC_LIB=build/libkcdc_trace.so KCDC_ALLOW_VARIANT_LIB=1 timeout -k 10 300 python3 -u tools/ztrace.py 64 deflate-default > gpurun_out/z10/deflate.json 2> gpurun_out/z10/err.log || exit $?
KCDC_LIB=build/libkcdc_trace.so KCDC_ALLOW_VARIANT_LIB=1 timeout -k 10 300 python3 -u tools/ztrace.py 64 zstd > gpurun_out/z10/zstd.json 2>> gpurun_out/z10/err.log || exit $?
python3 -c "
import json
for f in ['deflate','zstd']:
    d=json.load(open('gpurun_out/z10/'+f+'.json')); print(f, {k:(v['mean'] if isinstance(v,dict) and 'mean' in v else v) for k,v in d.items() if k not in ('bytes_per_span',)})"
for n in deflate-default zstd; do
timeout -k 10 300 python -u tools/compress_bench.py --gib 4 --name $n --iters 3 > gpurun_out/z10/bench_$n.log 2>&1 || exit $?
grep -h '"mixed"' gpurun_out/z10/bench_$n.log | head -1 | cut -c1-120
done

#!/bin/bash
# zstd span-level blocks: the compression tests that touch zstd, then the zstd throughput/ratio bench
set -o pipefail
mkdir -p gpurun_out/z1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_compress.py -k "zstd or mixed_ratio" > gpurun_out/z1/t.log 2>&1
rc=$?; tail -3 gpurun_out/z1/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/compress_bench.py --gib 4 --name zstd --iters 3 > gpurun_out/z1/bench_zstd.log 2>&1
rc=$?; tail -2 gpurun_out/z1/bench_zstd.log | cut -c1-700; exit $rc

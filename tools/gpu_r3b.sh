#!/bin/bash
# Round 3, second GPU call: batching writers, compressors (S2/zstd new), multi-rank, crypt side stream.
set -u
OUT=gpurun_out/r3b
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_writer.py tests/test_gpu_crypt.py -x -v --timeout 200 --timeout-method thread > $OUT/writer_crypt.log 2>&1 || { tail -40 $OUT/writer_crypt.log; exit 1; }
tail -2 $OUT/writer_crypt.log
for w in 64 16 1; do
  timeout -k 10 200 build/writer_bench $w $((4096 / w > 256 ? 256 : 4096 / w)) 64 DYNAMIC-4M-BUZHASH 256 3 >> $OUT/writer_bench.jsonl 2> $OUT/writer_bench.err || { cat $OUT/writer_bench.err; exit 1; }
done
cat $OUT/writer_bench.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_compress.py tests/test_gpu_multirank.py -x -v --timeout 200 --timeout-method thread > $OUT/compress_multirank.log 2>&1 || { tail -40 $OUT/compress_multirank.log; exit 1; }
tail -2 $OUT/compress_multirank.log
for n in deflate-default deflate-best-compression s2-default zstd zstd-best-compression; do
  timeout -k 10 200 python -u tools/compress_bench.py --gib 4 --name $n --iters 3 >> $OUT/compress_bench.log 2>&1 || { tail -20 $OUT/compress_bench.log; exit 1; }
done
tail -40 $OUT/compress_bench.log

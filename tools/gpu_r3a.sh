#!/bin/bash
# Round 3, first GPU call: Rabin-Karp two-byte hop parity + A/B timing, batching writers, crypt side stream.
set -u
OUT=gpurun_out/r3a
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_long.py -x -v --timeout 200 --timeout-method thread > $OUT/parity.log 2>&1 || { tail -40 $OUT/parity.log; exit 1; }
tail -2 $OUT/parity.log
timeout -k 10 300 python -u tools/kbench.py --name DYNAMIC-4M-RABINKARP --rounds 5 --reps 5 > $OUT/kbench_rk4m.log 2>&1 || { tail -30 $OUT/kbench_rk4m.log; exit 1; }
grep -A12 '^{' $OUT/kbench_rk4m.log | head -14
timeout -k 10 300 python -u tools/kbench.py --name DYNAMIC-128K-RABINKARP --rounds 3 --reps 5 > $OUT/kbench_rk128k.log 2>&1 || { tail -30 $OUT/kbench_rk128k.log; exit 1; }
grep -A12 '^{' $OUT/kbench_rk128k.log | head -14
timeout -k 10 400 python -u -m pytest tests/test_gpu_writer.py tests/test_gpu_crypt.py -x -v --timeout 200 --timeout-method thread > $OUT/writer_crypt.log 2>&1 || { tail -40 $OUT/writer_crypt.log; exit 1; }
tail -2 $OUT/writer_crypt.log
for w in 64 16 1; do
  timeout -k 10 200 build/writer_bench $w $((4096 / w > 256 ? 256 : 4096 / w)) 64 DYNAMIC-4M-BUZHASH 256 3 >> $OUT/writer_bench.jsonl 2> $OUT/writer_bench.err || { cat $OUT/writer_bench.err; exit 1; }
done
cat $OUT/writer_bench.jsonl
timeout -k 10 500 python -u -m pytest tests/test_gpu_compress.py tests/test_gpu_multirank.py -x -v --timeout 200 --timeout-method thread > $OUT/compress_multirank.log 2>&1 || { tail -40 $OUT/compress_multirank.log; exit 1; }
tail -2 $OUT/compress_multirank.log
for n in deflate-default deflate-best-compression s2-default; do
  timeout -k 10 200 python -u tools/compress_bench.py --gib 4 --name $n --iters 3 >> $OUT/compress_bench.log 2>&1 || { tail -20 $OUT/compress_bench.log; exit 1; }
done
tail -30 $OUT/compress_bench.log

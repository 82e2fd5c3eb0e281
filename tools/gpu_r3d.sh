#!/bin/bash
# Round 3: hashes (HMAC-SHA2/SHA3, BLAKE3 new), batching writers (single-writer stall fixed),
# compressors (S2/zstd new), multi-rank.  Every step logs to gpurun_out/r3d and prints progress.
set -u
OUT=gpurun_out/r3d
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  echo "== $n $(date +%T)"
  timeout -k 10 $t "$@" > $OUT/$n.log 2>&1
  local rc=$?
  tail -3 $OUT/$n.log
  return $rc
}
run hash 600 python -u -m pytest tests/test_gpu_hash.py -x -v --timeout 300 --timeout-method thread || exit 1
run writer 400 python -u -m pytest tests/test_gpu_writer.py -x -v --timeout 200 --timeout-method thread || exit 1
for w in 64 16 4 1; do
  run wb$w 200 build/writer_bench $w $((4096 / w > 256 ? 256 : 4096 / w)) 64 DYNAMIC-4M-BUZHASH 256 3 || exit 1
done
run compress 600 python -u -m pytest tests/test_gpu_compress.py tests/test_gpu_multirank.py -x -v --timeout 200 --timeout-method thread || exit 1
for n in deflate-default deflate-best-compression s2-default zstd zstd-best-compression; do
  run cb_$n 200 python -u tools/compress_bench.py --gib 4 --name $n --iters 3 || exit 1
done
run bench 600 python -u bench.py --steps 20 --warmup 3 || exit 1

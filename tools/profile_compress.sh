#!/bin/bash
# rocprofv3 kernel trace + stats over tools/compress_bench.py (run from the repo root via gpurun)
# for one compressor name: per-kernel times of span_count/scan, deflate_spans, span_pos,
# deflate_copy, crc_spans (gzip family) and deflate_frame.
set -u
NAME=${1:-gzip}
OUT=${2:-gpurun_out/cmprof}
mkdir -p $OUT
export TMPDIR=/tmp
R=$PWD
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$OUT/$NAME -o run --output-format csv -- python3 $R/tools/compress_bench.py --name $NAME --iters 2 > $R/$OUT/$NAME.log 2>&1 || exit 1

#!/bin/bash
# Per-config rocprofv3 passes on the GPU box (run from the repo root via gpurun):
#   <tag>_trace : --kernel-trace --stats  (per-kernel durations)
#   <tag>_fetch : --pmc FETCH_SIZE        (HBM read bytes per launch; own pass)
# usage: tools/profile_configs.sh OUTDIR TAG "bench args" [TAG "bench args" ...]
set -u
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
while [ $# -ge 2 ]; do
  TAG=$1; ARGS=$2; shift 2
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_trace" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/${TAG}_trace.json" 2> "$OUT/${TAG}_trace.err" || exit $?
  timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE -d "$OUT/${TAG}_fetch" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/${TAG}_fetch.json" 2> "$OUT/${TAG}_fetch.err" || exit $?
  echo "profiled $TAG"
done
echo done

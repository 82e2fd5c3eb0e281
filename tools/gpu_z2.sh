#!/bin/bash
# per-kernel times of the zstd compressor on the mixed data
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/z2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/z2/prof -o z -- python3 tools/compress_bench.py --gib 1 --name zstd --iters 3 --only mixed > gpurun_out/z2/b.log 2>&1
rc=$?; tail -1 gpurun_out/z2/b.log | cut -c1-300; find gpurun_out/z2/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cut -d, -f1-8 {} | head -12; exit $rc

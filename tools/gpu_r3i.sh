#!/bin/bash
# Round 3 final profiles: the driver's default command and the Rabin-Karp config-2 command under
# rocprofv3 (kernel trace + stats, then a FETCH_SIZE pass of its own), on the final build.
set -u
OUT=gpurun_out/r3i
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/profile_configs.sh $OUT default "--gpus 1 --steps 20 --warmup 5" \
  c2rk "--gpus 1 --steps 20 --warmup 5 --splitter DYNAMIC-4M-RABINKARP --no-hash --no-encrypt --no-host-inclusive --no-cpu-baseline" || exit 1

#!/bin/bash
set -u
OUT=gpurun_out/r3def
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/profile_configs.sh $OUT default "--steps 20 --warmup 3" || exit 1
tail -1 $OUT/default_trace.json

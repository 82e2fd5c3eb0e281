#!/bin/bash
# Round 3 profiles: kernel traces + FETCH_SIZE passes (default bench, config-2 RK, config-3 RK),
# and the content-hash timings of every registered name.
set -u
OUT=gpurun_out/r3prof
mkdir -p $OUT
export TMPDIR=/tmp
echo "== hash $(date +%T)"
timeout -k 10 300 python -u tools/hash_bench.py > $OUT/hash_bench.json 2> $OUT/hash_bench.err || { tail -5 $OUT/hash_bench.err; exit 1; }
cat $OUT/hash_bench.json
echo "== profiles $(date +%T)"
bash tools/profile_configs.sh $OUT default "--steps 20 --warmup 3" \
  c2rk "--splitter DYNAMIC-4M-RABINKARP --steps 20 --warmup 3 --no-hash --no-encrypt --no-cpu-baseline --no-host-inclusive" \
  c3rk "--config 3 --splitter DYNAMIC-4M-RABINKARP --steps 3 --warmup 1 --no-cpu-baseline" || exit 1

#!/bin/bash
# Batching writers: throughput and where a round's time goes, across writer counts (16 GiB per pass).
set -u
OUT=gpurun_out/wb
mkdir -p $OUT
for cfg in "8 2048 64 256" "16 1024 64 256" "24 683 64 256" "32 512 64 256" "48 341 64 256" "64 256 64 256" "64 256 64 512" "16 1024 1000 256"; do
  set -- $cfg
  echo "== $cfg $(date +%T)"
  timeout -k 10 150 build/writer_bench $1 $2 $3 DYNAMIC-4M-BUZHASH $4 3 | tee -a $OUT/wb.jsonl || exit 1
done

#!/bin/bash
# round 6 (late): 1024 x 16 MiB and 2048 x 8 MiB lines on the 4 KiB-lane policy, with kernel
# stats and a FETCH_SIZE pass each, then the plain bench lines carrying the measured traffic
set -o pipefail
O=gpurun_out/s6m; mkdir -p $O
export TMPDIR=/tmp
A="--steps 20 --no-hash --pipeline-slots 0 --no-encrypt --no-cpu-baseline --no-host-inclusive"
bash tools/profile_configs.sh $O l16 "--streams 1024 --stream-mib 16 $A" l8 "--streams 2048 --stream-mib 8 $A" || exit 1
cp profiles/pmc_traffic.json $O/pmc_traffic.json
for t in "l16 config2-1024x16MiB" "l8 config2-2048x8MiB"; do
  set -- $t
  f=$(find $O/${1}_fetch -name '*counter_collection.csv' | head -1)
  python3 tools/pmc_traffic.py "$f" "kcdc::dev::split_batch_pipe_kernel<true>" $2 $O/pmc_traffic.json || exit 1
  f2=$(find $O/${1}_trace -name '*kernel_stats.csv' | head -1); cp "$f2" $O/${1}_kernel_stats.csv
  cp "$f" $O/${1}_fetch_counter_collection.csv
done
cp $O/pmc_traffic.json profiles/pmc_traffic.json
timeout -k 10 300 python3 -u bench.py --streams 1024 --stream-mib 16 > $O/bench_1024x16MiB.json 2> $O/bench_l16.err || exit 1
timeout -k 10 300 python3 -u bench.py --streams 2048 --stream-mib 8 > $O/bench_2048x8MiB.json 2> $O/bench_l8.err || exit 1
python3 -c "
import json
for f in ('bench_1024x16MiB','bench_2048x8MiB'):
    d=json.load(open('$O/'+f+'.json')); r=d['roofline']; print(f, d['value'], d['ms_per_step'], r['frac'], r['hbm_frac_measured'], r['kernel_ms'])"

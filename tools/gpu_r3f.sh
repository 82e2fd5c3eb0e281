#!/bin/bash
# Round 3 (re-entry): the driver's default bench command twice, a long-warmup run (DVFS check),
# then the default command under rocprofv3 (kernel trace + its own FETCH_SIZE pass).
set -u
OUT=gpurun_out/r3f
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  echo "== bench$i $(date +%T)"
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_default_$i.json 2> $OUT/bench_default_$i.err || exit $?
  python -c "import json;d=json.load(open('$OUT/bench_default_$i.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['roofline']['hbm_frac_measured'])"
done
echo "== bench warm60 $(date +%T)"
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 60 --no-hash --no-encrypt --no-host-inclusive --no-cpu-baseline > $OUT/bench_warm60.json 2> $OUT/bench_warm60.err || exit $?
python -c "import json;d=json.load(open('$OUT/bench_warm60.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel_ms'])"
echo "== kbench $(date +%T)"
timeout -k 10 200 python -u tools/kbench.py --glob 'build/variants/none*.so' > $OUT/kbench.log 2>&1 || exit $?
tail -8 $OUT/kbench.log
echo "== rocprof $(date +%T)"
bash tools/profile_configs.sh $OUT default "--gpus 1 --steps 20 --warmup 5" || exit 1

#!/bin/bash
# Launch gaps: kernel traces of kbench (events only around 5 launches) and of the bench (an
# event pair per launch), with the queue slots' no-system-fence event.
set -u
OUT=gpurun_out/r3k
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/kb -o run --output-format csv -- python3 tools/kbench.py --glob 'none' --rounds 4 --reps 5 > $OUT/kb.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/bn -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-hash --no-encrypt --no-host-inclusive --no-cpu-baseline > $OUT/bn.json 2> $OUT/bn.err || exit $?
echo done
